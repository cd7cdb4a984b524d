"""Device-resident LMI index and the search pipeline over liblmi_hip.so.

This is the host side of the hot path (SURVEY.md §3 "Build-side equivalent"):

    queries (HBM) --K1 lmi_router--> classes[:, :R]
                  --K2 lmi_bucket_topk--> per-(query, probe) top-k lists
                  [--RCCL all_gather + K3 lmi_merge_topk, G > 1 ranks]
                  --D2H (nq*R*k*8 B)--> lmi_replay (host C++) --> dists, anns

Layout in HBM (one shard): the search corpus sorted by bucket label, stable in
row order — the order in which the reference's ``groupby('category')`` visits
objects (LearnedIndex.py:143-145) — stored fp16 when every value is exactly
fp16-representable (then the fp16 MFMA products are exact) and fp32 otherwise,
rows padded to a multiple of 32 elements; per-row 1/||y|| (sklearn's
``normalize`` zero rule, utils.py:11); the global position of every row (the
tie-break key); bucket offsets and the chunk table of the scan.

A G-rank index stripes every bucket: rank g holds the g-th contiguous slice of
each bucket's rows (np.array_split boundaries), so every rank scans 1/G of
every probed bucket whatever the bucket popularity.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os
import time
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

DEFAULT_CHUNK_ROWS = 8192
SPLIT_D_PAD = 768  # the split mode's (storage "f32x") row width: the fp16 scan's


def default_chunk_rows(world: int, n_rows: Optional[int] = None) -> int:
    """The scan's chunk (rows) for a shard of a `world`-rank index: 8192 on one
    GPU, 4096 on 2-4, 2048 on more, so a 1/world stripe still cuts into enough
    tiles to fill 256 CUs (DESIGN.md §5 "Chunk size"; tools/gpu_shards.sh);
    given the index's rows, halved (down to 1024) while a rank's shard would
    hold fewer than 64 chunks (configs[1], 300K rows: 4096 -- the scan 0.63
    instead of 0.75 ms, the float64 line +8%, the stream as fast; smaller
    chunks speed the scan further but add plan and merge work to a launch
    the host already bounds, profiles/r05aa_300K_chunk_rows.txt)."""
    c = DEFAULT_CHUNK_ROWS if world <= 1 else 4096 if world <= 4 else 2048
    if n_rows is not None:
        per = n_rows / max(int(world), 1)
        while c > 1024 and per / c < 64:
            c //= 2
    return c
# LMI_Q_SEED_ROUND0 in the thresholded reference replay (LMI_NO_SEED=1: off,
# for A/B measurements; results are the same either way)
_SEED_ROUND0 = os.environ.get("LMI_NO_SEED") != "1"


def _as_torch(x, device=None, dtype=None) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        t = x
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if device is not None:
        t = t.to(device)
    return t.contiguous()


def _rows_f32(x, device) -> torch.Tensor:
    """x as float32 rows on `device` for a kernel that takes a row stride
    (ldq / ldx): a device float32 tensor whose rows are contiguous is passed
    as it is (e.g. a column slice of a staged query batch), anything else is
    converted to a contiguous tensor."""
    if isinstance(x, torch.Tensor) and x.dtype == torch.float32 and x.dim() == 2 and \
            x.device == torch.device(device) and (x.stride(1) == 1 or x.shape[1] == 1):
        return x
    return _as_torch(x, device, torch.float32)


def _inv_norm(rows: torch.Tensor) -> torch.Tensor:
    """1/||y|| per row as the scan uses it: sklearn normalize's rule (norms <
    10 * eps(float32) -> 1, utils.py:11), the norm computed in float64 from the
    stored values and rounded once to float32, so its relative error is at
    most 2^-24 whatever the reduction order (the float64 mode's refine band
    relies on that bound: refine_eps)."""
    f = rows.double()
    norm = torch.sqrt((f * f).sum(dim=1))
    norm = torch.where(norm < 10 * float(np.finfo(np.float32).eps), torch.ones_like(norm), norm)
    return (1.0 / norm).float()


def refine_eps(d_pad: int, f16math: bool, rounded_inputs: bool = False) -> float:
    """The float64 mode's band ε (lmi_bucket_topk_f64): a bound on |d32 - d64|
    for every (query, row), d32 the scan's float32 distance and d64 the
    reference's float64 one, rounded up to a power of two (>= 2^-16).  With
    u = 2^-24, gamma(n) = n*u / (1 - n*u), |cos| <= 1, and every float32
    rounding taken as <= 2u (covers round-to-nearest and truncation):
      dot   fp16 x fp16 products are exact in float32; a v_mfma_f32_32x32x16_f16
            chain adds 16 products per instruction into the accumulator, so a
            product passes at most 16 + d_pad/16 roundings: gamma(h) with
            h = 2 (d_pad/16 + 16) relative to sum |q_i y_i| <= ||q|| ||y||
            (the f32 path, v_mfma_f32_32x32x2_f32 = an fmaf chain: h = 2 (d_pad + 1));
      1/||q|| prep_kernel: per lane 4 * ceil(d_pad/256) fmaf terms, then a
            6-level butterfly: gamma(2 h_q)/2 for the sqrt of the sum, + 4u for
            sqrt and division (<= 2 ulp each);
      1/||y|| float64 norm rounded once (_inv_norm): u;
      scale (1/||q||)(1/||y||) one multiply: 2u; the final fma: 2u absolute.
    rounded_inputs: float64 rows or queries scanned after rounding to float32
    (lmi_index_desc.corpus64, lmi_bucket_topk_f64q): the cosine of the rounded
    vectors differs from the float64 one by <= 4u; 8u are added.
    d_pad = 768: 9.2e-6 (f16 path) -> 2^-16; 9.3e-5 (f32 path) -> 2^-13."""
    u = 2.0 ** -24

    def gamma(n):
        return n * u / (1.0 - n * u)
    h = 2 * (d_pad // 16 + 16) if f16math else 2 * (d_pad + 1)
    hq = 4 * (-(-d_pad // 256)) + 6
    bound = gamma(h) + gamma(2 * hq) / 2 + 4 * u + u + 2 * u + 2 * u + (8 * u if rounded_inputs else 0.0)
    eps = 2.0 ** -16
    while eps < bound:
        eps *= 2.0
    return eps


def _rows_q(x, device) -> torch.Tensor:
    """Query rows for the scan: float32 rows as _rows_f32; float64 queries stay
    float64 (bucket_topk_f64 keeps them for its float64 recomputation;
    bucket_topk rounds them)."""
    if (isinstance(x, torch.Tensor) and x.dtype == torch.float64) or \
            (isinstance(x, np.ndarray) and x.dtype == np.float64):
        return _as_torch(x, device, torch.float64)
    return _rows_f32(x, device)


def fp16_exact(x: torch.Tensor) -> bool:
    """True when every value of the float tensor round-trips through fp16."""
    x = x.float()
    return bool(torch.equal(x.half().float(), x))


# ---------------------------------------------------------------------------
# bucket layout (host arithmetic, shared by every rank)
# ---------------------------------------------------------------------------
@dataclasses.dataclass
class BucketLayout:
    """Bucket-sorted order of the corpus.  Global position p holds row order[p]."""

    n_buckets: int
    order: np.ndarray        # int64 [n]: row index of each global position
    bucket_off: np.ndarray   # int64 [C+1] global offsets

    @classmethod
    def from_labels(cls, labels, n_buckets: int) -> "BucketLayout":
        lab = np.asarray(labels).astype(np.int64, copy=False).ravel()
        if lab.size and (lab.min() < 0 or lab.max() >= n_buckets):
            raise ValueError(f"labels must lie in [0, {n_buckets})")
        order = np.argsort(lab, kind="stable").astype(np.int64)
        size = np.bincount(lab, minlength=n_buckets).astype(np.int64)
        off = np.zeros(n_buckets + 1, np.int64)
        np.cumsum(size, out=off[1:])
        return cls(n_buckets, order, off)

    @property
    def bucket_size(self) -> np.ndarray:
        return np.diff(self.bucket_off)

    def shard(self, rank: int, world: int):
        """(global positions of the shard's rows, local bucket offsets [C+1])."""
        if world == 1:
            return np.arange(self.bucket_off[-1], dtype=np.int64), self.bucket_off.copy()
        parts, loc = [], np.zeros(self.n_buckets + 1, np.int64)
        for c in range(self.n_buckets):
            a, b = self.bucket_off[c], self.bucket_off[c + 1]
            n = b - a
            lo = a + (n * rank) // world
            hi = a + (n * (rank + 1)) // world
            parts.append(np.arange(lo, hi, dtype=np.int64))
            loc[c + 1] = loc[c] + (hi - lo)
        return (np.concatenate(parts) if parts else np.zeros(0, np.int64)), loc


# ---------------------------------------------------------------------------
# device index
# ---------------------------------------------------------------------------
class RowSource:
    """A corpus too large to materialise twice (BASELINE configs[4], 100M x 768):
    ``fn(a, b)`` returns rows [a, b) as an fp16 device tensor [b - a, d] and is
    called on whole chunks [i·chunk, (i+1)·chunk).  DeviceIndex scatters every
    chunk straight into its bucket-sorted slots, so HBM holds the shard once."""

    def __init__(self, n: int, d: int, fn, chunk: int = 1 << 20):
        self.n, self.d, self.fn, self.chunk = int(n), int(d), fn, int(chunk)
        self.shape = (self.n, self.d)

    def chunks(self):
        for a in range(0, self.n, self.chunk):
            b = min(self.n, a + self.chunk)
            yield a, b, self.fn(a, b)


class DeviceIndex:
    """One shard of the bucket-sorted search corpus, resident in HBM.

    storage: "f16" (every value fp16-exact: the fp16 MFMA scan is exact),
    "f32x" (float32 values that are not: the split mode of ABI 9 -- the fp16
    scan runs on each row L2-normalised and rounded to fp16, `corpus`, and the
    rows within its rounding bound of every pair's k-th distance are re-scored
    exactly from the float32 rows, `corpus32`; d_pad 768), or "f32" (the
    general exact-fp32 MFMA scan).  "auto" picks the first that applies."""

    corpus64 = None  # float64 rows (float64 input that float32 rounding changes)
    corpus32 = None  # float32 rows of the split mode (storage "f32x")
    corpus32n = None  # corpus32 normalised as sklearn does in float32 (ABI 11)
    inv_norm32 = None  # 1/||y|| of corpus32 (the general scan's, k > 16 in f32x)

    def __init__(self, data, labels, n_buckets: int, *, ids=None, device=None,
                 storage: str = "auto", chunk_rows: Optional[int] = None,
                 rank: int = 0, world: int = 1, subcluster: bool = False):
        _lib.load()
        self.device = torch.device(device if device is not None else "cuda")
        lab = labels.cpu().numpy() if isinstance(labels, torch.Tensor) else np.asarray(labels)
        self.layout = BucketLayout.from_labels(lab, n_buckets)
        self.n_buckets = n_buckets
        n = int(self.layout.bucket_off[-1])
        self.n_total = n
        if ids is None:
            ids = np.arange(1, n + 1, dtype=np.int64)  # DataFrame.index += 1 (search.py:72)
        ids = np.asarray(ids).astype(np.int64, copy=False)
        if ids.shape != (n,):
            raise ValueError("ids must have one entry per corpus row")
        self.pos_to_id = ids[self.layout.order]
        self.bucket_size = self.layout.bucket_size.copy()
        self.rank, self.world = rank, world

        gpos, loc_off = self.layout.shard(rank, world)
        if isinstance(data, RowSource):
            self._fill_from_source(data, gpos)
        else:
            self._fill(data, gpos, storage)
        self.gpos = torch.from_numpy(gpos.astype(np.int32)).to(self.device)
        self.n_rows = int(gpos.size)
        # (default: by the index's size and world, default_chunk_rows)
        self.chunk_rows = int(chunk_rows) if chunk_rows else default_chunk_rows(world, n)
        cf = np.zeros(n_buckets + 1, np.int32)
        lib = _lib.load()
        mx = lib.lmi_plan_chunks(loc_off.ctypes.data, n_buckets, self.chunk_rows, cf.ctypes.data)
        if mx < 0:
            check("lmi_plan_chunks", -mx)
        self.max_chunks = int(mx)
        self.n_chunks = int(cf[-1])
        self.bucket_off_local = torch.from_numpy(loc_off).to(self.device)
        # every bucket's rows in the whole index (lmi_index_desc.bucket_rows):
        # the shape of the reference's per-bucket product
        self.bucket_rows = torch.from_numpy(np.ascontiguousarray(self.bucket_size, dtype=np.int64)).to(self.device)
        self.chunk_first = torch.from_numpy(cf).to(self.device)
        self.chunk_centroid = None
        if subcluster and self.n_chunks > 0:
            self._subcluster_layout(loc_off, cf)
        self._desc = IndexDescHolder(self)
        self._ws = {}

    @torch.no_grad()
    def _fill(self, data, gpos, storage):
        n = self.n_total
        rows = torch.from_numpy(self.layout.order[gpos])
        if isinstance(data, torch.Tensor):
            src = data
        else:
            a = np.asarray(data)
            a = a if a.dtype in (np.float16, np.float32, np.float64) else a.astype(np.float32)
            src = torch.from_numpy(np.ascontiguousarray(a))
        if src.dim() != 2 or src.shape[0] != n:
            raise ValueError("data must be [n, d] with one row per label")
        src64 = None
        if src.dtype == torch.float64:
            # float64 rows (a float64 data_search): the scan reads them rounded
            # to float32; the float64 mode recomputes from the float64 values
            # when rounding changed any (lmi_index_desc.corpus64)
            src64 = src
            src = src.float()
            step64 = 1 << 20
            if all(torch.equal(src64[a:a + step64].to(self.device),
                               src[a:a + step64].to(self.device).double())
                   for a in range(0, n, step64)):
                src64 = None
        elif src.dtype not in (torch.float16, torch.float32):
            src = src.float()
        self.d = int(src.shape[1])
        self.d_pad = (self.d + 31) // 32 * 32
        step = 1 << 20
        if src64 is not None:
            self.corpus64 = torch.zeros((int(gpos.size), self.d_pad), dtype=torch.float64,
                                        device=self.device)
            for a in range(0, int(gpos.size), step):
                self.corpus64[a:a + step, : self.d] = src64.index_select(
                    0, rows[a:a + step].to(src64.device)).to(self.device)
        if storage == "auto":
            storage = "f16" if src.dtype == torch.float16 or all(
                fp16_exact(src[a:a + step].to(self.device)) for a in range(0, n, step)) else \
                ("f32x" if self.d_pad == SPLIT_D_PAD else "f32")
        if storage not in ("f16", "f32", "f32x"):
            raise ValueError("storage must be 'auto', 'f16', 'f32' or 'f32x'")
        if storage == "f32x" and self.d_pad != SPLIT_D_PAD:
            raise ValueError(f"storage='f32x' needs d_pad {SPLIT_D_PAD}")
        self.storage = storage
        tdt = torch.float32 if storage == "f32" else torch.float16
        n_rows = int(gpos.size)
        self.corpus = torch.zeros((n_rows, self.d_pad), dtype=tdt, device=self.device)
        self.inv_norm = torch.empty((n_rows,), dtype=torch.float32, device=self.device)
        if storage == "f32x":
            self.corpus32 = torch.zeros((n_rows, self.d_pad), dtype=torch.float32, device=self.device)
            self.inv_norm32 = torch.empty((n_rows,), dtype=torch.float32, device=self.device)
        for a in range(0, n_rows, step):
            blk = src.index_select(0, rows[a:a + step].to(src.device)).to(self.device)
            f = blk.float()
            if storage == "f16" and blk.dtype != torch.float16 and not fp16_exact(f):
                raise ValueError("storage='f16' needs fp16-representable data (exact products)")
            if storage == "f32x":
                # the rows as given, and each row / its float64 norm (sklearn's
                # zero rule) rounded to fp16: the split mode's scan rows
                self.corpus32[a:a + step, : self.d] = f
                self.inv_norm32[a:a + step] = _inv_norm(f)
                nrm = torch.sqrt((f.double() * f.double()).sum(dim=1))
                nrm = torch.where(nrm < 10 * float(np.finfo(np.float32).eps), torch.ones_like(nrm), nrm)
                h = (f.double() / nrm[:, None]).float().half()
                self.corpus[a:a + step, : self.d] = h
                self.inv_norm[a:a + step] = _inv_norm(h)
                del blk, f, h, nrm
                continue
            self.corpus[a:a + step, : self.d] = blk.to(tdt)
            self.inv_norm[a:a + step] = _inv_norm(blk.to(tdt))
            del blk, f
        if storage == "f32x" and self.d % 16 == 0 and os.environ.get("LMI_SPLIT_NORM32", "1") != "0":
            # every row divided by its float32 norm as the reference's
            # normalize(Y) computes it, once (lmi_index_desc.corpus32n): the
            # float32 re-score then runs only the product's chains per row
            # (LMI_SPLIT_NORM32=0: normalised per candidate; the same values)
            self.corpus32n = torch.empty_like(self.corpus32)
            check("lmi_split_normalize", _lib.load().lmi_split_normalize(
                ptr(self.corpus32), n_rows, self.d, self.d_pad, ptr(self.corpus32n),
                _lib.stream_handle(self.device)))

    @torch.no_grad()
    def _fill_from_source(self, src: "RowSource", gpos):
        """Scatter every generated chunk into this shard's bucket-sorted slots
        (fp16 storage; 1/||y|| as sklearn's normalize, zero norms -> 1)."""
        n = self.n_total
        if src.n != n:
            raise ValueError("RowSource must have one row per label")
        self.d = src.d
        self.d_pad = (self.d + 31) // 32 * 32
        self.storage = "f16"
        n_rows = int(gpos.size)
        self.corpus = torch.zeros((n_rows, self.d_pad), dtype=torch.float16, device=self.device)
        self.inv_norm = torch.empty((n_rows,), dtype=torch.float32, device=self.device)
        slot = torch.full((n,), -1, dtype=torch.int64, device=self.device)
        slot[torch.from_numpy(self.layout.order[gpos]).to(self.device)] = torch.arange(
            n_rows, dtype=torch.int64, device=self.device)
        for a, b, blk in src.chunks():
            if blk.dtype != torch.float16 or blk.shape != (b - a, self.d):
                raise ValueError("RowSource chunks must be fp16 [b - a, d]")
            sl = slot[a:b]
            m = sl >= 0
            dst = sl[m]
            x = blk[m]
            self.corpus[dst, : self.d] = x
            self.inv_norm[dst] = _inv_norm(x)
            del blk, x
        del slot

    @torch.no_grad()
    def _subcluster_layout(self, loc_off, cf, iters: int = 8, seed: int = 1):
        """Lay out every bucket of more than one chunk by sub-cluster and keep
        each chunk's unit centroid (lmi_index_desc.chunk_centroid).

        Spherical k-means with one centroid per chunk groups the bucket's rows;
        the rows are ordered by (sub-cluster, global position), cut into the
        usual chunks, and every chunk is put back in ascending global position
        (the scan's tie order inside a chunk).  Only the order of rows inside a
        bucket changes: results are identical with or without it; the scan
        uses the centroids to visit each (query, probe)'s nearest chunk first,
        which tightens its pruning bound early (index build, not hot path)."""
        d, cr = self.d, self.chunk_rows
        cent = torch.zeros((self.n_chunks, self.d_pad), dtype=torch.float32, device=self.device)
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        for c in range(self.n_buckets):
            a, b = int(loc_off[c]), int(loc_off[c + 1])
            nch = int(cf[c + 1] - cf[c])
            if nch == 0:
                continue
            if nch > 1:
                x = self.corpus[a:b, :d].float()
                x = x * self.inv_norm[a:b, None]
                n = b - a
                init = torch.randperm(n, generator=g, device=self.device)[:nch]
                ctr = x[init].clone()
                for _ in range(iters):
                    lab = (x @ ctr.T).argmax(dim=1)
                    s = torch.zeros_like(ctr).index_add_(0, lab, x)
                    nrm = s.norm(dim=1, keepdim=True)
                    ctr = torch.where(nrm > 0, s / nrm.clamp(min=1e-30), ctr)
                lab = (x @ ctr.T).argmax(dim=1)
                del x
                gp = self.gpos[a:b].long()
                # order by (sub-cluster, global position), cut into chunks, and
                # restore ascending global position inside every chunk
                order = torch.argsort(lab * (1 << 32) + gp)
                chunk_of = torch.arange(n, device=self.device) // cr
                order = order[torch.argsort(chunk_of * (1 << 32) + gp[order])]
                self.corpus[a:b] = self.corpus[a:b][order]
                self.inv_norm[a:b] = self.inv_norm[a:b][order]
                self.gpos[a:b] = self.gpos[a:b][order]
                # the row arrays that share corpus's local row index (the
                # split mode's float32 rows, the float64 rows) move with it
                for name in ("corpus32", "corpus32n", "inv_norm32", "corpus64"):
                    t = getattr(self, name)
                    if t is not None:
                        t[a:b] = t[a:b][order]
            for j in range(nch):
                ra, rb = a + j * cr, min(b, a + (j + 1) * cr)
                v = (self.corpus[ra:rb, :d].float() * self.inv_norm[ra:rb, None]).sum(dim=0)
                cent[int(cf[c]) + j, :d] = v / v.norm().clamp(min=1e-30)
        self.chunk_centroid = cent

    @property
    def desc(self) -> _lib.IndexDesc:
        return self._desc.desc

    def desc_for(self, k: int) -> _lib.IndexDesc:
        """The descriptor a call with k entries per list takes: the split mode
        (storage "f32x") holds k <= LMI_MAX_K; wider lists scan the float32
        rows with the general exact-fp32 kernel (a second descriptor over
        corpus32)."""
        if self.storage != "f32x" or k <= _lib.LMI_MAX_K:
            return self.desc
        if getattr(self, "_desc32", None) is None:
            self._desc32 = IndexDescHolder(self, general32=True)
        return self._desc32.desc

    def workspace(self, nq: int, R: int, k: int, qmode: int) -> torch.Tensor:
        lib = _lib.load()
        need = lib.lmi_scan_workspace_bytes(C.byref(self.desc_for(k)), nq, R, k, qmode)
        ws = self._ws.get("buf")
        if ws is None or ws.numel() < need:
            ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
            self._ws["buf"] = ws
        return ws


class IndexDescHolder:
    def __init__(self, ix: DeviceIndex, general32: bool = False):
        d = _lib.IndexDesc()
        d.corpus = ptr(ix.corpus32 if general32 else ix.corpus)
        d.dtype = _lib.LMI_F32 if (general32 or ix.storage == "f32") else _lib.LMI_F16
        d.d = ix.d
        d.d_pad = ix.d_pad
        d.n_rows = ix.n_rows
        d.inv_norm = ptr(ix.inv_norm32 if general32 else ix.inv_norm)
        d.gpos = ptr(ix.gpos)
        d.n_buckets = ix.n_buckets
        d.bucket_off = ptr(ix.bucket_off_local)
        d.chunk_rows = ix.chunk_rows
        d.chunk_first = ptr(ix.chunk_first)
        d.n_chunks = ix.n_chunks
        d.max_chunks = ix.max_chunks
        d.chunk_centroid = ptr(ix.chunk_centroid) if ix.chunk_centroid is not None else None
        d.corpus64 = ptr(ix.corpus64) if ix.corpus64 is not None else None
        d.corpus32 = ptr(ix.corpus32) if (ix.corpus32 is not None and not general32) else None
        d.bucket_rows = ptr(ix.bucket_rows)
        d.corpus32n = ptr(ix.corpus32n) if (ix.corpus32n is not None and not general32) else None
        self.desc = d


# ---------------------------------------------------------------------------
# router
# ---------------------------------------------------------------------------
class DeviceRouter:
    """Weights of a Linear/ReLU stack in HBM, evaluated by K1 (lmi_router)."""

    def __init__(self, layers: Sequence, device=None):
        _lib.load()
        self.device = torch.device(device if device is not None else "cuda")
        if not 1 <= len(layers) <= _lib.LMI_MAX_LAYERS:
            raise ValueError("1..8 Linear layers supported")
        self.W, self.b = [], []
        dims = [int(_as_torch(layers[0][0]).shape[1])]
        for (w, b) in layers:
            w = _as_torch(w, self.device, torch.float32)
            b = _as_torch(b, self.device, torch.float32)
            if w.shape[1] != dims[-1] or b.shape != (w.shape[0],):
                raise ValueError("inconsistent layer shapes")
            dims.append(int(w.shape[0]))
            self.W.append(w)
            self.b.append(b)
        self.dims = dims
        self.n_classes = dims[-1]
        m = _lib.MlpDesc()
        m.n_layers = len(self.W)
        for i, v in enumerate(dims):
            m.dims[i] = v
        for i, (w, b) in enumerate(zip(self.W, self.b)):
            m.W[i] = ptr(w)
            m.b[i] = ptr(b)
        self._desc = m

    @classmethod
    def from_module(cls, module: torch.nn.Module, device=None) -> "DeviceRouter":
        """From a reference-shaped ``Model`` (model.py:15-83): ``layers`` is a
        Sequential of Linear with ReLU between consecutive Linears."""
        seq = getattr(module, "layers", module)
        mods = list(seq.children()) if isinstance(seq, torch.nn.Sequential) else [seq]
        layers = []
        for i, m in enumerate(mods):
            if isinstance(m, torch.nn.Linear):
                layers.append((m.weight.detach(), m.bias.detach()))
            elif isinstance(m, torch.nn.ReLU):
                if not layers or i == len(mods) - 1:
                    raise ValueError("ReLU must sit between Linear layers")
            else:
                raise ValueError(f"unsupported router layer {type(m).__name__}")
        for a, b in zip(mods, mods[1:]):
            if isinstance(a, torch.nn.Linear) and not isinstance(b, torch.nn.ReLU):
                raise ValueError("expected ReLU after every hidden Linear")
        return cls(layers, device)

    def topr(self, x: torch.Tensor, R: int, with_probs: bool = False, stream=None, out=None):
        """K1 TOPR: classes [nq, R] int32 (into `out` when given, a contiguous
        int32 tensor of nq*R elements) and, with `with_probs`, their softmax
        probabilities."""
        x = _rows_f32(x, self.device)
        nq = x.shape[0]
        if out is not None:
            if out.dtype != torch.int32 or out.numel() != nq * R or not out.is_contiguous():
                raise ValueError("out must be a contiguous int32 tensor of nq*R elements")
            classes = out.view(nq, R)
        else:
            classes = torch.empty((nq, R), dtype=torch.int32, device=self.device)
        probs = torch.empty((nq, R), dtype=torch.float32, device=self.device) if with_probs else None
        s = stream if stream is not None else _lib.stream_handle(self.device)
        check("lmi_router", _lib.load().lmi_router(ptr(x), nq, x.stride(0), C.byref(self._desc), R,
                                                   _lib.LMI_ROUTER_TOPR, ptr(classes), ptr(probs), s))
        return classes, probs

    def argmax(self, x: torch.Tensor, stream=None) -> torch.Tensor:
        x = _rows_f32(x, self.device)
        nq = x.shape[0]
        out = torch.empty((nq,), dtype=torch.int32, device=self.device)
        s = stream if stream is not None else _lib.stream_handle(self.device)
        check("lmi_router", _lib.load().lmi_router(ptr(x), nq, x.stride(0), C.byref(self._desc), 1,
                                                   _lib.LMI_ROUTER_ARGMAX, ptr(out), 0, s))
        return out


# ---------------------------------------------------------------------------
# scan / merge / replay
# ---------------------------------------------------------------------------
def _workspace(ws, need: int, what: str) -> torch.Tensor:
    if ws.dtype != torch.uint8 or ws.numel() < need:
        raise ValueError(f"{what} workspace too small ({ws.numel()} < {need} bytes)")
    return ws


def bucket_topk(index: DeviceIndex, q: torch.Tensor, classes: torch.Tensor, k: int,
                qmode: Optional[int] = None, stream=None, out=None, ws=None,
                seed_round0: bool = False, phases: int = 0):
    """K2 on one shard.  Returns (d [nq,R,k] f32, pos [nq,R,k] int32, status int32 tensor);
    `out` = such a triple to write into (the status word zeroed by the caller);
    `ws` = a caller-owned uint8 workspace (default: the index's cached one,
    which a later call with a larger batch may replace — a captured graph
    passes its own).  `seed_round0` (LMI_Q_SEED_ROUND0, the thresholded
    replay only): probes r >= 1 keep only objects under the round-0 bound.
    `phases` (LMI_Q_PHASE_* bits, 0 = all): run only those phases of the call
    (StreamedSearch overlaps one batch's plan with another's scan)."""
    lib = _lib.load()
    q = _rows_f32(q, index.device)
    classes = _as_torch(classes, index.device, torch.int32)
    nq, R = classes.shape
    if q.shape[0] != nq or q.shape[1] != index.d:
        raise ValueError("query shape does not match the index")
    if qmode is None:
        qmode = _lib.LMI_Q_F16 if index.storage == "f16" else _lib.LMI_Q_F32
    desc = index.desc_for(k)
    if out is None:
        out_d = torch.empty((nq, R, k), dtype=torch.float32, device=index.device)
        out_pos = torch.empty((nq, R, k), dtype=torch.int32, device=index.device)
        status = torch.zeros((1,), dtype=torch.int32, device=index.device)
    else:
        out_d, out_pos, status = out
    if ws is None:
        ws = index.workspace(nq, R, k, qmode)
    else:
        _workspace(ws, lib.lmi_scan_workspace_bytes(C.byref(desc), nq, R, k, qmode), "scan")
    s = stream if stream is not None else _lib.stream_handle(index.device)
    if index.storage == "f32x":
        seed_round0 = False  # (the split mode scans every pair whole)
    flags = (_lib.LMI_Q_SEED_ROUND0 if seed_round0 else 0) | phases
    check("lmi_bucket_topk", lib.lmi_bucket_topk(C.byref(desc), ptr(q), nq, q.stride(0),
                                                 ptr(classes), R, k, qmode | flags, ptr(out_d),
                                                 ptr(out_pos), ptr(status), ptr(ws), ws.numel(), s))
    return out_d, out_pos, status


def bucket_topk_f64(index: DeviceIndex, q: torch.Tensor, classes: torch.Tensor, k: int,
                    qmode: Optional[int] = None, eps: Optional[float] = None, stream=None,
                    fallback_count: bool = False, out=None, ws=None, seed_round0: bool = False,
                    phases: int = 0, band_x=None):
    """K2 with float64 distances (lmi_bucket_topk_f64): the reference's
    arithmetic when either operand is not float32 (utils.py:11, :19).  Returns
    (d f64 [nq,R,k], pos [nq,R,k] int32, status int32 tensor[, n_fallback]);
    `out` and `ws` as bucket_topk.  Float64 queries whose float32 rounding
    changes them are kept for the float64 recomputation (lmi_bucket_topk_f64q;
    the scan reads them rounded).  `band_x` = (kth_send, kth_all, G): the
    band decided over G ranks (lmi_bucket_topk_f64g, ABI 10; kth_send f32
    [nq*R*k] written by the MERGE phase, kth_all f32 [G, nq*R*k] read by the
    REFINE phase, LMI_Q_PHASE_REFINE in `phases`)."""
    lib = _lib.load()
    q64 = None
    if isinstance(q, torch.Tensor) and q.dtype == torch.float64 or \
            isinstance(q, np.ndarray) and q.dtype == np.float64:
        q64 = _as_torch(q, index.device, torch.float64)
        q = q64.float()
        if torch.equal(q.double(), q64):
            q64 = None
    q = _rows_f32(q, index.device)
    classes = _as_torch(classes, index.device, torch.int32)
    nq, R = classes.shape
    if q.shape[0] != nq or q.shape[1] != index.d:
        raise ValueError("query shape does not match the index")
    if qmode is None:
        qmode = _lib.LMI_Q_F16 if index.storage == "f16" else _lib.LMI_Q_F32
    if eps is None:
        eps = refine_eps(index.d_pad, index.storage == "f16" and qmode == _lib.LMI_Q_F16,
                         rounded_inputs=q64 is not None or index.corpus64 is not None)
    if out is None:
        out_d = torch.empty((nq, R, k), dtype=torch.float64, device=index.device)
        out_pos = torch.empty((nq, R, k), dtype=torch.int32, device=index.device)
        status = torch.zeros((1,), dtype=torch.int32, device=index.device)
    else:
        out_d, out_pos, status = out
    desc = index.desc_for(k)
    need = lib.lmi_scan_f64_workspace_bytes(C.byref(desc), nq, R, k, qmode)
    if ws is None:
        ws = index._ws.get("f64")
        if ws is None or ws.numel() < need:
            ws = torch.empty(max(need, 256), dtype=torch.uint8, device=index.device)
            index._ws["f64"] = ws
    else:
        _workspace(ws, need, "float64 scan")
    s = stream if stream is not None else _lib.stream_handle(index.device)
    if index.storage == "f32x":
        seed_round0 = False  # (the split mode scans every pair whole)
    flags = (_lib.LMI_Q_SEED_ROUND0 if seed_round0 else 0) | phases
    if band_x is not None:
        kth_send, kth_all, G = band_x
        check("lmi_bucket_topk_f64g", lib.lmi_bucket_topk_f64g(
            C.byref(desc), ptr(q), nq, q.stride(0), ptr(q64), 0 if q64 is None else q64.stride(0),
            ptr(classes), R, k, qmode | flags, float(eps), ptr(kth_send), ptr(kth_all), int(G),
            nq * R * k, ptr(out_d), ptr(out_pos), ptr(status), ptr(ws), ws.numel(), s))
    else:
        check("lmi_bucket_topk_f64q", lib.lmi_bucket_topk_f64q(
            C.byref(desc), ptr(q), nq, q.stride(0), ptr(q64), 0 if q64 is None else q64.stride(0),
            ptr(classes), R, k, qmode | flags, float(eps), ptr(out_d), ptr(out_pos), ptr(status),
            ptr(ws), ws.numel(), s))
    if not fallback_count:
        return out_d, out_pos, status
    n = C.c_int32(0)
    check("lmi_refine_fallback_count", lib.lmi_refine_fallback_count(
        ptr(ws), C.byref(desc), nq, R, k, qmode, C.byref(n), s))
    return out_d, out_pos, status, int(n.value)


def split_sample_fallback_count(index: DeviceIndex, nq: int, R: int, k: int, ws=None,
                                f64: bool = False, stream=None) -> int:
    """The split mode (k <= 10, ABI 13): how many pairs of the last call on
    this workspace (`ws`, else the index's own: bucket_topk's, or
    bucket_topk_f64's with f64=True) had a band reaching their skipped
    sample's k-th and were scored over the sample rows and candidates
    (lmi_split_sample_fallback_count)."""
    lib = _lib.load()
    if ws is None:
        ws = index._ws.get("f64" if f64 else "buf")
    n = C.c_int32(0)
    s = stream if stream is not None else _lib.stream_handle(index.device)
    check("lmi_split_sample_fallback_count", lib.lmi_split_sample_fallback_count(
        ptr(ws), C.byref(index.desc_for(k)), nq, R, k, C.byref(n), s))
    return int(n.value)


def global_band(index: DeviceIndex, nq: int, R: int, k: int, qmode: int) -> bool:
    """True when the float64 search of a striped index can decide its band
    over every rank's lists (lmi_f64_global_band: the band lists, k <= 10 on
    the fp16 scan, no split mode); LMI_F64_LOCAL_BAND=1 turns it off (every
    rank refines the band of its own list, the round-5 form)."""
    if os.environ.get("LMI_F64_LOCAL_BAND") == "1":
        return False
    return bool(_lib.load().lmi_f64_global_band(C.byref(index.desc_for(k)), nq, R, k, qmode))


def merge_topk(d_in: torch.Tensor, pos_in: torch.Tensor, k: int, stream=None):
    """K3: merge [G, rows, k] lists -> [rows, k] by (distance, global position);
    float32 (lmi_merge_topk) or float64 (lmi_merge_topk_f64) distances."""
    G = d_in.shape[0]
    rows = d_in[0].numel() // k
    f64 = d_in.dtype == torch.float64
    out_d = torch.empty(d_in.shape[1:], dtype=d_in.dtype, device=d_in.device)
    out_pos = torch.empty(d_in.shape[1:], dtype=torch.int32, device=d_in.device)
    s = stream if stream is not None else _lib.stream_handle(d_in.device)
    fn = "lmi_merge_topk_f64" if f64 else "lmi_merge_topk"
    check(fn, getattr(_lib.load(), fn)(ptr(d_in.contiguous()), ptr(pos_in.contiguous()), G, rows, k,
                                       ptr(out_d), ptr(out_pos), s))
    return out_d, out_pos


def replay(classes: np.ndarray, lists_d: np.ndarray, lists_pos: np.ndarray, *, k_round: int,
           k_final: int, bucket_size: np.ndarray, pos_to_id: np.ndarray, use_threshold: bool,
           thr_round0: Optional[np.ndarray] = None):
    """A5 on the host (lmi_replay, or lmi_replay_f64 for float64 lists):
    per-(query, probe) lists -> reference output."""
    classes = np.ascontiguousarray(classes, dtype=np.int32)
    if classes.ndim == 1:
        classes = classes[:, None]
    nq, R = classes.shape
    f64 = np.asarray(lists_d).dtype == np.float64
    lists_d = np.ascontiguousarray(lists_d, dtype=np.float64 if f64 else np.float32).reshape(nq, R, -1)
    lists_pos = np.ascontiguousarray(lists_pos, dtype=np.int32).reshape(nq, R, -1)
    k_list = lists_d.shape[2]
    bucket_size = np.ascontiguousarray(bucket_size, dtype=np.int64)
    pos_to_id = np.ascontiguousarray(pos_to_id, dtype=np.int64)
    w = k_round if R == 1 else k_final
    dists = np.empty((nq, w), np.float64)
    anns = np.empty((nq, w), np.uint32)
    thr = None
    if thr_round0 is not None:
        thr = np.ascontiguousarray(np.asarray(thr_round0, dtype=np.float64).ravel())
        if thr.shape != (nq,):
            raise ValueError("threshold_dist must have one value per query")
    w_out = C.c_int32(0)
    fn = "lmi_replay_f64" if f64 else "lmi_replay"
    check(fn, getattr(_lib.load(), fn)(
        classes.ctypes.data, nq, R, k_list, lists_d.ctypes.data, lists_pos.ctypes.data,
        k_round, k_final, bucket_size.ctypes.data, bucket_size.size, pos_to_id.ctypes.data,
        pos_to_id.size, int(bool(use_threshold)), ptr(thr), dists.ctypes.data, anns.ctypes.data,
        C.byref(w_out)))
    return dists, anns


def replay_device(classes: torch.Tensor, lists_d: torch.Tensor, lists_pos: torch.Tensor, *,
                  k_round: int, k_final: int, bucket_size: torch.Tensor, pos_to_id: torch.Tensor,
                  use_threshold: bool, thr_round0: Optional[torch.Tensor] = None, stream=None,
                  out=None, phases: int = 3, ws: Optional[torch.Tensor] = None,
                  k_list: Optional[int] = None):
    """A5 on the device (lmi_replay_device_phase; float32 or float64 lists):
    same results as `replay`, device tensors in and out: (dists f64 [nq, w],
    anns uint32-as-int32 [nq, w], status); `out` = such a triple to write into
    (the status word zeroed by the caller, or by a GROUPS phase).  `phases`:
    LMI_REPLAY_PHASE_GROUPS (classes only: lists_d / lists_pos may be None,
    then give `k_list`, the lists' width, and float32 is assumed for sizing),
    LMI_REPLAY_PHASE_ROUNDS, or both (3); the calls of one replay share `ws`
    (a caller-owned uint8 workspace; default: a new one per call)."""
    lib = _lib.load()
    dev = classes.device if lists_d is None else lists_d.device
    classes = _as_torch(classes, dev, torch.int32)
    if classes.dim() == 1:
        classes = classes[:, None].contiguous()
    nq, R = classes.shape
    f64 = lists_d is not None and lists_d.dtype == torch.float64
    if lists_d is not None:
        lists_d = _as_torch(lists_d, dev, torch.float64 if f64 else torch.float32).reshape(nq, R, -1).contiguous()
        lists_pos = _as_torch(lists_pos, dev, torch.int32).reshape(nq, R, -1).contiguous()
        k_list = lists_d.shape[2]
    w = k_round if R == 1 else k_final
    if out is None:
        dists = torch.empty((nq, w), dtype=torch.float64, device=dev)
        anns = torch.empty((nq, w), dtype=torch.int32, device=dev)  # uint32 bits
        status = torch.zeros((1,), dtype=torch.int32, device=dev)
    else:
        dists, anns, status = out
    n_b = int(bucket_size.numel())
    need = lib.lmi_replay_device_workspace_bytes(nq, R, k_list, k_round, k_final, n_b)
    if ws is None:
        ws = torch.empty(max(int(need), 256), dtype=torch.uint8, device=dev)
    else:
        _workspace(ws, need, "replay")
    thr = None
    if thr_round0 is not None:
        thr = _as_torch(thr_round0, dev, torch.float64).reshape(-1)
        if thr.numel() != nq:
            raise ValueError("threshold_dist must have one value per query")
    s = stream if stream is not None else _lib.stream_handle(dev)
    check("lmi_replay_device_phase", lib.lmi_replay_device_phase(
        int(phases), int(f64), ptr(classes), nq, R, k_list, ptr(lists_d), ptr(lists_pos), k_round,
        k_final, ptr(bucket_size), n_b, ptr(pos_to_id), int(pos_to_id.numel()),
        int(bool(use_threshold)), ptr(thr), ptr(dists), ptr(anns), ptr(status), ptr(ws), ws.numel(), s))
    return dists, anns, status


def answer_buffer(nq: int, w: int, device):
    """The step's answer in ONE device buffer, so it crosses PCIe in one copy:
    int32 words [dists f64 nq*w (2 words each)][anns uint32 nq*w][scan status,
    replay status] -> (buf, dists [nq, w], anns [nq, w], status words [2],
    zeroed)."""
    n = nq * w
    buf = torch.empty((3 * n + 2,), dtype=torch.int32, device=device)
    st = buf[3 * n:]
    st.zero_()
    return buf, buf[:2 * n].view(torch.float64).view(nq, w), buf[2 * n:3 * n].view(nq, w), st


def answer_views(h: torch.Tensor, nq: int, w: int):
    """numpy views of an answer buffer copied to the host:
    (dists f64 [nq, w], anns uint32 [nq, w], scan status, replay status)."""
    a = h.numpy()
    n = nq * w
    return (a[:2 * n].view(np.float64).reshape(nq, w), a[2 * n:3 * n].view(np.uint32).reshape(nq, w),
            int(a[3 * n]), int(a[3 * n + 1]))


class Searcher:
    """Runs the whole hot path for one shard set (one process per GPU).

    ``search`` times like search.py:116-141 (router + scan + merge + replay)."""

    def __init__(self, index: DeviceIndex, router: DeviceRouter, group=None,
                 exchange: Optional[bool] = None):
        """`exchange`: run the list exchange (route_sharded, K2 into the packed
        send buffer, the all-gather, lmi_merge_topk_packed) over the process
        group.  None (default): when a group is initialised and the index is
        a stripe of a G > 1 index, the group has G > 1 ranks, or
        LMI_FORCE_EXCHANGE=1 (li.dist.force_exchange: a one-rank RCCL group
        then takes the G > 1 branch of every step form, so the exchange runs
        on one GPU exactly as on eight)."""
        import torch.distributed as tdist
        from .dist import force_exchange
        self.index = index
        self.router = router
        self.group = group
        grouped = tdist.is_available() and tdist.is_initialized()
        if exchange is None:
            exchange = grouped and (index.world > 1 or tdist.get_world_size(group) > 1
                                    or force_exchange())
        if exchange and not grouped:
            raise ValueError("the list exchange needs an initialised process group")
        self.exchange = bool(exchange)
        self._pinned = {}
        self._qcheck = None

    def _host(self, name, shape, dtype):
        buf = self._pinned.get(name)
        if buf is None or tuple(buf.shape) != tuple(shape) or buf.dtype != dtype:
            buf = torch.empty(shape, dtype=dtype, pin_memory=torch.cuda.is_available())
            self._pinned[name] = buf
        return buf

    def qmode(self, q_search: torch.Tensor) -> int:
        """The scan's query path, decided before the scan: LMI_Q_F16 (exact
        fp16 MFMA products) when the corpus is stored fp16 and every query
        value is fp16-representable, else LMI_Q_F32 (exact fp32 MFMA).  The
        check is one device reduction, run once per query batch (cached by the
        tensor's storage, shape and version counter); every rank holds the same
        batch, so every rank decides the same."""
        if self.index.storage != "f16":
            return _lib.LMI_Q_F32
        import weakref
        q = q_search
        # keyed by the live tensor object (a weak reference) and its version
        # counter: a new tensor that reuses a freed one's memory, or the same
        # tensor written in place, is checked again
        key = (q.data_ptr(), q._version, tuple(q.shape), q.stride(), q.dtype, q.device)
        if self._qcheck is not None and self._qcheck[0] == key and self._qcheck[2]() is q:
            return self._qcheck[1]
        mode = _lib.LMI_Q_F16 if fp16_exact(q) else _lib.LMI_Q_F32
        self._qcheck = (key, mode, weakref.ref(q))
        return mode

    def _scan(self, q_search, classes, k_list: int, qmode: int, f64: bool, lap=None,
              status_out=None, ws=None, seed_round0: bool = False):
        """K2 on this shard (+ all-gather and K3 for G > 1 ranks, the status
        words riding along so every rank sees every rank's bits).  `lap`
        (measurement only) is called after the scan and after the exchange.
        `status_out` (a zeroed device int32 word): the status lands there.
        `ws`: a caller-owned scan workspace (GraphedSearch's)."""
        out = None
        if not self.exchange and status_out is not None:
            nq, R = classes.shape
            dev = self.index.device
            out = (torch.empty((nq, R, k_list), dtype=torch.float64 if f64 else torch.float32,
                               device=dev),
                   torch.empty((nq, R, k_list), dtype=torch.int32, device=dev), status_out)
        if self.exchange:
            # the lists and the status word land in this rank's slice of the
            # all-gather's packed send buffer (li.dist.packed_lists)
            from .dist import packed_lists
            nq, R = classes.shape
            buf, dv, pv, sv = packed_lists(nq * R, k_list, f64, self.index.device)
            out = (dv.view(nq, R, k_list), pv.view(nq, R, k_list), sv)
        if f64 and self.exchange and global_band(self.index, nq, R, k_list, qmode):
            # the band decided over every rank's lists (ABI 10): the ranks'
            # k smallest d32 per pair are all-gathered between the chunk merge
            # and the float64 refinement, so each rank refines only its own
            # rows of the merged band
            from .dist import _all_gather
            G = torch.distributed.get_world_size(self.group)
            kth = torch.empty((nq * R * k_list,), dtype=torch.float32, device=q_search.device)
            kall = torch.empty((G, nq * R * k_list), dtype=torch.float32, device=q_search.device)
            ph = _lib.LMI_Q_PHASE_PLAN | _lib.LMI_Q_PHASE_SCAN | _lib.LMI_Q_PHASE_MERGE
            bucket_topk_f64(self.index, q_search, classes, k_list, qmode=qmode, out=out, ws=ws,
                            seed_round0=seed_round0, phases=ph, band_x=(kth, None, G))
            _all_gather(kall.view(-1), kth, self.group)
            d, pos, status = bucket_topk_f64(self.index, q_search, classes, k_list, qmode=qmode,
                                             out=out, ws=ws, seed_round0=seed_round0,
                                             phases=_lib.LMI_Q_PHASE_REFINE, band_x=(None, kall, G))
        elif f64:
            d, pos, status = bucket_topk_f64(self.index, q_search, classes, k_list, qmode=qmode,
                                             out=out, ws=ws, seed_round0=seed_round0)
        else:
            d, pos, status = bucket_topk(self.index, q_search, classes, k_list, qmode=qmode, out=out,
                                         ws=ws, seed_round0=seed_round0)
        if lap:
            lap("scan")
        if self.exchange:
            from .dist import gather_merge_packed
            d, pos, status = gather_merge_packed(buf, nq * R, k_list, f64, self.group,
                                                 status_out=status_out)
            d, pos = d.view(nq, R, k_list), pos.view(nq, R, k_list)
            if lap:
                lap("allgather")
        return d, pos, status

    def lists(self, q_nav: torch.Tensor, q_search: torch.Tensor, R: int, k_list: int,
              classes: Optional[torch.Tensor] = None, dist: str = "f32"):
        """Device part: router + scan (+ RCCL merge).  Returns device tensors."""
        if classes is None:
            classes = self.route(q_nav, R)
        q_search = _rows_q(q_search, self.index.device)
        d, pos, status = self._scan(q_search, classes, k_list, self.qmode(q_search), dist == "f64")
        return classes, d, pos, status

    def route(self, q_nav, R: int) -> torch.Tensor:
        """K1 classes [nq, R]; with G > 1 ranks each routes nq/G queries and
        the classes are all-gathered (li.dist.route_sharded)."""
        if self.exchange:
            from .dist import route_sharded
            return route_sharded(self.router, _rows_f32(q_nav, self.index.device), R, self.group)
        return self.router.topr(q_nav, R)[0]

    def _device_tables(self):
        """bucket sizes and position -> id map in HBM for the device replay."""
        t = getattr(self, "_dev_tables", None)
        if t is None:
            dev = self.index.device
            t = (torch.from_numpy(np.ascontiguousarray(self.index.bucket_size, dtype=np.int64)).to(dev),
                 torch.from_numpy(np.ascontiguousarray(self.index.pos_to_id, dtype=np.int64)).to(dev))
            self._dev_tables = t
        return t

    def streamed(self, q_nav, q_search, R: int, k: int = 10, **kw) -> "StreamedSearch":
        """The step as a four-stage pipeline of captured graphs over a stream
        of batches (StreamedSearch); answers equal search(...) per batch."""
        from .stream import StreamedSearch
        return StreamedSearch(self, q_nav, q_search, R, k, **kw)

    def graph(self, q_nav, q_search, R: int, k: int = 10, **kw) -> "GraphedSearch":
        """The step captured as a HIP graph (GraphedSearch), from the batch in
        host memory to the answer in host memory: same results as
        search(..., semantics="reference", replay_on="device")."""
        from .graphed import GraphedSearch
        return GraphedSearch(self, q_nav, q_search, R, k, **kw)

    def search(self, q_nav, q_search, R: int, k: int = 10, *, k_round: int = 10,
               use_threshold: bool = True, classes: Optional[torch.Tensor] = None,
               timings: Optional[dict] = None, replay_on: str = "device",
               semantics: str = "reference", dist: str = "f32"):
        """Whole hot path for one batch -> (dists f64 [nq, w], anns u32 [nq, w]).

        semantics="reference" (default) reproduces LearnedIndex.search's round
        merge (thresholds, fillers, the <k quirk).
        semantics="exact" returns instead the exact top-k, by (distance, id
        position), of the union of each query's R probed buckets (K3 merge of
        its R lists on the device; fewer than k objects pad with (10000, 0)),
        the option SURVEY.md §8(a) asks for beside the reference semantics.

        dist="f32": distances in float32, the reference's arithmetic when the
        corpus and the queries are both float32; dist="f64": float64 distances
        (lmi_bucket_topk_f64), its arithmetic otherwise — e.g. the real clip768
        'emb', which is float16 (utils.py:11, :19).

        replay_on="device" (default) runs the reference's round merge on the GPU
        (lmi_replay_device) and copies back only the result; "host" copies the
        lists back and runs lmi_replay (same results, the checker of the device
        replay).  `timings` (measurement only) receives per-stage wall times in
        ms; the stages are then separated by stream synchronisations."""
        import time
        if replay_on not in ("device", "host"):
            raise ValueError("replay_on must be 'device' or 'host'")
        if semantics not in ("reference", "exact"):
            raise ValueError("semantics must be 'reference' or 'exact'")
        if dist not in ("f32", "f64"):
            raise ValueError("dist must be 'f32' or 'f64'")
        k_list = k_round if semantics == "reference" else max(k_round, k)
        f64 = dist == "f64"
        kmax = _lib.LMI_MAX_K_F64 if f64 else _lib.LMI_MAX_K_PASSES
        if k_list > kmax:
            raise ValueError(f"k={k_list} > {kmax}")
        if k_round > _lib.LMI_REPLAY_DEVICE_MAX_KR or k > _lib.LMI_REPLAY_DEVICE_MAX_K:
            replay_on = "host"  # the device replay holds rows of <= 32 / 64 entries
        dev = self.index.device
        sync = (lambda: torch.cuda.current_stream(dev).synchronize()) if timings is not None else None

        def lap(name, t0):
            if sync:
                sync()
                t1 = time.perf_counter()
                timings[name] = timings.get(name, 0.0) + (t1 - t0) * 1e3
                return t1
            return t0

        t0 = time.perf_counter()
        q_search = _rows_q(q_search, dev)
        qmode = self.qmode(q_search)
        if classes is None:
            classes = self.route(q_nav, R)
        t0 = lap("router", t0)
        tl = [t0]

        def lap_at(name):
            tl[0] = lap(name, tl[0])

        nq = classes.shape[0]
        ans = None
        if semantics == "reference" and replay_on == "device":
            # the answer and both status words in one buffer: one D2H copy
            w_ans = k_round if classes.shape[1] == 1 else k
            ans = answer_buffer(nq, w_ans, dev)
        # (valid while the merged width k is at most the round lists' k_round:
        # the running threshold then never exceeds round 0's k-th distance;
        # with k > k_round the first merge pads with 10000s)
        seed = semantics == "reference" and use_threshold and k <= k_round and _SEED_ROUND0
        d, pos, status = self._scan(q_search, classes, k_list, qmode, f64, lap_at if sync else None,
                                    status_out=None if ans is None else ans[3][0:1],
                                    seed_round0=seed)
        t0 = tl[0]
        h_st = self._host("st", (2,), torch.int32)

        def check_status(st, rst=0):
            # every rank holds the OR of all ranks' scan bits (they rode the
            # all-gather) and runs the same replay: all ranks raise together
            if st & _lib.LMI_STATUS_INTERNAL or rst:
                raise RuntimeError(f"search: internal status {st}/{rst}")
            return bool(st & _lib.LMI_STATUS_QUERY_NOT_F16)

        if semantics == "exact":
            _, p2id = self._device_tables()

            def exact(d, pos):
                Rr = classes.shape[1]
                md, mp = merge_topk(d.view(nq, Rr, k_list).transpose(0, 1).contiguous(),
                                    pos.view(nq, Rr, k_list).transpose(0, 1).contiguous(), k_list)
                md, mp = md[:, :k], mp[:, :k]
                none = mp < 0
                ids = p2id[mp.clamp(min=0).long()]
                return (torch.where(none, torch.full_like(md, 10000.0), md).double(),
                        torch.where(none, torch.zeros_like(ids), ids).to(torch.int32))

            rd, ra = exact(d, pos)
            t0 = lap("replay", t0)
            h_d = self._host("xd", tuple(rd.shape), torch.float64)
            h_a = self._host("xa", tuple(ra.shape), torch.int32)
            h_d.copy_(rd, non_blocking=True)
            h_a.copy_(ra, non_blocking=True)
            h_st[0:1].copy_(status, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
            t0 = lap("d2h", t0)
            if check_status(int(h_st[0])):
                # the cached fp16 check was stale: redo with exact fp32 MFMA
                d, pos, status = self._scan(q_search, classes, k_list, _lib.LMI_Q_F32, f64)
                rd, ra = exact(d, pos)
                h_d.copy_(rd)
                h_a.copy_(ra)
                h_st[0:1].copy_(status)
                check_status(int(h_st[0]) & ~_lib.LMI_STATUS_QUERY_NOT_F16)
            return h_d.numpy().copy(), h_a.numpy().view(np.uint32).copy()
        if replay_on == "device":
            bsz, p2id = self._device_tables()

            def run_replay(d, pos, ans):
                replay_device(classes, d, pos, k_round=k_round, k_final=k, bucket_size=bsz,
                              pos_to_id=p2id, use_threshold=use_threshold,
                              out=(ans[1], ans[2], ans[3][1:2]))
                # a fresh pinned buffer from torch's caching host allocator,
                # handed to the caller as numpy views (no host copy; it returns
                # to the cache when the caller drops the arrays)
                h = torch.empty(tuple(ans[0].shape), dtype=torch.int32, pin_memory=True)
                h.copy_(ans[0], non_blocking=True)
                return h

            h = run_replay(d, pos, ans)
            t0 = lap("replay", t0)
            torch.cuda.current_stream(dev).synchronize()
            t0 = lap("d2h", t0)
            hd, ha, st0, st1 = answer_views(h, nq, w_ans)
            if check_status(st0, st1):
                ans = answer_buffer(nq, w_ans, dev)
                d, pos, status = self._scan(q_search, classes, k_list, _lib.LMI_Q_F32, f64,
                                            status_out=ans[3][0:1], seed_round0=seed)
                h = run_replay(d, pos, ans)
                torch.cuda.current_stream(dev).synchronize()
                hd, ha, st0, st1 = answer_views(h, nq, w_ans)
                check_status(st0 & ~_lib.LMI_STATUS_QUERY_NOT_F16, st1)
            return hd, ha
        h_cls = self._host("cls", (nq, R), torch.int32)
        h_d = self._host("d", tuple(d.shape), d.dtype)
        h_pos = self._host("pos", tuple(pos.shape), torch.int32)
        h_cls.copy_(classes, non_blocking=True)
        h_d.copy_(d, non_blocking=True)
        h_pos.copy_(pos, non_blocking=True)
        h_st[0:1].copy_(status, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        t0 = lap("d2h", t0)
        if check_status(int(h_st[0])):
            d, pos, status = self._scan(q_search, classes, k_list, _lib.LMI_Q_F32, f64,
                                        seed_round0=seed)
            h_d.copy_(d)
            h_pos.copy_(pos)
            h_st[0:1].copy_(status)
            check_status(int(h_st[0]) & ~_lib.LMI_STATUS_QUERY_NOT_F16)
        out = replay(h_cls.numpy(), h_d.numpy(), h_pos.numpy(), k_round=k_round, k_final=k,
                     bucket_size=self.index.bucket_size, pos_to_id=self.index.pos_to_id,
                     use_threshold=use_threshold)
        lap("replay", t0) if sync else None
        return out
