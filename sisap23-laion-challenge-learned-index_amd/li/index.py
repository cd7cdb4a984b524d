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
    """One shard of the bucket-sorted search corpus, resident in HBM."""

    corpus64 = None  # float64 rows (float64 input that float32 rounding changes)

    def __init__(self, data, labels, n_buckets: int, *, ids=None, device=None,
                 storage: str = "auto", chunk_rows: int = DEFAULT_CHUNK_ROWS,
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
        self.chunk_rows = int(chunk_rows)
        cf = np.zeros(n_buckets + 1, np.int32)
        lib = _lib.load()
        mx = lib.lmi_plan_chunks(loc_off.ctypes.data, n_buckets, self.chunk_rows, cf.ctypes.data)
        if mx < 0:
            check("lmi_plan_chunks", -mx)
        self.max_chunks = int(mx)
        self.n_chunks = int(cf[-1])
        self.bucket_off_local = torch.from_numpy(loc_off).to(self.device)
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
                fp16_exact(src[a:a + step].to(self.device)) for a in range(0, n, step)) else "f32"
        if storage not in ("f16", "f32"):
            raise ValueError("storage must be 'auto', 'f16' or 'f32'")
        self.storage = storage
        tdt = torch.float16 if storage == "f16" else torch.float32
        n_rows = int(gpos.size)
        self.corpus = torch.zeros((n_rows, self.d_pad), dtype=tdt, device=self.device)
        self.inv_norm = torch.empty((n_rows,), dtype=torch.float32, device=self.device)
        for a in range(0, n_rows, step):
            blk = src.index_select(0, rows[a:a + step].to(src.device)).to(self.device)
            f = blk.float()
            if storage == "f16" and blk.dtype != torch.float16 and not fp16_exact(f):
                raise ValueError("storage='f16' needs fp16-representable data (exact products)")
            self.corpus[a:a + step, : self.d] = blk.to(tdt)
            self.inv_norm[a:a + step] = _inv_norm(blk.to(tdt))
            del blk, f

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
            for j in range(nch):
                ra, rb = a + j * cr, min(b, a + (j + 1) * cr)
                v = (self.corpus[ra:rb, :d].float() * self.inv_norm[ra:rb, None]).sum(dim=0)
                cent[int(cf[c]) + j, :d] = v / v.norm().clamp(min=1e-30)
        self.chunk_centroid = cent

    @property
    def desc(self) -> _lib.IndexDesc:
        return self._desc.desc

    def workspace(self, nq: int, R: int, k: int, qmode: int) -> torch.Tensor:
        lib = _lib.load()
        need = lib.lmi_scan_workspace_bytes(C.byref(self.desc), nq, R, k, qmode)
        ws = self._ws.get("buf")
        if ws is None or ws.numel() < need:
            ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
            self._ws["buf"] = ws
        return ws


class IndexDescHolder:
    def __init__(self, ix: DeviceIndex):
        d = _lib.IndexDesc()
        d.corpus = ptr(ix.corpus)
        d.dtype = _lib.LMI_F16 if ix.storage == "f16" else _lib.LMI_F32
        d.d = ix.d
        d.d_pad = ix.d_pad
        d.n_rows = ix.n_rows
        d.inv_norm = ptr(ix.inv_norm)
        d.gpos = ptr(ix.gpos)
        d.n_buckets = ix.n_buckets
        d.bucket_off = ptr(ix.bucket_off_local)
        d.chunk_rows = ix.chunk_rows
        d.chunk_first = ptr(ix.chunk_first)
        d.n_chunks = ix.n_chunks
        d.max_chunks = ix.max_chunks
        d.chunk_centroid = ptr(ix.chunk_centroid) if ix.chunk_centroid is not None else None
        d.corpus64 = ptr(ix.corpus64) if ix.corpus64 is not None else None
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
    if out is None:
        out_d = torch.empty((nq, R, k), dtype=torch.float32, device=index.device)
        out_pos = torch.empty((nq, R, k), dtype=torch.int32, device=index.device)
        status = torch.zeros((1,), dtype=torch.int32, device=index.device)
    else:
        out_d, out_pos, status = out
    if ws is None:
        ws = index.workspace(nq, R, k, qmode)
    else:
        _workspace(ws, lib.lmi_scan_workspace_bytes(C.byref(index.desc), nq, R, k, qmode), "scan")
    s = stream if stream is not None else _lib.stream_handle(index.device)
    flags = (_lib.LMI_Q_SEED_ROUND0 if seed_round0 else 0) | phases
    check("lmi_bucket_topk", lib.lmi_bucket_topk(C.byref(index.desc), ptr(q), nq, q.stride(0),
                                                 ptr(classes), R, k, qmode | flags, ptr(out_d),
                                                 ptr(out_pos), ptr(status), ptr(ws), ws.numel(), s))
    return out_d, out_pos, status


def bucket_topk_f64(index: DeviceIndex, q: torch.Tensor, classes: torch.Tensor, k: int,
                    qmode: Optional[int] = None, eps: Optional[float] = None, stream=None,
                    fallback_count: bool = False, out=None, ws=None, seed_round0: bool = False,
                    phases: int = 0):
    """K2 with float64 distances (lmi_bucket_topk_f64): the reference's
    arithmetic when either operand is not float32 (utils.py:11, :19).  Returns
    (d f64 [nq,R,k], pos [nq,R,k] int32, status int32 tensor[, n_fallback]);
    `out` and `ws` as bucket_topk.  Float64 queries whose float32 rounding
    changes them are kept for the float64 recomputation (lmi_bucket_topk_f64q;
    the scan reads them rounded)."""
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
    need = lib.lmi_scan_f64_workspace_bytes(C.byref(index.desc), nq, R, k, qmode)
    if ws is None:
        ws = index._ws.get("f64")
        if ws is None or ws.numel() < need:
            ws = torch.empty(max(need, 256), dtype=torch.uint8, device=index.device)
            index._ws["f64"] = ws
    else:
        _workspace(ws, need, "float64 scan")
    s = stream if stream is not None else _lib.stream_handle(index.device)
    flags = (_lib.LMI_Q_SEED_ROUND0 if seed_round0 else 0) | phases
    check("lmi_bucket_topk_f64q", lib.lmi_bucket_topk_f64q(
        C.byref(index.desc), ptr(q), nq, q.stride(0), ptr(q64), 0 if q64 is None else q64.stride(0),
        ptr(classes), R, k, qmode | flags, float(eps), ptr(out_d), ptr(out_pos), ptr(status),
        ptr(ws), ws.numel(), s))
    if not fallback_count:
        return out_d, out_pos, status
    n = C.c_int32(0)
    check("lmi_refine_fallback_count", lib.lmi_refine_fallback_count(
        ptr(ws), C.byref(index.desc), nq, R, k, qmode, C.byref(n), s))
    return out_d, out_pos, status, int(n.value)


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
                  out=None):
    """A5 on the device (lmi_replay_device, or lmi_replay_device_f64 for
    float64 lists): same results as `replay`, device tensors in and out:
    (dists f64 [nq, w], anns uint32-as-int32 [nq, w], status); `out` = such a
    triple to write into (the status word zeroed by the caller)."""
    lib = _lib.load()
    dev = lists_d.device
    classes = _as_torch(classes, dev, torch.int32)
    if classes.dim() == 1:
        classes = classes[:, None].contiguous()
    nq, R = classes.shape
    f64 = lists_d.dtype == torch.float64
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
    ws = torch.empty(max(int(need), 256), dtype=torch.uint8, device=dev)
    thr = None
    if thr_round0 is not None:
        thr = _as_torch(thr_round0, dev, torch.float64).reshape(-1)
        if thr.numel() != nq:
            raise ValueError("threshold_dist must have one value per query")
    s = stream if stream is not None else _lib.stream_handle(dev)
    fn = "lmi_replay_device_f64" if f64 else "lmi_replay_device"
    check(fn, getattr(lib, fn)(
        ptr(classes), nq, R, k_list, ptr(lists_d), ptr(lists_pos), k_round, k_final,
        ptr(bucket_size), n_b, ptr(pos_to_id), int(pos_to_id.numel()), int(bool(use_threshold)),
        ptr(thr), ptr(dists), ptr(anns), ptr(status), ptr(ws), ws.numel(), s))
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

    def __init__(self, index: DeviceIndex, router: DeviceRouter, group=None):
        self.index = index
        self.router = router
        self.group = group
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
        if self.index.world == 1 and status_out is not None:
            nq, R = classes.shape
            dev = self.index.device
            out = (torch.empty((nq, R, k_list), dtype=torch.float64 if f64 else torch.float32,
                               device=dev),
                   torch.empty((nq, R, k_list), dtype=torch.int32, device=dev), status_out)
        if self.index.world > 1:
            # the lists and the status word land in this rank's slice of the
            # all-gather's packed send buffer (li.dist.packed_lists)
            from .dist import packed_lists
            nq, R = classes.shape
            buf, dv, pv, sv = packed_lists(nq * R, k_list, f64, self.index.device)
            out = (dv.view(nq, R, k_list), pv.view(nq, R, k_list), sv)
        if f64:
            d, pos, status = bucket_topk_f64(self.index, q_search, classes, k_list, qmode=qmode,
                                             out=out, ws=ws, seed_round0=seed_round0)
        else:
            d, pos, status = bucket_topk(self.index, q_search, classes, k_list, qmode=qmode, out=out,
                                         ws=ws, seed_round0=seed_round0)
        if lap:
            lap("scan")
        if self.index.world > 1:
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
        if self.index.world > 1:
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
        return StreamedSearch(self, q_nav, q_search, R, k, **kw)

    def graph(self, q_nav, q_search, R: int, k: int = 10, **kw) -> "GraphedSearch":
        """The step captured as a HIP graph (GraphedSearch), from the batch in
        host memory to the answer in host memory: same results as
        search(..., semantics="reference", replay_on="device")."""
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


def _host_array(x) -> np.ndarray:
    """A query batch (numpy, or a torch tensor on any device) as a host array."""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class GraphedSearch:
    """One search step captured once as a HIP graph and replayed per batch,
    from queries in HOST memory to the answer in host memory, as the
    reference's timer sees it (search.py:116-141; its queries are host arrays,
    search.py:49, :85-87):

        H2D of the staged batch (pinned host rows)
        -> router (K1) -> scan (K2) [-> all-gather + K3] -> replay (K4)
        -> D2H of the answer and of both status words

    The ~25 launches and the copies go to the GPU as one graph launch, with no
    host work between them.

    Staging (`stage`, outside the step, like the reference's h5 loads before
    its timer): the batch is written into a pinned host buffer laid out per
    rank block as [pca96 f32 (per x 96) | clip768 (per x d) | classes (per x
    R, G > 1 only)].  The clip768 rows are staged as fp16 when the index is
    fp16 and every query value is fp16-representable (checked on the host at
    staging; float16 input is exact by construction): half the bytes over
    PCIe, widened to float32 on the device.  A batch that is not fp16-exact
    under an fp16 capture is answered by the eager path instead.

    G > 1 ranks: rank g uploads only its block (1/G of the batch), routes its
    queries into the block's classes, and ONE all-gather over xGMI hands every
    rank the whole batch and all classes; then the striped scan and the list
    exchange as in Searcher.search.

    The graph owns its scan workspace (index._ws may be replaced by a later
    eager call with a bigger batch).  `run()` returns numpy views
    of the graph's pinned output buffer, valid until the next run."""

    def __init__(self, searcher: "Searcher", q_nav, q_search, R: int,
                 k: int = 10, *, k_round: int = 10, use_threshold: bool = True, dist: str = "f32",
                 capture: bool = True, pipeline: bool = False):
        s = searcher
        ix = s.index
        dev = ix.device
        lib = _lib.load()
        self.searcher, self.R, self.k, self.k_round = s, R, k, k_round
        self.use_threshold, self.dist = use_threshold, dist
        G = ix.world
        grouped = G > 1 and torch.distributed.is_initialized()
        if k_round > _lib.LMI_MAX_K or (capture and grouped and
                                       torch.distributed.get_backend(s.group) != "nccl"):
            raise ValueError("graph capture needs k_round <= 16 and RCCL collectives "
                             "(capture=False runs the same step eagerly, e.g. over gloo)")
        nav = _host_array(q_nav)
        qs = _host_array(q_search)
        nq, d, dn = int(qs.shape[0]), ix.d, int(nav.shape[1])
        if qs.shape != (nq, d) or nav.shape[0] != nq:
            raise ValueError("query shapes do not match the index")
        self.nq, self.d, self.dn = nq, d, dn
        # the batch's precision class is decided on the host, once per capture
        self.f16_up = ix.storage == "f16" and d % 2 == 0 and (
            qs.dtype == np.float16 or _np_fp16_exact(qs))
        self.qmode = _lib.LMI_Q_F16 if self.f16_up else _lib.LMI_Q_F32
        f64 = dist == "f64"
        # the batch is shared over the ranks of the process group (the index's
        # world is the stripe count; they differ only in a one-process
        # rehearsal of one stripe, tools/shard_step.py)
        Gi = G if grouped else 1
        G = torch.distributed.get_world_size(s.group) if Gi > 1 else 1
        g = torch.distributed.get_rank(s.group) if Gi > 1 else 0
        self.per = per = -(-nq // G)
        self.wq = wq = d // 2 if self.f16_up else d          # int32 words per staged row
        self.bw = bw = per * dn + per * wq + (per * R if G > 1 else 0)
        pin = torch.cuda.is_available()
        self.bw_all = bw
        self.h_blk = torch.zeros((G, bw), dtype=torch.int32, pin_memory=pin)
        if not self.stage(nav, qs):
            raise ValueError("staging failed")
        need = (lib.lmi_scan_f64_workspace_bytes if f64 else lib.lmi_scan_workspace_bytes)(
            C.byref(ix.desc), nq, R, k_round, self.qmode)
        self.ws = torch.empty(max(int(need), 256), dtype=torch.uint8, device=dev)
        # pipeline: two device copies of the staged block, each with its own
        # captured graph; run() uploads the next one on a copy stream while
        # the current graph runs (the upload leaves the graph)
        self.pipeline = bool(pipeline) and capture
        self.d_blks = [torch.empty((bw,), dtype=torch.int32, device=dev)
                       for _ in range(2 if self.pipeline else 1)]
        self.d_blk = self.d_blks[0]
        self.d_all = torch.empty((G, bw), dtype=torch.int32, device=dev) if G > 1 else None
        self.q32 = torch.empty((G * per, d), dtype=torch.float32, device=dev) \
            if (self.f16_up or G > 1) else None
        self.cls = torch.empty((G * per, R), dtype=torch.int32, device=dev) if G > 1 else None
        bsz, p2id = s._device_tables()
        self.w = k_round if R == 1 else k
        self.rank_in_group = g
        self.G = G
        # collectives inside a replayed graph are GPU work the process group's
        # watchdog does not track: run() bounds its own wait instead
        self.timeout_s = float(os.environ.get("LMI_DIST_TIMEOUT_S", "300"))
        copy_stream = torch.cuda.Stream(dev)

        def step(slot=0):
            ans = answer_buffer(nq, self.w, dev)
            main = torch.cuda.current_stream(dev)
            d_blk = self.d_blks[slot]
            if G == 1:
                if not self.pipeline:
                    # pca96 rows first; the clip768 rows come in on a second
                    # stream while the router runs
                    d_blk[:per * dn].copy_(self.h_blk[0, :per * dn], non_blocking=True)
                    copy_stream.wait_stream(main)
                    with torch.cuda.stream(copy_stream):
                        d_blk[per * dn:].copy_(self.h_blk[0, per * dn:], non_blocking=True)
                classes = s.router.topr(d_blk[:per * dn].view(torch.float32).view(per, dn), R)[0]
                if not self.pipeline:
                    main.wait_stream(copy_stream)
                sv = d_blk[per * dn:per * dn + per * wq]
                if self.f16_up:
                    q = self.q32
                    q.copy_(sv.view(torch.float16).view(per, d))
                else:
                    q = sv.view(torch.float32).view(per, d)
            else:
                # this rank's block: upload, route its queries into the block,
                # one all-gather of every block (queries + classes)
                from .dist import _all_gather
                if not self.pipeline:
                    d_blk.copy_(self.h_blk[g], non_blocking=True)
                s.router.topr(d_blk[:per * dn].view(torch.float32).view(per, dn), R,
                              out=d_blk[per * (dn + wq):])
                _all_gather(self.d_all.view(-1), d_blk, s.group)
                sv = self.d_all[:, per * dn:per * (dn + wq)]
                if self.f16_up:
                    self.q32.view(G, per, d).copy_(sv.view(torch.float16).view(G, per, d))
                else:
                    self.q32.view(G, per, d).copy_(sv.view(torch.float32).view(G, per, d))
                self.cls.view(G, per, R).copy_(self.d_all[:, per * (dn + wq):].view(G, per, R))
                q = self.q32[:nq]
                classes = self.cls[:nq]
            d_, pos, _ = s._scan(q, classes, k_round, self.qmode, f64, status_out=ans[3][0:1],
                                 ws=self.ws, seed_round0=use_threshold and k <= k_round and _SEED_ROUND0)
            replay_device(classes, d_, pos, k_round=k_round, k_final=k, bucket_size=bsz,
                          pos_to_id=p2id, use_threshold=use_threshold,
                          out=(ans[1], ans[2], ans[3][1:2]))
            return ans[0]

        # warm up on a side stream (allocations, kernel attributes, RCCL
        # communicators), then capture.  G > 1: the ranks agree that every
        # rank's warm-up succeeded before any rank captures (a rank that
        # raised before entering a collective would otherwise leave the others
        # waiting in the next one; a rank that fails inside a collective is
        # ended by the process group's timeout, li.dist.init_from_env)
        self._step = None
        if not capture:
            # the same step, launched eagerly per run (the multi-process gloo
            # rehearsal of the sharded upload on one GPU: tests/test_gpu_dist.py)
            buf = step()
            torch.cuda.synchronize(dev)
            self.h = torch.empty(tuple(buf.shape), dtype=torch.int32, pin_memory=True)
            self.graph = None
            self._step = step
            return
        self._cs = copy_stream
        if self.pipeline:
            self._up_ev = [torch.cuda.Event() for _ in range(2)]
            self._done_ev = [torch.cuda.Event() for _ in range(2)]
            for slot in range(2):
                self.d_blks[slot].copy_(self.h_blk[g], non_blocking=True)
            torch.cuda.synchronize(dev)
        slots = (0, 1) if self.pipeline else (0, 0)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        err = None
        try:
            with torch.cuda.stream(side):
                for slot in slots:
                    buf = step(slot)
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
        except Exception as e:  # noqa: BLE001 (re-raised below on every rank)
            err = e
        if Gi > 1:
            ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
            torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN, group=s.group)
            if int(ok.item()) == 0:
                raise RuntimeError(f"graph warm-up failed on some rank: {err!r}")
        elif err is not None:
            raise err
        # one pinned answer buffer per graph: with launch() / result() a graph
        # may run while the host reads the other's answer
        self.hs = [torch.empty(tuple(buf.shape), dtype=torch.int32, pin_memory=True)
                   for _ in range(2 if self.pipeline else 1)]
        self.h = self.hs[0]
        self.graphs, self._keep = [], []
        for slot in range(2 if self.pipeline else 1):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                buf = step(slot)
                self.hs[slot].copy_(buf, non_blocking=True)
            self.graphs.append(gr)
            self._keep.append(buf)
        self.graph = self.graphs[0]
        self._slot = 0
        self._fresh = [True, True]   # d_blks[slot] holds the staged batch
        torch.cuda.synchronize(dev)

    def stage(self, q_nav, q_search) -> bool:
        """Write a batch (host or device arrays of the captured shape) into the
        pinned staging buffer.  False if it cannot be staged in the captured
        precision (clip768 values not fp16-representable under an fp16
        capture): run() then answers it on the eager path."""
        nav = _host_array(q_nav).astype(np.float32, copy=False)
        qs = _host_array(q_search)
        nq, d, dn, per, wq = self.nq, self.d, self.dn, self.per, self.wq
        if nav.shape != (nq, dn) or qs.shape != (nq, d):
            raise ValueError("a staged batch must have the captured shape")
        if self.f16_up:
            if qs.dtype == np.float16:
                q16 = qs
            else:
                q32 = qs.astype(np.float32, copy=False)
                q16 = q32.astype(np.float16)
                if not np.array_equal(q16.astype(np.float32), q32):
                    return False
            src, sdt = q16, np.float16
        else:
            src, sdt = qs.astype(np.float32, copy=False), np.float32
        if getattr(self, "pipeline", False):
            # an upload from the pinned buffer may be in flight (run());
            # both device copies are stale from now on
            self._cs.synchronize()
            self._fresh = [False, False]
        blk = self.h_blk.numpy()
        for g in range(blk.shape[0]):
            lo, hi = min(nq, g * per), min(nq, (g + 1) * per)
            nv = blk[g, :per * dn].view(np.float32).reshape(per, dn)
            nv[:hi - lo] = nav[lo:hi]
            nv[hi - lo:] = 0
            sv = blk[g, per * dn:per * (dn + wq)].view(sdt).reshape(per, d)
            sv[:hi - lo] = src[lo:hi]
            sv[hi - lo:] = 0
        self._staged = (nav, qs)
        return True

    def upload_bytes(self) -> int:
        """Bytes this rank moves host -> device per step."""
        per, dn, wq = self.per, self.dn, self.wq
        return 4 * per * (dn + wq)

    def run(self, q_nav=None, q_search=None):
        """Replay the step (after staging a new batch, if given) -> (dists f64
        [nq, w], anns uint32 [nq, w])."""
        s = self.searcher
        dev = s.index.device
        if q_nav is not None or q_search is not None:
            if q_nav is None or q_search is None:
                raise ValueError("stage both q_nav and q_search")
            if not self.stage(q_nav, q_search):
                return self._eager(q_nav, q_search)
        if self.pipeline:
            return self.result(self.launch())
        elif self.graph is not None:
            self.graph.replay()
        else:
            self.h.copy_(self._step(), non_blocking=True)
        if self.G > 1 and self.graph is not None:
            _wait_with_deadline(dev, self.timeout_s)
        else:
            torch.cuda.current_stream(dev).synchronize()
        return self._answer(self.h)

    def _answer(self, h):
        hd, ha, st, rst = answer_views(h, self.nq, self.w)
        if st & _lib.LMI_STATUS_INTERNAL or rst:
            raise RuntimeError(f"search: internal status {st}/{rst}")
        return hd, ha

    def launch(self) -> int:
        """pipeline=True: enqueue one step on the staged batch without waiting
        for it (the next batch's upload starts beside it); returns a ticket for
        result().  Keeping one launch ahead of result() hides the host's
        synchronise-to-launch gap between steps (at most two in flight: a
        ticket's answer is valid until the launch after next)."""
        if not self.pipeline:
            raise ValueError("launch() needs GraphedSearch(pipeline=True)")
        slot = self._slot
        self._run_pipelined(self.searcher.index.device)
        return slot

    def result(self, ticket: int):
        """Wait for the step of `ticket` (from launch()) -> (dists f64 [nq, w],
        anns uint32 [nq, w]): numpy views of that step's pinned answer."""
        ev = self._done_ev[ticket]
        if self.G > 1:
            _wait_event_with_deadline(ev, self.timeout_s)
        else:
            ev.synchronize()
        return self._answer(self.hs[ticket])

    def _upload(self, slot):
        """The staged block into d_blks[slot] on the copy stream, once the
        graph that last read that copy has finished."""
        cs = self._cs
        cs.wait_event(self._done_ev[slot])
        with torch.cuda.stream(cs):
            self.d_blks[slot].copy_(self.h_blk[self.rank_in_group], non_blocking=True)
        self._up_ev[slot].record(cs)
        self._fresh[slot] = True

    def _run_pipelined(self, dev):
        """Replay the current slot's graph; meanwhile upload the staged batch
        into the other slot for the next run (a stream of batches: the copy
        engine moves batch i + 1 while batch i is searched)."""
        main = torch.cuda.current_stream(dev)
        slot = self._slot
        if not self._fresh[slot]:
            self._upload(slot)
        main.wait_event(self._up_ev[slot])
        self.graphs[slot].replay()
        self._done_ev[slot].record(main)
        self._fresh[slot] = False
        nxt = 1 - slot
        if not self._fresh[nxt]:
            self._upload(nxt)
        self._slot = nxt

    def _eager(self, q_nav, q_search):
        dev = self.searcher.index.device
        self.searcher._qcheck = None
        return self.searcher.search(_as_torch(_host_array(q_nav), dev, torch.float32),
                                    _as_torch(_host_array(q_search), dev, torch.float32),
                                    self.R, k=self.k, k_round=self.k_round,
                                    use_threshold=self.use_threshold, dist=self.dist)



class StreamedSearch:
    """A stream of query batches through the step as a four-stage pipeline
    ("The batch stream"):

        R  batch b+3: H2D of its staged host rows (copy engine) -> router (K1)
        P  batch b+3: the queries widened, K2's PLAN phase (fragments and
           norms, the tile plan, the seed map, the tail split, the bounds)
        S  batch b+1: K2's SCAN phase (of a batch planned two launches ago)
        F  batch b:   K2's MERGE phase (+ the float64 refinement)
           [-> all-gather + K3 at G > 1] -> replay (K4) -> D2H of the answer

    One launch (`step`) runs the four stages on five streams, each stage a
    captured graph per slot, ordered across launches by per-slot events, and
    returns the answer of the batch it finished.  The persistent scan holds
    every CU while it runs, so the latency-bound R, P and F chains start in
    its tail and run side by side; the next scan, enqueued ahead, waits for a
    plan done a launch earlier, so the scans run back to back.  Every
    batch passes every stage (the same kernels as Searcher.search), so each
    answer equals Searcher.search of its batch bit for bit; a launch answers
    the batch submitted three launches earlier.

    Four slots of per-batch device state (staged rows, classes, scan
    workspace, lists, answer) rotate over the launches: launch t routes and
    plans slot t mod 4, scans t+2 and finishes t+1 (mod 4).  A stage runs only
    on a slot whose earlier stages ran (the fill and drain run the same stage
    functions eagerly), so no kernel reads an unplanned workspace.

    G > 1: every rank uploads and routes the whole batch (no collective in R
    or P, both off the critical path); the one collective, the list exchange,
    runs in F as in Searcher.search.  fp16 index and fp16-exact query batches
    only (the phased scan is the fp16 scan); other batches go through
    GraphedSearch / Searcher.search."""

    NS = 4

    def __init__(self, searcher: "Searcher", q_nav, q_search, R: int, k: int = 10, *,
                 k_round: int = 10, use_threshold: bool = True, dist: str = "f32",
                 capture: bool = True, lookahead=None):
        s = searcher
        ix = s.index
        dev = ix.device
        lib = _lib.load()
        self.searcher, self.R, self.k, self.k_round = s, R, k, k_round
        self.use_threshold, self.dist = use_threshold, dist
        G = ix.world
        # the list exchange spans the process group's ranks (a stripe of a
        # G-way index in a process without a group: the rank's own lists)
        self.G = torch.distributed.get_world_size(s.group) if (
            G > 1 and torch.distributed.is_initialized()) else 1
        if k_round > _lib.LMI_MAX_K:
            raise ValueError("the phased scan needs k_round <= 16")
        if capture and self.G > 1 and torch.distributed.get_backend(s.group) != "nccl":
            raise ValueError("graph capture needs RCCL collectives (capture=False runs the "
                             "branches eagerly, e.g. over gloo)")
        nav, qs = _host_array(q_nav), _host_array(q_search)
        nq, d, dn = int(qs.shape[0]), ix.d, int(nav.shape[1])
        if qs.shape != (nq, d) or nav.shape[0] != nq:
            raise ValueError("query shapes do not match the index")
        if not (ix.storage == "f16" and d % 2 == 0):
            raise ValueError("the batch stream needs an fp16 index with an even d")
        self.nq, self.d, self.dn = nq, d, dn
        f64 = dist == "f64"
        self.w = k_round if R == 1 else k
        kl = k_round
        NS = self.NS
        self.bw = nq * dn + nq * (d // 2)
        pin = torch.cuda.is_available()
        self.h_stage = [torch.zeros((self.bw,), dtype=torch.int32, pin_memory=pin) for _ in range(NS)]
        self.d_blk = [torch.empty((self.bw,), dtype=torch.int32, device=dev) for _ in range(NS)]
        self.q32 = [torch.empty((nq, d), dtype=torch.float32, device=dev) for _ in range(NS)]
        self.cls = [torch.empty((nq, R), dtype=torch.int32, device=dev) for _ in range(NS)]
        wsb = (lib.lmi_scan_f64_workspace_bytes if f64 else lib.lmi_scan_workspace_bytes)(
            C.byref(ix.desc), nq, R, kl, _lib.LMI_Q_F16)
        self.ws = [torch.empty(max(int(wsb), 256), dtype=torch.uint8, device=dev) for _ in range(NS)]
        self.ans = [answer_buffer(nq, self.w, dev) for _ in range(NS)]
        self.h_ans = [torch.empty((3 * nq * self.w + 2,), dtype=torch.int32, pin_memory=pin)
                      for _ in range(NS)]
        ldt = torch.float64 if f64 else torch.float32
        if self.G > 1:
            from .dist import packed_lists
            self.pk = [packed_lists(nq * R, kl, f64, dev) for _ in range(NS)]
            self.lists = [(b[1].view(nq, R, kl), b[2].view(nq, R, kl), b[3]) for b in self.pk]
        else:
            self.pk = None
            self.lists = [(torch.empty((nq, R, kl), dtype=ldt, device=dev),
                           torch.empty((nq, R, kl), dtype=torch.int32, device=dev),
                           self.ans[j][3][0:1]) for j in range(NS)]
        bsz, p2id = s._device_tables()
        seed = use_threshold and k <= k_round and _SEED_ROUND0
        scan_fn = bucket_topk_f64 if f64 else bucket_topk
        self.timeout_s = float(os.environ.get("LMI_DIST_TIMEOUT_S", "300"))

        def phase(j, ph):
            dl, pl, st = self.lists[j]
            scan_fn(ix, self.q32[j], self.cls[j], kl, qmode=_lib.LMI_Q_F16, out=(dl, pl, st),
                    ws=self.ws[j], seed_round0=seed, phases=ph)

        def upload(j):
            self.d_blk[j].copy_(self.h_stage[j], non_blocking=True)

        def route(j):
            # (the staged rows are in d_blk[j]: upload(j) ran before, on the
            # copy stream in a launch)
            blk = self.d_blk[j]
            s.router.topr(blk[:nq * dn].view(torch.float32).view(nq, dn), R, out=self.cls[j])

        def plan(j):
            self.lists[j][2].zero_()
            self.q32[j].copy_(self.d_blk[j][nq * dn:].view(torch.float16).view(nq, d))
            phase(j, _lib.LMI_Q_PHASE_PLAN)

        def scan(j):
            phase(j, _lib.LMI_Q_PHASE_SCAN)

        def finish(j):
            phase(j, _lib.LMI_Q_PHASE_MERGE)
            buf, ad, aa, ast = self.ans[j]
            ast[1:2].zero_()
            if self.G > 1:
                from .dist import gather_merge_packed
                dd, pp, _ = gather_merge_packed(self.pk[j][0], nq * R, kl, f64, s.group,
                                                status_out=ast[0:1])
                dd, pp = dd.view(nq, R, kl), pp.view(nq, R, kl)
            else:
                dd, pp = self.lists[j][0], self.lists[j][1]
            replay_device(self.cls[j], dd, pp, k_round=k_round, k_final=k, bucket_size=bsz,
                          pos_to_id=p2id, use_threshold=use_threshold, out=(ad, aa, ast[1:2]))
            self.h_ans[j].copy_(buf, non_blocking=True)

        self._upload, self._route, self._plan, self._scan, self._finish = upload, route, plan, scan, finish
        # five streams: uploads (the copy engine), route, plan, scan (the
        # caller's stream), finish; per-slot events order them across launches
        self._cs = torch.cuda.Stream(dev)
        self._rs = torch.cuda.Stream(dev)
        self._ps = torch.cuda.Stream(dev)
        self._fs = torch.cuda.Stream(dev)
        ev = lambda: [torch.cuda.Event() for _ in range(NS)]
        self._up, self._rdone, self._pdone, self._sdone, self._fdone = ev(), ev(), ev(), ev(), ev()
        self.graphs = None
        self._t = None  # launch counter once primed
        # the next launch's scan enqueued ahead (its plan ran a launch
        # earlier), waiting on the device for this launch's finish
        # (lookahead="finish", the default): no host round trip before it, and
        # it does not take the CUs the route / plan / finish chains wait for.
        # Same box (profiles/r03_stream_lookahead3_ab.txt): one GPU 7.03-7.04 ms
        # per launch against 7.08-7.09 with the scan right behind the last one
        # (True) and 7.15-7.16 without lookahead (False); a stripe of 8
        # 1.25-1.26 / 1.23-1.24 / 1.26-1.27 (True was the slowest on another box)
        self.lookahead = "finish" if lookahead is None else lookahead
        self._s_ahead = False  # the next launch's scan is already enqueued
        if not self.stage(nav, qs):
            raise ValueError("the batch stream needs fp16-exact query batches")
        for j in range(NS):
            self.h_stage[j].copy_(self.h_stage[0])
        # warm-up: one eager pass of every branch on every slot (allocations,
        # kernel attributes, communicators), in pipeline order, on a side stream
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        err = None
        try:
            with torch.cuda.stream(side):
                for j in range(NS):
                    upload(j)
                    route(j)
                    plan(j)
                    scan(j)
                    finish(j)
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
        except Exception as e:  # noqa: BLE001 (re-raised below on every rank)
            err = e
        if self.G > 1:
            ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
            torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN, group=s.group)
            if int(ok.item()) == 0:
                raise RuntimeError(f"stream warm-up failed on some rank: {err!r}")
        elif err is not None:
            raise err
        if capture:
            # one graph per (stage, slot): route, plan, scan and finish each a chain
            self.graphs = {}
            for name, fn in (("R", route), ("P", plan), ("S", scan), ("F", finish)):
                for j in range(NS):
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr):
                        fn(j)
                    self.graphs[name, j] = gr
            torch.cuda.synchronize(dev)

    def stage(self, q_nav, q_search, slot: Optional[int] = None) -> bool:
        """Write a batch into the pinned staging rows of `slot` (default: the
        slot the next launch plans).  False if a clip768 value is not
        fp16-representable (the stream cannot take that batch)."""
        nav = _host_array(q_nav).astype(np.float32, copy=False)
        qs = _host_array(q_search)
        nq, d, dn = self.nq, self.d, self.dn
        if nav.shape != (nq, dn) or qs.shape != (nq, d):
            raise ValueError("a staged batch must have the stream's shape")
        if qs.dtype == np.float16:
            q16 = qs
        else:
            q32 = qs.astype(np.float32, copy=False)
            q16 = q32.astype(np.float16)
            if not np.array_equal(q16.astype(np.float32), q32):
                return False
        if slot is None:
            slot = (self._t or 0) % self.NS
        blk = self.h_stage[slot].numpy()
        blk[:nq * dn].view(np.float32).reshape(nq, dn)[:] = nav
        blk[nq * dn:].view(np.float16).reshape(nq, d)[:] = q16
        return True

    def prime(self):
        """Fill the pipeline with the staged rows of slots 1, 2 and 3 (eagerly:
        slot 1 up to its scan, slots 2 and 3 up to their plans): the next
        launch answers slot 1."""
        dev = self.searcher.index.device
        for j, upto in ((1, 3), (2, 2), (3, 2)):
            self._upload(j)
            for f in (self._route, self._plan, self._scan)[:upto]:
                f(j)
        torch.cuda.current_stream(dev).synchronize()
        self._t = 0
        self._s_ahead = False

    def _run(self, name, j):
        if self.graphs is not None:
            self.graphs[name, j].replay()
        else:
            {"R": self._route, "P": self._plan, "S": self._scan, "F": self._finish}[name](j)

    def step(self):
        """One launch -> (dists f64 [nq, w], anns uint32 [nq, w]) of the batch
        it finished (numpy views, valid for the next three launches).  Slot
        t mod 4 is uploaded and routed (stage() before step() streams a new
        batch; without it the slot's previous rows are used again) and
        planned, slot t + 2 scanned and t + 1 finished (mod 4), on five streams
        ordered by per-slot events:

            copy:   H2D of slot t                      (the copy engine)
            route:  wait H2D -> router (slot t)
            plan:   wait route -> widen, K2 PLAN (slot t)
            scan:   wait plan(two launches ago) -> K2 SCAN (slot t+2)
            finish: wait scan(last launch) -> merge [all-gather + K3],
                    replay, D2H (slot t+1)

        The scan holds every CU while it runs; the latency-bound chains start
        in its tail.  With `lookahead` the next launch's scan, of a slot
        planned a launch earlier, is enqueued too: right behind this scan
        (True), or (the default, "finish") behind this launch's finish on the
        device, without a host round trip."""
        if self._t is None:
            self.prime()
        dev = self.searcher.index.device
        NS = self.NS
        g = self._t % NS
        jr, js, jf = g, (g + 2) % NS, (g + 1) % NS
        main = torch.cuda.current_stream(dev)
        # (d_blk[jr] was last read by the plan three launches ago, which the
        # finish the host waited for in the last step depended on)
        with torch.cuda.stream(self._cs):
            self._upload(jr)
        self._up[jr].record(self._cs)
        if not self._s_ahead:
            main.wait_event(self._pdone[js])
            self._run("S", js)
            self._sdone[js].record(main)
        self._rs.wait_event(self._up[jr])
        with torch.cuda.stream(self._rs):
            self._run("R", jr)
        self._rdone[jr].record(self._rs)
        self._ps.wait_event(self._rdone[jr])
        with torch.cuda.stream(self._ps):
            self._run("P", jr)
        self._pdone[jr].record(self._ps)
        self._fs.wait_event(self._sdone[jf])
        with torch.cuda.stream(self._fs):
            self._run("F", jf)
        self._fdone[jf].record(self._fs)
        if self.lookahead:
            # the next launch's scan: slot t+3, planned in the last launch (in
            # the tail of its scan), so it follows this scan at once
            jn = (g + 3) % NS
            main.wait_event(self._pdone[jn])
            if self.lookahead == "finish":
                main.wait_event(self._fdone[jf])
            elif self.lookahead == "plan":  # (a study: gate on this launch's plan)
                main.wait_event(self._pdone[jr])
            self._run("S", jn)
            self._sdone[jn].record(main)
        self._s_ahead = bool(self.lookahead)
        self._t += 1
        if self.G > 1 and self.graphs is not None:
            _wait_event_with_deadline(self._fdone[jf], self.timeout_s)
        else:
            self._fdone[jf].synchronize()
        return self._answer(jf)

    def _answer(self, j):
        hd, ha, st, rst = answer_views(self.h_ans[j], self.nq, self.w)
        if st & (_lib.LMI_STATUS_INTERNAL | _lib.LMI_STATUS_QUERY_NOT_F16) or rst:
            raise RuntimeError(f"stream: status {st}/{rst}")
        return hd, ha

    def stream(self, batches):
        """Answer an iterable of (q_nav, q_search) batches in order, yielding
        (dists, anns) copies per batch: three batches fill the pipeline, then
        one launch per batch, then the last three finish eagerly."""
        dev = self.searcher.index.device
        NS = self.NS
        sync = lambda: torch.cuda.current_stream(dev).synchronize()
        ans = lambda j: tuple(a.copy() for a in self._answer(j))
        it = iter(batches)
        first = []
        for b in it:
            first.append(b)
            if len(first) == NS - 1:
                break
        for j, b in zip(range(1, NS), first):
            if not self.stage(*b, slot=j):
                raise ValueError("the batch stream needs fp16-exact query batches")
        if len(first) < NS - 1:
            for j in range(1, 1 + len(first)):
                self._upload(j); self._route(j); self._plan(j); self._scan(j); self._finish(j); sync()
                yield ans(j)
            return
        self.prime()
        for b in it:
            if not self.stage(*b, slot=self._t % NS):
                raise ValueError("the batch stream needs fp16-exact query batches")
            yield tuple(a.copy() for a in self.step())
        # drain: slot t+1 is scanned, t+2 and t+3 planned (mod 4; t+2's scan
        # enqueued when lookahead), t the launch count
        torch.cuda.synchronize(dev)  # (every stream of the last launch)
        t = self._t
        j1, j2, j3 = (t + 1) % NS, (t + 2) % NS, (t + 3) % NS
        self._finish(j1); sync()
        yield ans(j1)
        if not self._s_ahead:
            self._scan(j2)
        self._finish(j2); sync()
        yield ans(j2)
        self._scan(j3); self._finish(j3); sync()
        yield ans(j3)
        self._t = None
        self._s_ahead = False

def _wait_event_with_deadline(ev, timeout_s: float) -> None:
    """_wait_with_deadline on a recorded event."""
    deadline = time.monotonic() + timeout_s
    spins = 0
    while not ev.query():
        spins += 1
        if spins > 1000:
            if time.monotonic() > deadline:
                raise RuntimeError(f"search step not finished after {timeout_s:.0f} s: a peer rank "
                                   "stopped inside the step's collectives; end this process")
            time.sleep(1e-4)


def _wait_with_deadline(dev, timeout_s: float) -> None:
    """Wait for the current stream's work, raising after `timeout_s`: a graph
    replay whose all-gather waits for a rank that died never completes, and
    RCCL kernels captured in a graph are outside the process group's watchdog
    (li.dist.init_from_env).  The caller should end the process: the stalled
    kernels stay queued on the device until its context is torn down."""
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    deadline = time.monotonic() + timeout_s
    spins = 0
    while not ev.query():
        spins += 1
        if spins > 1000:
            if time.monotonic() > deadline:
                raise RuntimeError(f"search step not finished after {timeout_s:.0f} s: a peer rank "
                                   "stopped inside the step's collectives; end this process")
            time.sleep(1e-4)


def _np_fp16_exact(x: np.ndarray) -> bool:
    """True when every value of a host array round-trips through fp16."""
    x = np.asarray(x)
    if x.dtype == np.float16:
        return True
    x32 = x.astype(np.float32, copy=False)
    if x.dtype != np.float32 and not np.array_equal(x32.astype(x.dtype), x):
        return False
    return bool(np.array_equal(x32.astype(np.float16).astype(np.float32), x32))
