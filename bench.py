#!/usr/bin/env python3
"""LMI search hot path on MI355X: queries/s on a 10k-query batch (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W] [--scale 10M|300K|...]

One step = one search of the whole 10k-query batch exactly as the reference
times it (search.py:116-141): H2D of the query batch from pinned host memory
(the reference's queries are host arrays, search.py:49, :85-87) + router (K1)
+ per-(query, probe) bucket scan (K2) [+ RCCL all-gather + K3 merge for N > 1]
+ the replay of the reference's merge (K4) + D2H of the answer.  The corpus
index is resident in HBM before the timed region.  N > 1: one process per GPU,
started by torchrun or, without one, by this script itself (launch_ranks);
the corpus striped over the ranks; all ranks search the same batch (strong
scaling: value = nq / max-over-ranks step time, the RCCL all-gather inside).

Besides the JSON fields of the driver contract the line carries:
  roofline      K2 scan kernel: algorithmic bytes per launch / its average
                duration (HIP events on the launch stream, every timed step)
  cpu_baseline  the oracle restatement (oracle/lmi_oracle.py, "port") timed on
                a bounded sample of the same workload on this host's cores
  recall        recall@k of the returned ids against exact k-NN on a sample
  parity        the graph's first answer vs an eager step (bitwise), and the
                per-(query, probe) lists of sampled queries (rank 0's merged
                lists at N > 1) vs a float64 brute force (list_parity)
  h2d           the step's query upload alone (HIP events)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))

from li import _lib, synth  # noqa: E402
from li.dist import init_from_env  # noqa: E402
from li.index import DeviceIndex, DeviceRouter, RowSource, Searcher, default_chunk_rows  # noqa: E402

METRIC = "queries/sec @ recall≥90% on 10M clip768, 10k-query batch; % HBM roofline"
PUBLISHED_QPS_10M = 19.42  # README:17,30 — 514.91 s for 10k queries, EPYC 7532, 1 core
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
F16_PEAK_TFLOPS = 2500.0   # dense fp16 MFMA

SCALES = {"100M": 100_000_000, "10M": 10_000_000, "1M": 1_000_000, "300K": 300_000, "100K": 100_000}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def build_workload(args, device, rank, world):
    """Synthetic clip768/pca96 corpus + queries, a router fitted to k-means
    buckets, object labels = router argmax (LearnedIndex.py:240); deterministic."""
    n, C = SCALES[args.scale], args.n_buckets
    t0 = time.time()
    if args.scale == "100M":
        # configs[4]: random vectors, k-means buckets; the corpus is generated
        # chunk by chunk straight into each rank's shard (never whole in HBM)
        x, q, qn, layers, labels = synth.build_random_workload(n, args.nq, C, args.arch, device,
                                                               train_steps=args.train_steps)
        router = DeviceRouter(layers, device=device)
        torch.cuda.synchronize()
        log(f"[bench] workload n={n} (random, generated per chunk) in {time.time() - t0:.1f}s")
        t0 = time.time()
        index = DeviceIndex(x, labels, C, device=device, chunk_rows=args.chunk_rows, rank=rank,
                            world=world)
        torch.cuda.synchronize()
        log(f"[bench] index (rank {rank}/{world}, {index.n_rows} rows, {index.storage}) "
            f"in {time.time() - t0:.1f}s; bucket sizes min/median/max = "
            f"{index.bucket_size.min()}/{int(np.median(index.bucket_size))}/"
            f"{index.bucket_size.max()}")
        return x, q, qn, router, index, labels
    x, q, qn, xn, layers = synth.build_lmi_workload(n, args.nq, C, args.arch, device,
                                                    centres=args.centres,
                                                    train_steps=args.train_steps)
    router = DeviceRouter(layers, device=device)
    labels = router.argmax(xn)
    del xn
    if args.corpus == "f32":
        x, q = not_fp16(x, 11), not_fp16(q, 12)
    torch.cuda.synchronize()
    log(f"[bench] workload n={n} built in {time.time() - t0:.1f}s")
    t0 = time.time()
    index = DeviceIndex(x, labels, C, device=device, chunk_rows=args.chunk_rows, rank=rank,
                        world=world)
    torch.cuda.synchronize()
    log(f"[bench] index (rank {rank}/{world}, {index.n_rows} rows, {index.storage}) "
        f"in {time.time() - t0:.1f}s; bucket sizes min/median/max = "
        f"{index.bucket_size.min()}/{int(np.median(index.bucket_size))}/{index.bucket_size.max()}")
    return x, q, qn, router, index, labels


@torch.no_grad()
def not_fp16(x, seed, rel=2e-5, chunk=1 << 20):
    """--corpus f32: float32 values that are NOT fp16-exact (x (1 + rel N)),
    generated on x's device in chunks (a seeded torch generator per call):
    the split mode's workload (lmi_index_desc.corpus32)."""
    g = torch.Generator(device=x.device)
    g.manual_seed(seed)
    out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    for a in range(0, x.shape[0], chunk):
        blk = x[a:a + chunk].float()
        out[a:a + chunk] = blk * (1.0 + rel * torch.randn(blk.shape, generator=g, device=x.device))
    return out


@torch.no_grad()
def exact_knn(x, qs, k, chunk=1 << 20):
    """Exact cosine k-NN of the sample queries (ids 1-based, Baseline.py:17-19)."""
    qn = qs / qs.norm(dim=1, keepdim=True)
    best_s = torch.full((qs.shape[0], k), -2.0, device=qs.device)
    best_i = torch.zeros((qs.shape[0], k), dtype=torch.int64, device=qs.device)
    blocks = x.chunks() if isinstance(x, RowSource) else (
        (a, None, x[a:a + chunk]) for a in range(0, x.shape[0], chunk))
    for a, _, blk in blocks:
        blk = blk.float()
        s = qn @ (blk / blk.norm(dim=1, keepdim=True)).T
        v, i = s.topk(k, dim=1)
        cs = torch.cat([best_s, v], 1)
        ci = torch.cat([best_i, i + a], 1)
        o = cs.topk(k, dim=1).indices
        best_s, best_i = cs.gather(1, o), ci.gather(1, o)
    return (best_i + 1).cpu().numpy()


def algorithmic_bytes(index, classes, nq):
    """K2 per launch: every probed bucket's rows once (d_pad*s + 4 B of 1/||y||)
    + the queries as the scan reads them."""
    probed = np.unique(classes)
    loc = index.bucket_off_local.cpu().numpy()
    rows = int(sum(loc[c + 1] - loc[c] for c in probed))
    if index.storage == "f32x":
        # the split mode's two scans (lmi_scan.hip bucket_topk_x): the sample
        # scan over each probed bucket's first s_c = max(chunk_rows, n_c / 16)
        # rows, then the collect scan over the rest -- or over the whole bucket
        # where the sample is more than a quarter of it (x_sample_desc_kernel,
        # LMI_X_SKIP_SHARE), those sample rows read twice -- both streaming
        # the fp16 rounding
        n_c = np.array([loc[c + 1] - loc[c] for c in probed], dtype=np.int64)
        s_c = np.minimum(n_c, np.maximum(index.chunk_rows, (n_c // 16 + 31) // 32 * 32))
        share = int(os.environ.get("LMI_X_SKIP_SHARE", "4"))
        skipped = (share > 0) & (s_c < n_c) & (s_c * max(share, 1) <= n_c)
        rows += int(s_c[~skipped].sum())
    s = 4 if index.storage == "f32" else 2   # (f32x: its scans stream the fp16 rounding)
    byts = rows * (index.d_pad * s + 4) + nq * index.d_pad * s * (2 if index.storage == "f32x" else 1)
    sizes = np.diff(loc)
    flops = 2.0 * index.d * float(sizes[classes].sum())
    return byts, flops, rows


def cpu_baseline(index, q, classes, lists_d, args, budget_s=15.0):
    """The oracle port (oracle/lmi_oracle.py) on a bounded sample of the same
    batch, shaped like the reference's own loop (LearnedIndex.py:143-172):
    whole (round, bucket) groups drawn at random (seeded) from ALL R rounds,
    each: the gather of the bucket's rows (pandas .loc, :152-153/:168), then
    round 0: pairwise_cosine (sklearn normalize + GEMM, utils.py:10-11);
    rounds >= 1: pairwise_cosine_threshold (utils.py:14-43, its Python list
    comprehension over the relevant pairs included) against the running k-th
    distance of the earlier rounds (taken from the GPU's own lists); then the
    full-row argsort (:170).  Groups are timed until `budget_s` is spent; the
    rate is (query, probe) pairs / R per second, i.e. queries/s.  The
    reference itself, timed in the build container (tools/ref_cpu_baseline.py),
    is reported beside it from profiles/ref_cpu_*.json."""
    import glob
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import lmi_oracle as O
    off = index.layout.bucket_off
    qh = q.cpu().numpy()
    xh = (index.corpus32 if index.corpus32 is not None else index.corpus)[:, : index.d].cpu().numpy()
    R, k = args.R, args.k
    ld = lists_d.cpu().numpy().astype(np.float64)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    groups = [(r, int(c)) for r in range(R) for c in np.unique(classes[:, r])]
    rng = np.random.default_rng(0)
    groups = [groups[i] for i in rng.permutation(len(groups))]
    pairs = rows = ngroups = 0
    per_round = [0] * R
    el = 0.0
    for r, c in groups:
        a, b = int(off[c]), int(off[c + 1])
        G = np.nonzero(classes[:, r] == c)[0]
        if a == b or G.size == 0:
            continue
        thr = None
        if r > 0:  # running k-th distance after rounds < r (LearnedIndex.py:71-72)
            thr = np.full(qh.shape[0], np.inf)
            thr[G] = np.sort(ld[G, :r, :].reshape(G.size, -1), axis=1)[:, k - 1]
        t1 = time.time()
        y = xh[a:b].astype(np.float32)                      # the bucket gather
        if r == 0:
            D = O.pairwise_cosine(qh[G], y)
        else:
            D = O.pairwise_cosine_threshold(qh[G], y, thr, G, k)[0]
        if D is not None:
            np.argsort(D, axis=1, kind="quicksort")[:, :k]
        el += time.time() - t1
        ngroups += 1
        per_round[r] += 1
        pairs += G.size
        rows += b - a
        if el > budget_s:
            break
    out = {"value": round(pairs / R / el, 3), "unit": "queries/s", "cores": threads, "kind": "port",
           "sample": f"{ngroups} of the {len(groups)} (round, bucket) groups of the same {args.scale} "
                     f"batch, drawn at random from all rounds (per round {per_round}); "
                     f"{pairs} (query, probe) pairs over {rows} bucket rows, R={R}, k={k}: per group "
                     f"the bucket gather, sklearn-normalize + fp32 GEMM (round 0) or the threshold "
                     f"variant (rounds >= 1), full-row argsort, as LearnedIndex.py:143-172; "
                     f"rate = pairs / R / s; {threads} BLAS threads"}
    refs = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "ref_cpu_*.json"))):
        d = json.load(open(f))
        refs[os.path.basename(f)[:-5]] = {kk: d[kk] for kk in ("size", "R", "dtype", "threads", "qps",
                                                              "search_s", "nproc")}
    if refs:
        out["reference"] = {"kind": "reference", "unit": "queries/s",
                            "what": "the reference's own LearnedIndex.search timed as search.py:116-141 "
                                    "on the bench's synthetic workload in the build container "
                                    "(tools/ref_cpu_baseline.py; it cannot run on the GPU box)",
                            "runs": refs}
    return out


@torch.no_grad()
def list_parity(index, x, q, classes, lists_d, lists_pos, n_sample, f64, seed=5):
    """Parity of the per-(query, probe) lists the timed step is built on, on
    `n_sample` sampled queries: every list against an independent brute force
    over the same bucket rows -- torch float64 on the GPU, sklearn's arithmetic
    (rows and query normalised, then the dot, utils.py:11), full rows sorted
    by (distance, global position), first k (LearnedIndex.py:170-172).  At
    G > 1 these are rank 0's lists after the all-gather + K3 merge, and the
    rows come from the full corpus (every rank generated it), so the check
    covers the striped scan and the exchange.  Distances must agree within
    1e-5 (float32 lists; north_star) or 1e-12 (float64 lists); ids must be
    equal, except inside runs of distances tied within 1e-6 / 1e-12 (the
    reference's unstable argsort order there is unspecified):
    `tie_window_rows` counts the lists that needed that window."""
    nq, R, k = lists_d.shape
    atol, tie = (1e-12, 1e-12) if f64 else (1e-5, 1e-6)
    sample = np.sort(np.random.default_rng(seed).choice(nq, min(n_sample, nq), replace=False))
    ld = lists_d.double().cpu().numpy()[sample]
    lp = lists_pos.cpu().numpy()[sample]
    cls = np.asarray(classes)[sample]
    off = index.layout.bucket_off
    dev = index.device
    qs = q[torch.from_numpy(sample).to(q.device)].double().to(dev)
    qs = qs / torch.where(qs.norm(dim=1, keepdim=True) < 10 * 1.1920929e-07, 1.0,
                          qs.norm(dim=1, keepdim=True))
    full = index.world == 1
    if not full and not isinstance(x, torch.Tensor):
        return {"checked_lists": 0, "note": "corpus not materialised on rank 0 (RowSource)"}
    order = torch.from_numpy(index.layout.order)
    checked = bad = tie_rows = 0
    for c in np.unique(cls):
        a, b = int(off[c]), int(off[c + 1])
        if full:
            y = (index.corpus32 if index.corpus32 is not None else index.corpus)[a:b, :index.d]
        else:
            y = x[order[a:b].to(x.device)].to(dev)
        y = y.double()
        yn = y.norm(dim=1, keepdim=True)
        y = y / torch.where(yn < 10 * 1.1920929e-07, 1.0, yn)
        sel_q, sel_r = np.nonzero(cls == c)
        D = 1.0 - qs[torch.from_numpy(sel_q).to(dev)] @ y.T          # [pairs, N_c]
        o = torch.sort(D, dim=1, stable=True).indices[:, :k]       # (d, position) order
        rd = torch.gather(D, 1, o).cpu().numpy()
        rp = (o + a).cpu().numpy()
        Dh = D.cpu().numpy()
        for j, (i, r) in enumerate(zip(sel_q, sel_r)):
            kk = min(k, b - a)
            gd, gp = ld[i, r, :kk], lp[i, r, :kk]
            checked += 1
            ok = np.allclose(gd, rd[j, :kk], rtol=0, atol=atol) and bool(np.all(gp >= a)) and \
                bool(np.all(gp < b))
            used_tie = False
            if ok and not np.array_equal(gp, rp[j, :kk]):
                # ids differ: each must sit at its rank's distance within the tie window
                dd = Dh[j, gp - a]
                ok = bool(np.all(np.abs(dd - rd[j, :kk]) <= tie)) and len(set(gp)) == kk
                used_tie = ok
            if kk < k:
                ok = ok and bool(np.all(lp[i, r, kk:] < 0))
            bad += 0 if ok else 1
            tie_rows += 1 if used_tie else 0
    return {"checked_lists": int(checked), "queries": int(sample.size), "mismatches": int(bad),
            "tie_window_rows": int(tie_rows), "atol": atol, "tie": tie,
            "checker": "torch float64 brute force over the same bucket rows (bench.list_parity)"}


@torch.no_grad()
def h2d_ms(src, dst, reps=10):
    """The step's host -> device upload alone (a pinned staged block into its
    device copy), HIP events on the current stream: ms per copy and GB/s."""
    dst = torch.empty_like(dst)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dst.copy_(src, non_blocking=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    e1.record()
    torch.cuda.synchronize(dst.device)
    ms = e0.elapsed_time(e1) / reps
    return ms, src.numel() * src.element_size() / (ms * 1e-3) / 1e9


STEP_TEXT = {
    "stream": lambda a: ("batch stream (StreamedSearch): per launch, a new host batch staged into "
                         "pinned memory, then on five streams -- the H2D of that batch (copy engine) "
                         "and its router and plan, the scan of the batch of two launches before, the "
                         "chunk merge" + (" + one all-gather (lists + the next batch's query blocks) "
                                          "+ K3" if (a.gpus > 1 or os.environ.get("LMI_FORCE_EXCHANGE") == "1")
                                          else "") + " + replay + D2H of the "
                         "answer of the batch of three launches before (each a captured graph); every "
                         "batch passes every stage, each timed launch answers one batch"),
    "graph": lambda a: ("hip-graph replay per step (GraphedSearch.stream): each batch staged on the "
                        "host cores into its slot's pinned buffer and uploaded on a copy stream while "
                        "the previous batch's step runs, its step (router + search + replay + D2H of "
                        "the answer) enqueued behind it before the previous answer is read"
                        if not a.no_pipeline else
                        "hip-graph replay per step: a new host batch staged, then its H2D (inside the "
                        "step) + search + D2H of the answer"),
    "eager": lambda a: "eager launches (H2D of the host batch + search + D2H)",
}


def pmc_traffic(kernel_ms, split=False):
    """HBM-side bytes per scan launch from the committed rocprofv3 PMC passes
    (tools/gpu_profile.sh -> profiles/*pmc_traffic.json; the split mode's two
    scans per step: tools/pmc_split.sh -> profiles/*split_pmc_traffic.json):
    FETCH_SIZE x 2 (gfx950 reports half of wide streaming reads,
    MI355X_MICROARCH.md HBM section) + WRITE_SIZE, in bytes; None when no
    summary is committed."""
    import glob
    import re

    def session(f):
        # (rNN then the session letters a .. z, aa, ab, ...: the latest last)
        m = re.match(r"r(\d+)([a-z]*)", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2), f) if m else (0, 0, "", f)
    files = sorted((f for f in glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json"))
                    if ("split_pmc" in os.path.basename(f)) == split), key=session)
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    byts = (2.0 * d["FETCH_SIZE"]["mean_kb"] + d["WRITE_SIZE"]["mean_kb"]) * 1024.0
    return byts, os.path.relpath(files[-1], ROOT)


_ROCTX = []


def _roctx():
    """The ROCTx marker API (rocprofiler-sdk), for rocprofv3 --marker-trace to
    bracket the timed region (tools/timed_scans.py picks the scan launches
    inside it); None where the library is absent (the markers are then no-ops)."""
    if not _ROCTX:
        import ctypes
        try:
            lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
        except OSError:
            lib = None
        _ROCTX.append(lib)
    return _ROCTX[0]


def marker_push(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def marker_pop():
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePop()


def _gpus_arg(argv):
    from li.dist import gpus_arg
    return gpus_arg(argv)


def launch_ranks(n: int, argv, script: str = None) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes of
    this script (li.dist.launch_ranks: RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* in their env, one GPU each), relay rank 0's JSON line, and exit
    with the first failing rank's code (the other ranks are stopped: they
    would wait at a collective).  This process never initialises the GPU."""
    from li.dist import launch_ranks as _launch
    return _launch(n, argv, script or os.path.abspath(__file__), relay_stdout=True)


def main():
    if "WORLD_SIZE" not in os.environ and _gpus_arg(sys.argv[1:]) > 1:
        sys.exit(launch_ranks(_gpus_arg(sys.argv[1:]), sys.argv[1:]))
    # Libraries print banners to stdout (RCCL's version block at communicator
    # init): fd 1 goes to stderr for the run, and only the JSON line is written
    # to the original stdout.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scale", default="10M", choices=list(SCALES))
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--R", type=int, default=4)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n-buckets", type=int, default=122)
    ap.add_argument("--arch", default="MLP-5")
    ap.add_argument("--centres", type=int, default=400)
    ap.add_argument("--train-steps", type=int, default=200)
    ap.add_argument("--chunk-rows", type=int, default=None,
                    help="scan chunk (rows); default by GPU count: 8192 on 1, 4096 on 2-4, 2048 on "
                         "more (a shard's tiles must still fill 256 CUs; tools/gpu_shards.sh)")
    ap.add_argument("--recall-sample", type=int, default=200)
    ap.add_argument("--parity-sample", type=int, default=64,
                    help="queries whose lists are checked against a float64 brute force")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single", action="store_true",
                    help="skip the one-batch-at-a-time step graph (single_batch in the line)")
    ap.add_argument("--no-stream", action="store_true",
                    help="time the per-batch step graph (GraphedSearch, the upload pipelined on a "
                         "copy stream) instead of the batch stream (StreamedSearch, the default: the "
                         "H2D + plan of batch b+2, the scan of b+1 and the merge/replay/D2H of b per "
                         "launch on four streams; DESIGN.md §5)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one captured graph instead of two (GraphedSearch(pipeline=False)): each "
                         "batch staged and uploaded inside its step (the default stages batch i + 1 "
                         "and uploads it beside batch i's step, GraphedSearch.stream)")
    ap.add_argument("--no-graph", action="store_true",
                    help="time the eager step (every launch from the host) instead of the "
                         "HIP-graph replay of the captured step")
    ap.add_argument("--batches", type=int, default=4,
                    help="distinct 10k-query batches the timed loop rotates through (host "
                         "arrays, each staged into pinned memory inside the timed loop)")
    ap.add_argument("--corpus", default="f16", choices=["f16", "f32"],
                    help="f16: the synthetic clip768 values are fp16-exact (stored float32, as "
                         "clip768v2's float16 data widened); f32: float32 values that are NOT "
                         "fp16-exact (x (1 + 2e-5 N)): the split mode (storage f32x), timed with "
                         "the per-batch step graph (the batch stream is the fp16 scan's)")
    ap.add_argument("--dist", default="f32", choices=["f32", "f64"],
                    help="distance arithmetic of the headline line: f32 = the reference's on "
                         "float32 DataFrames (the synthetic corpus is float32 holding fp16-exact "
                         "values); f64 = its arithmetic on float16 data (sklearn promotes). The "
                         "other one is timed too and reported under 'other_dist'")
    args = ap.parse_args()

    rank, world, local = init_from_env()
    if args.chunk_rows is None:
        args.chunk_rows = default_chunk_rows(world, SCALES[args.scale])
    if world != args.gpus:
        log(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world} (set by the launcher); "
            f"using {world}")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    group = None
    x, q, qn, router, index, labels = build_workload(args, device, rank, world)
    searcher = Searcher(index, router, group)
    # distinct query batches of the same distribution, held as host arrays as
    # the reference's queries are (search.py:49, :85-87); batch 0 is (qn, q)
    qb = synth.query_batches(max(1, args.batches), args.nq, device,
                             kind="random" if args.scale == "100M" else "mixture",
                             centres=args.centres)
    if args.corpus == "f32":
        qb = [(q if i == 0 else not_fp16(b_q, 100 + i), b_qn) for i, (b_q, b_qn) in enumerate(qb)]
    host_batches = [(b_qn.cpu().numpy(), b_q.cpu().numpy()) for b_q, b_qn in qb]
    del qb

    lib = _lib.load()

    capture = world == 1 or torch.distributed.get_backend() == "nccl"
    use_graph = not args.no_graph and capture
    graph_failed = []
    stream_failed = []
    step_mode = {}
    # the batch starts in HOST memory, as the reference's (search.py:49,
    # :85-87); every timed step stages a new batch into pinned memory,
    # uploads it (H2D), searches and copies the answer back
    qn_h, q_h = host_batches[0]
    q16_exact = index.storage == "f16" and all(
        bool(np.array_equal(b.astype(np.float16).astype(np.float32), b)) for _, b in host_batches)
    # the batch stream takes fp16-exact batches on an fp16 index (the phased
    # scan), or float32 batches on the split mode's index (its phases, ABI 11);
    # over gloo (the multi-rank rehearsal on one GPU) its stages run eagerly
    # (gloo collectives cannot be captured)
    use_stream = not args.no_graph and not args.no_stream and (q16_exact or index.storage == "f32x")
    qn_pin = torch.from_numpy(qn_h).pin_memory()
    q_pin = torch.from_numpy(q_h.astype(np.float16) if q16_exact else q_h).pin_memory()
    checks = {}

    def eager_step(dist):
        qn_d = qn_pin.to(device, non_blocking=True)
        q_d = q_pin.to(device, non_blocking=True).float()
        return searcher.search(qn_d, q_d, args.R, k=args.k, use_threshold=True, dist=dist)

    def agree(flag):
        if world == 1:
            return bool(flag)
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device if capture else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
        return bool(t.item())

    def kernel_ms(dist):
        """The scan kernel's time per step: HIP events the library records on
        the launch stream around every timed launch, over K eager steps, summed
        per step (the split mode launches two scans a step; events recorded into
        a graph cannot be timed on ROCm; a kernel runs the same whichever way it
        is launched)."""
        lib.lmi_timing_read(None, 0)
        lib.lmi_timing_enable(1)
        for _ in range(args.steps):
            eager_step(dist)
        torch.cuda.synchronize()
        lib.lmi_timing_enable(0)
        cap = 4 * max(args.steps, 1)
        ms = (_lib.C.c_float * cap)()
        n_ev = lib.lmi_timing_read(ms, cap)
        return float(np.sum(list(ms)[:n_ev])) / args.steps if n_ev > 0 else float("nan")

    B = len(host_batches)
    scan_stats = {}
    q16_h = [b.astype(np.float16) for _, b in host_batches] if q16_exact else None

    def hb(i, dist):
        """Batch i as host arrays in the line's input type: float32 clip768 rows
        (the reference's float32 branch) or, for the float64 arithmetic, float16
        rows (its float64 branch comes from float16 data: the clip768 'emb')."""
        nav, qs = host_batches[i % B]
        return (nav, q16_h[i % B]) if (dist == "f64" and q16_h is not None) else (nav, qs)

    eager_ans = {}

    def eager_of(i, dist):
        """Searcher.search of batch i (the checker of every timed answer)."""
        key = (i % B, dist)
        if key not in eager_ans:
            nav, qs = host_batches[i % B]
            eager_ans[key] = searcher.search(torch.from_numpy(nav).to(device),
                                             torch.from_numpy(qs).to(device), args.R, k=args.k,
                                             use_threshold=True, dist=dist)
        return eager_ans[key]

    def check_answers(name, answers, dist):
        """Every timed answer against Searcher.search of its batch, bit for bit
        (all ranks take part: at G > 1 the eager searches have collectives)."""
        bad = 0
        for i, (d_, a_) in answers:
            e_d, e_a = eager_of(i, dist)
            bad += 0 if (np.array_equal(d_, e_d) and np.array_equal(a_, e_a)) else 1
        ok = agree(bad == 0)
        checks[name] = (f"{len(answers)} timed answers of {len(set(i for i, _ in answers))} distinct "
                        f"batches: bitwise equal to Searcher.search" if ok else f"DIFFER ({bad})")
        return ok

    def timed_graph(dist, pipeline=None, single=False):
        """The step captured once as a HIP graph (Searcher.graph) and replayed,
        a new host batch staged before every step (GraphedSearch.run(q_nav,
        q_search)): W untimed steps, then K steps bracketed by barrier +
        synchronize.  Before timing, the first replay's answer must equal an
        eager step's bit for bit on every rank, else the eager step is timed
        instead; after timing every answer is checked against its batch."""
        pipeline = (not args.no_pipeline) if pipeline is None else pipeline
        try:
            gs = searcher.graph(*hb(0, dist), args.R, k=args.k, dist=dist, pipeline=pipeline)
            ok = 1
        except Exception as e:  # noqa: BLE001 (reported in the JSON line)
            log(f"[bench] graph capture failed ({e!r}); timing eager launches")
            graph_failed.append(repr(e)[:200])
            gs, ok = None, 0
        if not agree(ok):
            if not graph_failed:
                graph_failed.append("capture failed on another rank")
            if gs is not None:
                gs.close()
            del gs
            return None if single else timed_eager(dist)
        g_d, g_a = (a.copy() for a in gs.run())
        e_d, e_a = eager_of(0, dist)
        same = agree(np.array_equal(g_d, e_d) and np.array_equal(g_a, e_a))
        checks[f"{'single_' if single else ''}graph_vs_eager_{dist}"] = \
            "bitwise equal" if same else "DIFFER"
        if not same:
            log(f"[bench] graph replay differs from the eager step ({dist}); timing eager launches")
            graph_failed.append("first replay differs from the eager step")
            gs.close()
            del gs
            return None if single else timed_eager(dist)
        h2d = h2d_ms(gs.h_blk[gs.rank_in_group], gs.d_blk) + (gs.upload_bytes(),)
        answers = []

        def steps(i0, n, keep):
            # pipelined (the default): batch i + 1 staged and uploaded while
            # batch i's step runs (GraphedSearch.stream); single: one batch at a time
            if gs.pipeline and not single:
                for j, o in enumerate(gs.stream(hb(i, dist) for i in range(i0, i0 + n))):
                    if keep:
                        answers.append(((i0 + j) % B, o))
                return
            for i in range(i0, i0 + n):
                o = gs.run(*hb(i, dist))
                if keep:
                    answers.append((i % B, (o[0].copy(), o[1].copy())))

        steps(1, args.warmup, False)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        marker_push(f"bench timed {'single ' if single else ''}graph {dist}")
        t0 = time.perf_counter()
        steps(1 + args.warmup, args.steps, True)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        marker_pop()
        gs.close()
        del gs
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=device)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        check_answers(f"{'single_' if single else ''}graph_answers_{dist}", answers, dist)
        if single:
            return el
        step_mode[dist] = "graph"
        return el, kernel_ms(dist), answer_of_batch0(answers, dist), h2d

    def answer_of_batch0(answers, dist):
        for i, o in answers:
            if i == 0:
                return o
        return eager_of(0, dist)

    def timed_stream(dist):
        """The step as a stream of batches (Searcher.streamed -> StreamedSearch):
        launch t stages batch t mod B (host arrays -> this rank's pinned block)
        and runs one launch -- the H2D, router and plan of that batch, the scan
        of the batch of launch t-2, the merge / replay / D2H of the batch of
        launch t-3 -- and the host copies the answer out.  Before timing, the
        first launch's answer must equal an eager step's bit for bit on every
        rank, else the per-batch step graph is timed instead; after timing every
        timed answer is checked against Searcher.search of its batch."""
        try:
            ss = searcher.streamed(*hb(0, dist), args.R, k=args.k, dist=dist, capture=capture)
            ok = 1
        except Exception as e:  # noqa: BLE001 (reported in the JSON line)
            log(f"[bench] batch stream failed ({e!r}); timing the step graph")
            stream_failed.append(repr(e)[:200])
            ss, ok = None, 0
        if not agree(ok):
            if not stream_failed:
                stream_failed.append("stream set-up failed on another rank")
            if ss is not None:
                ss.close()
            del ss
            return timed_graph(dist) if use_graph else timed_eager(dist)
        staged = []   # batch index staged at launch t (all slots hold batch 0 at set-up)

        def launch(t):
            i = t % B
            ss.stage(*hb(i, dist))
            staged.append(i)
            o = ss.step()
            return (staged[t - 3] if t >= 3 else 0), o

        i0, (s_d, s_a) = launch(0)
        e_d, e_a = eager_of(i0, dist)
        same = agree(np.array_equal(s_d, e_d) and np.array_equal(s_a, e_a))
        checks[f"stream_vs_eager_{dist}"] = "bitwise equal" if same else "DIFFER"
        if not same:
            log(f"[bench] batch stream differs from the eager step ({dist}); timing the step graph")
            stream_failed.append("stream answer differs from the eager step")
            ss.close()
            del ss
            return timed_graph(dist) if use_graph else timed_eager(dist)
        h2d = h2d_ms(ss.h_stage[0][:ss.staged_words], ss.d_blk[0][:ss.staged_words]) + \
            (ss.upload_bytes(),)
        for t in range(1, 1 + args.warmup):
            launch(t)
        answers = []
        ss.time_scans = True   # HIP events around each scan graph on its stream
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        marker_push(f"bench timed stream {dist}")
        t0 = time.perf_counter()
        for t in range(1 + args.warmup, 1 + args.warmup + args.steps):
            i, o = launch(t)
            answers.append((i, (o[0].copy(), o[1].copy())))
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        marker_pop()
        scans = ss.scan_ms()
        ss.close()
        del ss
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=device if capture else "cpu")
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        check_answers(f"stream_answers_{dist}", answers, dist)
        step_mode[dist] = "stream" if capture else "stream (stages launched eagerly: gloo)"
        scan_stats[dist] = {"timed_scans": len(scans), "mean_ms": round(float(np.mean(scans)), 4),
                            "median_ms": round(float(np.median(scans)), 4),
                            "min_ms": round(float(np.min(scans)), 4),
                            "max_ms": round(float(np.max(scans)), 4),
                            "how": "HIP events on the scan's stream around each scan graph the "
                                   "timed launches enqueued"} if scans else None
        return el, (float(np.mean(scans)) if scans else kernel_ms(dist)), \
            answer_of_batch0(answers, dist), h2d

    def timed(dist):
        """W untimed warmup steps, then K steps bracketed by barrier +
        synchronize; returns (max-over-ranks seconds, mean scan-kernel ms,
        the last step's output, (H2D ms, GB/s, bytes) or None)."""
        if use_stream:
            return timed_stream(dist)
        if use_graph:
            return timed_graph(dist)
        return timed_eager(dist)

    def timed_eager(dist):
        out = None
        for _ in range(args.warmup):
            out = eager_step(dist)
        lib.lmi_timing_read(None, 0)  # drop warmup records
        lib.lmi_timing_enable(1)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = eager_step(dist)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        lib.lmi_timing_enable(0)
        # (a step may launch more than one scan -- the split mode's sample /
        # bound scan and its collect scan --: the scan time per step is the
        # sum of its launches)
        cap = 4 * max(args.steps, 1)
        ms = (_lib.C.c_float * cap)()
        n_ev = lib.lmi_timing_read(ms, cap)
        kms = float(np.sum(list(ms)[:n_ev])) / args.steps if n_ev > 0 else float("nan")
        if n_ev > args.steps:
            scan_stats[dist] = (f"HIP events around every scan launch over K eager steps (lmi_timing): "
                                f"{n_ev / args.steps:g} launches per step, summed per step")
        step_mode[dist] = "eager"
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64,
                             device=device if torch.distributed.get_backend() == "nccl" else "cpu")
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        return el, kms, out, None

    el, scan_ms, (dists, anns), h2d = timed(args.dist)
    ms_step = el / args.steps * 1e3
    # submission to answer: a streamed batch is answered by the fourth launch
    # that sees it (route, plan, scan, merge/replay), a graph-step batch by its own
    lat_ms = ms_step * (4 if step_mode.get(args.dist, "").startswith("stream") else
                        2 if step_mode.get(args.dist) == "graph" and not args.no_pipeline else 1)
    value = args.nq / (el / args.steps)
    # the other arithmetic, timed the same way (float64: the reference's on
    # float16 data, e.g. the real clip768 'emb'; float32: on float32 data)
    other = "f64" if args.dist == "f32" else "f32"
    el_o, scan_ms_o, (dists_o, anns_o), _ = timed(other)
    # one batch at a time, as the reference's timer sees it (search.py:116-141):
    # the per-batch step graph with the upload inside the step -- H2D of a new
    # host batch, search, D2H of its answer -- nothing of another batch beside it
    single = None
    if use_graph and not args.no_single:
        el_1 = timed_graph(args.dist, pipeline=False, single=True)
        if el_1 is not None:
            single = {"qps": round(args.nq / (el_1 / args.steps), 1),
                      "ms": round(el_1 / args.steps * 1e3, 3),
                      "step": "hip-graph replay per batch: stage a new host batch, H2D + router + "
                              "scan + merge + replay + D2H of its answer, wait; no overlap between "
                              "batches"}

    # per-stage breakdown (separate, synchronised passes; not the timed loop)
    tm = {}
    searcher.search(qn, q, args.R, k=args.k, use_threshold=True, dist=args.dist)  # pinned buffers
    for _ in range(3):
        searcher.search(qn, q, args.R, k=args.k, use_threshold=True, timings=tm, dist=args.dist)
    breakdown = {kk: round(v / 3, 3) for kk, v in tm.items()}
    if h2d is not None:
        breakdown = {"h2d": round(h2d[0], 3), **breakdown}
    # the optional exact-top-k semantics over the same probed buckets (untimed;
    # every rank takes part: with G > 1 the search has collectives)
    _, anns_x = searcher.search(qn, q, args.R, k=args.k, semantics="exact")
    classes, _ = router.topr(qn, args.R)
    classes = classes.cpu().numpy()
    byts, flops, rows = algorithmic_bytes(index, classes, args.nq)
    # parity of the lists the step is built on (all ranks take part in the
    # exchange; rank 0 checks), both arithmetics
    lists = {}
    for dd in (args.dist, other):
        _, l_d, l_p, l_st = searcher.lists(qn, q, args.R, args.k, dist=dd)
        lists[dd] = (l_d, l_p, int(l_st.item()))
    if rank != 0:
        if world > 1:
            torch.distributed.barrier()
        return
    achieved = byts / (scan_ms * 1e-3) / 1e9
    tflops = flops / (scan_ms * 1e-3) / 1e12
    # the committed PMC passes profile the default (10M, 1 GPU) command only
    traffic, traffic_src = pmc_traffic(scan_ms, split=index.storage == "f32x") \
        if (args.scale == "10M" and world == 1) else (None, None)
    # `bound` is the roof the kernel's arithmetic intensity selects: flops /
    # algorithmic bytes (401 flop/B at configs[2]) above the dense-fp16 ridge
    # (2.5 PF / 8 TB/s = 312 flop/B) means MFMA-bound, and achieved / peak /
    # frac are then flops against the dense fp16 peak.  north_star states its
    # target as a fraction of the HBM roofline: that fraction rides beside as
    # hbm_frac (algorithmic bytes / kernel time / 8 TB/s) whichever roof binds.
    ai = flops / byts
    mfma_roof = ai > F16_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
    if mfma_roof:
        head = {"bound": "mfma", "achieved": round(tflops, 1), "peak": F16_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(tflops / F16_PEAK_TFLOPS, 4)}
    else:
        head = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4)}
    roof = {**head,
            "traffic": None if traffic is None else int(traffic),
            "traffic_source": traffic_src,
            "kernel": "scan3_kernel (lmi_bucket_topk)", "kernel_ms": round(scan_ms, 4),
            "kernel_ms_source": scan_stats.get(args.dist) or
                                "HIP events around every scan launch over K eager steps (lmi_timing), summed per step",
            "arithmetic_intensity_flop_per_byte": round(ai, 1),
            "ridge_flop_per_byte": round(F16_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9), 1),
            "algorithmic_bytes": int(byts), "flops": flops,
            "hbm_gbs": round(achieved, 1), "hbm_frac": round(achieved / HBM_PEAK_GBS, 4),
            "hbm_target_note": "north_star's target is >= 0.50 of the HBM roofline (hbm_frac)",
            "mfma_tflops": round(tflops, 1), "mfma_frac": round(tflops / F16_PEAK_TFLOPS, 4)}
    sample = min(args.recall_sample, args.nq)
    truth = exact_knn(x, q[:sample], args.k)
    recall = float(np.mean([len(set(anns[i][: args.k]) & set(truth[i])) / args.k
                            for i in range(sample)]))
    recall_x = float(np.mean([len(set(anns_x[i][: args.k]) & set(truth[i])) / args.k
                              for i in range(sample)]))
    parity = dict(checks)
    for dd, (l_d, l_p, l_st) in lists.items():
        parity[f"lists_{dd}"] = list_parity(index, x, q, classes, l_d, l_p, args.parity_sample,
                                            dd == "f64")
        parity[f"lists_{dd}"]["status"] = l_st
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(index, q, classes, lists[args.dist][0], args)
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "queries/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
        "higher_is_better": True, "scaling": "strong",
        "vs_baseline": round(value / PUBLISHED_QPS_10M, 1) if args.scale == "10M" else None,
        "dtype": ("f16" if args.dist == "f32" else "f16+f64") if args.corpus == "f16" else
                 ("f16 scan + f64 re-score" if args.dist == "f32" else "f16 scan + f64"), "data": "synthetic",
        "config": {"workload": f"{args.scale} {'random unit (configs[4])' if args.scale == '100M' else 'clip768-like'} synthetic ({'fp16-exact' if args.corpus == 'f16' else 'float32, not fp16-exact: split mode'}), {args.n_buckets} "
                               f"buckets, R={args.R}, k={args.k}, {args.nq} queries, router "
                               f"{args.arch}", "n": SCALES[args.scale], "d": 768, "nq": args.nq,
                   "R": args.R, "k": args.k, "n_buckets": args.n_buckets, "router": args.arch,
                   "parallelism": f"corpus striped over {world} GPU(s)",
                   "chunk_rows": args.chunk_rows},
        "roofline": roof, "cpu_baseline": cpu,
        "recall": round(recall, 4), "recall_exact_semantics": round(recall_x, 4),
        "recall_sample": sample, "breakdown_ms": breakdown, "parity": parity,
        "h2d": None if h2d is None else {"ms": round(h2d[0], 4), "gb_s": round(h2d[1], 1),
                                         "bytes_per_rank": int(h2d[2]),
                                         "queries_staged_as": "f16" if q16_exact else "f32",
                                         "in_step": True,
                                         "overlapped": step_mode.get(args.dist, "").startswith("stream") or (
                                             step_mode.get(args.dist) == "graph" and not args.no_pipeline)},
        "dist": args.dist,
        "list_exchange": ("RCCL all-gather of the packed lists + K3 over a "
                          f"{world}-rank group" + (" (LMI_FORCE_EXCHANGE=1: the G > 1 branch on "
                                                   "one GPU)" if world == 1 else "")
                          if searcher.exchange else None),
        "step": STEP_TEXT[step_mode.get(args.dist, "eager").split(" ")[0]](args) +
                step_mode.get(args.dist, "eager")[len(step_mode.get(args.dist, "eager").split(" ")[0]):] +
                (f" (batch stream not used: {stream_failed[0]})" if stream_failed and use_stream else "") +
                (f" (graph not used: {graph_failed[0]})" if graph_failed else ""),
        "latency_ms_per_batch": round(lat_ms, 3) if lat_ms is not None else None,
        "single_batch": single,
        "batches": {"distinct": B, "held_as": "host numpy arrays (float32 rows; float16 for the "
                                             "float64 arithmetic)",
                    "staged": "every timed step stages a new batch (lmi_host_stage_f16 on the "
                              "host cores into pinned memory) inside the timed region"},
        "other_dist": {"dist": other, "value": round(args.nq / (el_o / args.steps), 1),
                       "ms_per_step": round(el_o / args.steps * 1e3, 3),
                       "scan_kernel_ms": round(scan_ms_o, 4),
                       "recall": round(float(np.mean([len(set(anns_o[i][: args.k]) & set(truth[i])) /
                                                      args.k for i in range(sample)])), 4)},
    }
    os.write(json_fd, (json.dumps(out) + "\n").encode())
    if world > 1:
        torch.distributed.barrier()


if __name__ == "__main__":
    main()
