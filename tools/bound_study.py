"""Study: how much of a stripe's scan the per-rank bound
costs.  Rank g of a G-way striped index keeps the top-10 of ITS stripe for
every pair, so its bound is its stripe's 10th distance, not the all-rank one.
Upper bound of what a cross-rank bound could save: seed every pair's bound
(thr_g) with the FINAL all-rank 10th distance before the SCAN phase
(lmi_debug_seed_bounds, the diagnostic library) and time the stripe's scan.

    LMI_LIB_NAME=liblmi_hip_abl.so python tools/bound_study.py [--world 8 --rank 0]

Prints per variant the scan kernel's median / min ms (lmi_timing HIP events)
and, with the ABL 7 counters, the candidates and insertion counts per launch.
Checks that the seeded stripe lists hold every entry of the unseeded ones at
or under the all-rank bound (so the merged lists are the same)."""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from li import _lib, synth  # noqa: E402
from li.index import DeviceIndex, DeviceRouter, bucket_topk, default_chunk_rows  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--nq", type=int, default=10_000)
ap.add_argument("--R", type=int, default=4)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--reps", type=int, default=7)
ap.add_argument("--abl7", action="store_true", help="also the ABL 7 counters (candidates)")
ap.add_argument("--sampled", action="store_true",
                help="VERDICT r5 item 3: the sampled-MIN scheme -- every stripe scans the first "
                     "chunk of each of its buckets (a pre-scan), the per-pair MIN of their 10ths "
                     "(what one all_reduce(MIN) of nq*R words gives) seeds the scan of the rest "
                     "of rank --rank's stripe; timed against the same rest unseeded and seeded "
                     "with the final all-rank 10th, plus the pre-scan itself")
a = ap.parse_args()

lib = _lib.load()
assert hasattr(lib, "lmi_debug_seed_bounds"), "needs LMI_LIB_NAME=liblmi_hip_abl.so (make ablation)"
lib.lmi_debug_seed_bounds.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                      C.c_void_p, C.c_void_p, C.c_void_p]
dev = torch.device("cuda")
x, q, qn, xn, layers = synth.build_lmi_workload(a.n, a.nq, 122, "MLP-5", dev)
router = DeviceRouter(layers)
labels = router.argmax(xn)
del xn
classes, _ = router.topr(qn, a.R)
# the all-rank lists (one GPU, the whole corpus): their 10th distance per pair
full = DeviceIndex(x, labels, 122, chunk_rows=8192)
gd, gp, _ = bucket_topk(full, q, classes, 10)
kth = gd[:, :, 9].contiguous().float().cpu().numpy()
del full, gd, gp
torch.cuda.empty_cache()
b = kth.view(np.uint32)
ordv = np.where(b & 0x80000000, ~b, b | 0x80000000).astype(np.uint32)   # f2ord
seed = torch.from_numpy(ordv.reshape(-1)).to(dev)
ix = DeviceIndex(x, labels, 122, chunk_rows=default_chunk_rows(a.world), rank=a.rank, world=a.world)
if not a.sampled:
    del x
    torch.cuda.empty_cache()
qmode = _lib.LMI_Q_F16
ws = ix.workspace(a.nq, a.R, 10, qmode)
s = _lib.stream_handle(dev)
P = a.nq * a.R


def run(seeded):
    if not seeded:
        return bucket_topk(ix, q, classes, 10, qmode=qmode, ws=ws)
    out = (torch.empty((a.nq, a.R, 10), dtype=torch.float32, device=dev),
           torch.empty((a.nq, a.R, 10), dtype=torch.int32, device=dev),
           torch.zeros((1,), dtype=torch.int32, device=dev))
    bucket_topk(ix, q, classes, 10, qmode=qmode, ws=ws, out=out, phases=_lib.LMI_Q_PHASE_PLAN)
    _lib.check("lmi_debug_seed_bounds", lib.lmi_debug_seed_bounds(
        C.byref(ix.desc), a.nq, a.R, 10, qmode, seed.data_ptr(), ws.data_ptr(), s))
    bucket_topk(ix, q, classes, 10, qmode=qmode, ws=ws, out=out, phases=_lib.LMI_Q_PHASE_SCAN)
    bucket_topk(ix, q, classes, 10, qmode=qmode, ws=ws, out=out, phases=_lib.LMI_Q_PHASE_MERGE)
    return out


def timed(seeded, abl="0"):
    os.environ["LMI_SCAN_ABL"] = abl
    lib.lmi_config_reload()
    for _ in range(2):
        run(seeded)
    torch.cuda.synchronize()
    cnt = (C.c_ulonglong * 16)()
    lib.lmi_debug_counters(cnt)
    lib.lmi_timing_read(None, 0)
    lib.lmi_timing_enable(1)
    for _ in range(a.reps):
        run(seeded)
    torch.cuda.synchronize()
    lib.lmi_timing_enable(0)
    ms = (C.c_float * a.reps)()
    n = lib.lmi_timing_read(ms, a.reps)
    v = sorted(list(ms)[:n])
    lib.lmi_debug_counters(cnt)
    line = f"world {a.world} rank {a.rank} {'seeded (all-rank 10th)' if seeded else 'own bound':24s} " \
           f"abl={abl} scan ms median {v[len(v) // 2]:.3f} min {v[0]:.3f}"
    if cnt[9]:
        line += f" | clock {cnt[8] / cnt[9] * 0.1:.2f} GHz"
    if abl == "7":
        names = ["wave-events", "candidates", "appends", "sorted-inserts", "fills", "wave-blocks"]
        line += " | " + ", ".join(f"{nm}={cnt[i] / a.reps:.4g}" for i, nm in enumerate(names))
    print(line, flush=True)


def f2ord(v):
    b = np.ascontiguousarray(v, dtype=np.float32).view(np.uint32)
    return torch.from_numpy(np.where(b & 0x80000000, ~b, b | 0x80000000).astype(np.uint32).reshape(-1)).to(dev)


def scan_ms(ixx, seed_ord=None, abl="0", reps=None):
    """Median / min ms of the scan kernel on index ixx (seeded with the
    ordinal bounds `seed_ord` when given), and the ABL 7 candidates."""
    reps = reps or a.reps
    os.environ["LMI_SCAN_ABL"] = abl
    lib.lmi_config_reload()
    wsx = ixx.workspace(a.nq, a.R, 10, qmode)
    out = (torch.empty((a.nq, a.R, 10), dtype=torch.float32, device=dev),
           torch.empty((a.nq, a.R, 10), dtype=torch.int32, device=dev),
           torch.zeros((1,), dtype=torch.int32, device=dev))

    def one():
        if seed_ord is None:
            return bucket_topk(ixx, q, classes, 10, qmode=qmode, ws=wsx, out=out)
        bucket_topk(ixx, q, classes, 10, qmode=qmode, ws=wsx, out=out, phases=_lib.LMI_Q_PHASE_PLAN)
        _lib.check("lmi_debug_seed_bounds", lib.lmi_debug_seed_bounds(
            C.byref(ixx.desc), a.nq, a.R, 10, qmode, seed_ord.data_ptr(), wsx.data_ptr(), s))
        bucket_topk(ixx, q, classes, 10, qmode=qmode, ws=wsx, out=out, phases=_lib.LMI_Q_PHASE_SCAN)
        return bucket_topk(ixx, q, classes, 10, qmode=qmode, ws=wsx, out=out, phases=_lib.LMI_Q_PHASE_MERGE)
    for _ in range(2):
        one()
    torch.cuda.synchronize()
    cnt = (C.c_ulonglong * 16)()
    lib.lmi_debug_counters(cnt)
    lib.lmi_timing_read(None, 0)
    lib.lmi_timing_enable(1)
    for _ in range(reps):
        one()
    torch.cuda.synchronize()
    lib.lmi_timing_enable(0)
    ms = (C.c_float * reps)()
    n = lib.lmi_timing_read(ms, reps)
    v = sorted(list(ms)[:n])
    lib.lmi_debug_counters(cnt)
    os.environ["LMI_SCAN_ABL"] = "0"
    lib.lmi_config_reload()
    return v[len(v) // 2], v[0], cnt[1] / reps


if a.sampled:
    # the stripes' bucket slices, as BucketLayout.shard cuts them
    lay = ix.layout
    off = lay.bucket_off
    ck = default_chunk_rows(a.world)
    firsts, rest0 = [], None
    for g in range(a.world):
        rows_first, rows_rest = [], []
        for c in range(122):
            n = int(off[c + 1] - off[c])
            lo, hi = int(off[c]) + (n * g) // a.world, int(off[c]) + (n * (g + 1)) // a.world
            rows_first.append(lay.order[lo:min(hi, lo + ck)])
            rows_rest.append(lay.order[min(hi, lo + ck):hi])
        firsts.append(np.concatenate(rows_first))
        if g == a.rank:
            rest0 = np.concatenate(rows_rest)
    xfull = x
    lab = labels.cpu().numpy() if isinstance(labels, torch.Tensor) else np.asarray(labels)
    kths = []
    for g in range(a.world):
        r = torch.from_numpy(firsts[g]).to(dev)
        ixg = DeviceIndex(xfull[r], lab[firsts[g]], 122, chunk_rows=ck)
        dg, _, _ = bucket_topk(ixg, q, classes, 10)
        kths.append(dg[:, :, 9].float().cpu().numpy())
        if g == a.rank:
            pre_ms = scan_ms(ixg, abl="0")
            pre_c = scan_ms(ixg, abl="7", reps=2)[2] if a.abl7 else float("nan")
        del ixg
    bmin = np.min(np.stack(kths), axis=0)
    r = torch.from_numpy(rest0).to(dev)
    ixr = DeviceIndex(xfull[r], lab[rest0], 122, chunk_rows=ck)
    del xfull, x
    torch.cuda.empty_cache()
    fin = kth
    print(f"# sampled-MIN bound: finite for {np.isfinite(bmin).mean():.4f} of the pairs; "
          f"bound / final 10th median {np.median(bmin[np.isfinite(bmin)] / fin[np.isfinite(bmin)]):.4f}",
          flush=True)
    for name, sd in (("rest of stripe, own bound", None), ("rest, sampled-MIN bound", f2ord(bmin)),
                     ("rest, final all-rank 10th", f2ord(fin))):
        med, mn, _ = scan_ms(ixr, sd)
        cand = scan_ms(ixr, sd, abl="7", reps=2)[2] if a.abl7 else float("nan")
        print(f"world {a.world} rank {a.rank} {name:28s} scan ms median {med:.3f} min {mn:.3f} "
              f"candidates {cand:.4g}", flush=True)
    print(f"world {a.world} rank {a.rank} {'pre-scan (first chunks)':28s} scan ms median {pre_ms[0]:.3f} "
          f"min {pre_ms[1]:.3f} candidates {pre_c:.4g}", flush=True)
    for name, sd in (("whole stripe, own bound", None), ("whole stripe, final 10th", seed)):
        med, mn, _ = scan_ms(ix, sd)
        cand = scan_ms(ix, sd, abl="7", reps=2)[2] if a.abl7 else float("nan")
        print(f"world {a.world} rank {a.rank} {name:28s} scan ms median {med:.3f} min {mn:.3f} "
              f"candidates {cand:.4g}", flush=True)
    sys.exit(0)

# correctness of the seed: every unseeded stripe entry at or under the
# all-rank 10th distance is in the seeded list, in the same order
d0, p0, _ = run(False)
d1, p1, _ = run(True)
torch.cuda.synchronize()
d0, p0, d1, p1 = (t.cpu().numpy() for t in (d0, p0, d1, p1))
keep0 = d0 <= kth[:, :, None]
keep1 = d1 <= kth[:, :, None]
ok = np.array_equal(keep0, keep1) and np.array_equal(np.where(keep0, p0, -1), np.where(keep1, p1, -1))
print(f"seeded lists hold the unseeded entries under the all-rank bound: {ok} "
      f"({int(keep0.sum())} entries of {keep0.size})", flush=True)
for rep in range(2):
    timed(False)
    timed(True)
if a.abl7:
    timed(False, "7")
    timed(True, "7")
