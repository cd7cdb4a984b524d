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
del x
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
