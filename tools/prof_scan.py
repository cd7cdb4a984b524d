"""Scan-kernel timing harness: 10M workload, lmi_bucket_topk only, optional
ablation variants (LMI_LIB_NAME=liblmi_hip_abl.so, LMI_SCAN_ABL=0..3)."""
import argparse, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import numpy as np, torch
from li import _lib, synth
from li.index import DeviceIndex, DeviceRouter, bucket_topk

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--nq", type=int, default=10_000)
ap.add_argument("--R", type=int, default=4)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--chunk-rows", type=int, default=8192)
ap.add_argument("--abl", default="0")
ap.add_argument("--world", type=int, default=1, help="time the shard of --rank out of --world GPUs")
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--no-subcluster", action="store_true")
ap.add_argument("--check", action="store_true", help="compare every variant's lists to abl=0 (bitwise)")
ap.add_argument("--variants", default="",
                help="'|'-separated env settings, e.g. 'LMI_SCAN_GROUPS=1,LMI_SCAN_LAG=1|LMI_SCAN_GROUPS=8'")
a = ap.parse_args()
dev = torch.device("cuda")
x, q, qn, xn, layers = synth.build_lmi_workload(a.n, a.nq, 122, "MLP-5", dev)
router = DeviceRouter(layers)
labels = router.argmax(xn); del xn
ix = DeviceIndex(x, labels, 122, chunk_rows=a.chunk_rows, subcluster=not a.no_subcluster,
                 rank=a.rank, world=a.world)
classes, _ = router.topr(qn, a.R)
lib = _lib.load()
ref = None
if a.check:
    os.environ["LMI_SCAN_ABL"] = "0"
    _lib.load().lmi_config_reload()
    ref = bucket_topk(ix, q, classes, 10)[:2]
runs = [(abl, "") for abl in a.abl.split(",")]
if a.variants:
    runs = [(abl, v) for v in a.variants.split("|") for abl in a.abl.split(",")]
prev = []
for abl, var in runs:
    os.environ["LMI_SCAN_ABL"] = abl
    for kk in prev:  # (a variant's settings end with it)
        os.environ.pop(kk, None)
    prev = []
    for kv in filter(None, var.split(",")):
        kk, vv = kv.split("=")
        os.environ[kk] = vv
        prev.append(kk)
    _lib.load().lmi_config_reload()
    for _ in range(2):
        bucket_topk(ix, q, classes, 10)
    torch.cuda.synchronize()
    dbg = hasattr(lib, "lmi_debug_counters")
    cnt = (_lib.C.c_ulonglong * 16)()
    if dbg:
        lib.lmi_debug_counters(cnt)  # clear
    lib.lmi_timing_read(None, 0)
    lib.lmi_timing_enable(1)
    for _ in range(a.reps):
        bucket_topk(ix, q, classes, 10)
    torch.cuda.synchronize()
    lib.lmi_timing_enable(0)
    ms = (_lib.C.c_float * a.reps)()
    n = lib.lmi_timing_read(ms, a.reps)
    v = sorted(list(ms)[:n])
    print(f"[{var}] abl={abl} scan ms: median {v[len(v)//2]:.3f} min {v[0]:.3f}", flush=True)
    if dbg:
        lib.lmi_debug_counters(cnt)
        if cnt[9] and cnt[12]:
            # shader clock = cycles / 100-MHz ticks; utilisation = mean
            # workgroup lifetime / (last exit - first entry) of the reps
            ghz = cnt[8] / cnt[9] * 0.1
            life_us = cnt[9] / cnt[12] * 0.01
            print(f"   clock {ghz:.3f} GHz, workgroup life {life_us:.0f} us avg over {cnt[12] // a.reps} WGs/launch",
                  flush=True)
        if abl == "7":
            names = ["wave-events", "candidates", "appends", "sorted-inserts", "fills", "wave-blocks"]
            print("   per launch: " + ", ".join(f"{nm}={cnt[i] / a.reps:.4g}" for i, nm in enumerate(names)),
                  flush=True)
        # one more launch alone: the spread of workgroup starts and ends
        # (100-MHz s_memrealtime ticks -> us), i.e. the persistent grid's tail
        lib.lmi_debug_counters(cnt)
        bucket_topk(ix, q, classes, 10)
        torch.cuda.synchronize()
        c1 = (_lib.C.c_ulonglong * 16)()
        lib.lmi_debug_counters(c1)
        if c1[12]:
            t0 = c1[10]
            print(f"   one launch: span {(c1[11] - t0) * 0.01:.1f} us, last start {(c1[13] - t0) * 0.01:.1f} us, "
                  f"first end {(c1[14] - t0) * 0.01:.1f} us, mean life {c1[9] / c1[12] * 0.01:.1f} us", flush=True)
    if ref is not None:
        d, p_ = bucket_topk(ix, q, classes, 10)[:2]
        same = bool(torch.equal(d, ref[0]) and torch.equal(p_, ref[1]))
        print(f"   lists identical to abl=0: {same}", flush=True)
