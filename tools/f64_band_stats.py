"""K2 in float64 at 10M (the bench workload): time of lmi_bucket_topk_f64 (scan,
chunk merge, refine, fallback) against the float32 lmi_bucket_topk on the same
lists, and the number of pairs the refine sent to the whole-shard fallback.
An A/B of two builds: LMI_LIB_NAME=<other .so>."""
import argparse, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import torch
from li import _lib, synth
from li.index import DeviceIndex, DeviceRouter, bucket_topk, bucket_topk_f64

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--R", type=int, default=4)
ap.add_argument("--chunk-rows", type=int, default=8192)
args = ap.parse_args()
dev = torch.device("cuda", 0)
x, q, qn, xn, layers = synth.build_lmi_workload(args.n, 10_000, 122, "MLP-5", dev)
router = DeviceRouter(layers)
labels = router.argmax(xn)
del xn
ix = DeviceIndex(x, labels, 122, chunk_rows=args.chunk_rows)
del x
cls, _ = router.topr(qn, args.R)


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for seed in (False, True):
    t32 = timed(lambda: bucket_topk(ix, q, cls, 10, seed_round0=seed))
    t64 = timed(lambda: bucket_topk_f64(ix, q, cls, 10, seed_round0=seed))
    _, _, st, nfb = bucket_topk_f64(ix, q, cls, 10, seed_round0=seed, fallback_count=True)
    print(f"[{_lib.LIB_NAME}] n {args.n} R {args.R} seed {int(seed)}: f32 {t32:.3f} ms, f64 {t64:.3f} ms (+{(t64 / t32 - 1) * 100:.1f}%), "
          f"fallback pairs {nfb} of {cls.numel()}, status {int(st.item())}", flush=True)
