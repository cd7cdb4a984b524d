"""Device replay (K4) timing on bench-shaped random lists: 10k queries, R=4,
122 buckets of skewed popularity, k=10; torch events around lmi_replay_device
(round 2's phase study and its numbers: profiles/r02_replay_phases.txt).
Times the whole replay and its ROUNDS phase alone (the part a batch stream's finish stage runs); an A/B of
two builds: LMI_LIB_NAME=<other .so>."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import numpy as np
import torch
from li import _lib  # noqa: E402
from li.index import replay_device


def _random_lists(seed, nq, R, C, kl):
    """sorted per-(query, probe) lists over buckets of 40-400 rows, skewed
    bucket popularity, ties likely (the shape tests/test_gpu_replay.py uses)"""
    rng = np.random.default_rng(seed)
    size = rng.integers(40, 400, C).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(size)])
    p = rng.dirichlet(np.full(C, 0.5))
    classes = np.stack([rng.choice(C, R, replace=False, p=p) for _ in range(nq)]).astype(np.int32)
    d = np.full((nq, R, kl), np.inf, np.float32)
    pos = np.full((nq, R, kl), -1, np.int32)
    for q in range(nq):
        for r in range(R):
            c = classes[q, r]
            n = min(kl, size[c])
            pp = rng.choice(size[c], n, replace=False) + off[c]
            dd = np.round(rng.random(n) * 0.6 + 0.2, 3).astype(np.float32)
            o = np.lexsort((pp, dd))
            d[q, r, :n], pos[q, r, :n] = dd[o], pp[o]
    ids = rng.permutation(int(off[-1])).astype(np.int64) + 1
    return classes, d, pos, size, ids


dev = torch.device("cuda")
if "--bench-lists" in sys.argv:
    # the bench's own 10M workload: its router classes and K2 lists
    from li import synth
    from li.index import DeviceIndex, DeviceRouter, bucket_topk
    x, q, qn, xn, layers = synth.build_lmi_workload(10_000_000, 10_000, 122, "MLP-5", dev)
    router = DeviceRouter(layers)
    labels = router.argmax(xn)
    del xn
    ix = DeviceIndex(x, labels, 122, chunk_rows=8192)
    del x
    cls_t, _ = router.topr(qn, 4)
    ld, lp, _ = bucket_topk(ix, q, cls_t, 10)
    args = [cls_t, ld, lp]
    bsz = torch.from_numpy(np.ascontiguousarray(ix.bucket_size, dtype=np.int64)).to(dev)
    p2id = torch.from_numpy(np.ascontiguousarray(ix.pos_to_id, dtype=np.int64)).to(dev)
    cl = cls_t.cpu().numpy()
    for r in range(cl.shape[1]):
        bc = np.bincount(cl[:, r], minlength=122)
        print(f"round {r}: group sizes max {bc.max()} p99 {np.percentile(bc, 99):.0f} "
              f"median {np.median(bc):.0f}; groups > 819 queries: {(bc > 819).sum()}", flush=True)
else:
    classes, d, pos, size, ids = _random_lists(3, nq=10000, R=4, C=122, kl=10)
    args = [torch.from_numpy(x).to(dev) for x in (classes, d, pos)]
    bsz, p2id = torch.from_numpy(size).to(dev), torch.from_numpy(ids).to(dev)
from li import _lib  # noqa: E402
nq, R = args[0].shape
w = torch.empty(1 << 26, dtype=torch.uint8, device=dev)
out = (torch.empty((nq, 10), dtype=torch.float64, device=dev), torch.empty((nq, 10), dtype=torch.int32, device=dev),
       torch.zeros((1,), dtype=torch.int32, device=dev))
kw = dict(k_round=10, k_final=10, bucket_size=bsz, pos_to_id=p2id, use_threshold=True, out=out, ws=w)
replay_device(args[0], None, None, phases=_lib.LMI_REPLAY_PHASE_GROUPS, k_list=args[1].shape[2], **kw)
for name, fn in (("whole replay (groups + rounds)", lambda: replay_device(*args, **kw)),
                 ("rounds only (the finish stage's part)",
                  lambda: replay_device(*args, phases=_lib.LMI_REPLAY_PHASE_ROUNDS, **kw))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"[{_lib.LIB_NAME}] {name}: {e0.elapsed_time(e1) / 50 * 1e3:8.1f} us", flush=True)
