"""QPS of a query batch that is NOT fp16-exact: the
Searcher decides the query mode once per batch before K2 (Searcher.qmode), so
such a batch goes straight to the fp32-query scan; this times both kinds on
the bench's 10M workload (eager steps, same router and index).

    python tools/fp32_queries.py [--n 10000000] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import torch

from li import _lib, synth
from li.index import DeviceIndex, DeviceRouter, Searcher

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--nq", type=int, default=10_000)
ap.add_argument("--R", type=int, default=4)
ap.add_argument("--steps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda")
x, q, qn, xn, layers = synth.build_lmi_workload(a.n, a.nq, 122, "MLP-5", dev)  # trains the router
torch.set_grad_enabled(False)
router = DeviceRouter(layers)
labels = router.argmax(xn)
del xn
ix = DeviceIndex(x, labels, 122, chunk_rows=8192)
del x
s = Searcher(ix, router)
g = torch.Generator(device=dev)
g.manual_seed(3)
# a relative perturbation far below fp16 resolution: the same neighbours, but
# the values are no longer fp16-representable
q32 = q.float() * (1 + 1e-6 * torch.randn(q.shape, generator=g, device=dev))
out = {"n": a.n, "nq": a.nq, "R": a.R}
lib = _lib.load()
for name, qq in (("f16_exact", q), ("f32", q32)):
    mode = s.qmode(qq)
    for _ in range(2):
        s.search(qn, qq, a.R, k=10)
    torch.cuda.synchronize()
    lib.lmi_timing_read(None, 0)
    lib.lmi_timing_enable(1)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s.search(qn, qq, a.R, k=10)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    lib.lmi_timing_enable(0)
    ms = (_lib.C.c_float * a.steps)()
    n = lib.lmi_timing_read(ms, a.steps)
    out[name] = {"qmode": int(mode), "ms_per_step": round(el * 1e3, 3), "qps": round(a.nq / el, 1),
                 "scan_kernel_ms": round(sum(list(ms)[:n]) / max(n, 1), 3)}
    print(json.dumps({name: out[name]}), flush=True)
print(json.dumps(out), flush=True)
