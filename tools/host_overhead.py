"""Host-side cost of one Searcher.search step (10M workload): cProfile of the
steady-state loop, top entries by own time.  The GPU idles for this long
between steps (the trace shows the gap before each step's router)."""
import cProfile, os, pstats, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import torch
from li import synth
from li.index import DeviceIndex, DeviceRouter, Searcher

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
dev = torch.device("cuda")
x, q, qn, xn, layers = synth.build_lmi_workload(n, 10_000, 122, "MLP-5", dev)
router = DeviceRouter(layers)
labels = router.argmax(xn); del xn
s = Searcher(DeviceIndex(x, labels, 122, device=dev), router)
for _ in range(5):
    s.search(qn, q, 4, k=10)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
t0 = time.perf_counter()
for _ in range(20):
    s.search(qn, q, 4, k=10)
el = (time.perf_counter() - t0) / 20
pr.disable()
print(f"step {el * 1e3:.3f} ms")
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
