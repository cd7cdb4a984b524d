"""Host gap between graph-replayed search steps.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/graph_gap.py [--n 10000000]
    python3 tools/graph_gap.py --trace DIR/.../run_kernel_trace.csv

The first form runs the bench's step (Searcher.graph: router, scan, replay and
the D2H replayed as one HIP graph, then a stream synchronise, as bench.py
times it) --steps times after --warmup replays.  The second reads the kernel
trace: a step starts at its router dispatch (the small-grid router_mfma_kernel)
and the gap is the GPU idle time between the previous step's last kernel and
it: the host's time from the end-of-step synchronisation to the next replay."""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--nq", type=int, default=10_000)
ap.add_argument("--R", type=int, default=4)
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--trace", default=None)
a = ap.parse_args()

if a.trace:
    ev = []
    for r in csv.DictReader(open(a.trace)):
        grid = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], grid))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if "router_mfma_kernel" in e[2] and e[3] < 10000]
    starts = starts[-a.steps:]
    gaps, steps = [], []
    for j, i in enumerate(starts):
        prev_end = max(e[1] for e in ev[:i]) if i > 0 else ev[i][0]
        gaps.append((ev[i][0] - prev_end) / 1e3)
        if j + 1 < len(starts):
            steps.append((ev[starts[j + 1]][0] - ev[i][0]) / 1e3)
    out = {"steps_seen": len(starts), "gap_us_median": round(statistics.median(gaps), 1),
           "gap_us_max": round(max(gaps), 1), "step_us_median": round(statistics.median(steps), 1),
           "gaps_us": [round(g, 1) for g in gaps]}
    print(json.dumps(out))
    sys.exit(0)

sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import torch  # noqa: E402

from li import synth  # noqa: E402
from li.index import DeviceIndex, DeviceRouter, Searcher  # noqa: E402

dev = torch.device("cuda")
x, q, qn, xn, layers = synth.build_lmi_workload(a.n, a.nq, 122, "MLP-5", dev)  # trains the router
torch.set_grad_enabled(False)
router = DeviceRouter(layers)
labels = router.argmax(xn)
del xn
ix = DeviceIndex(x, labels, 122, chunk_rows=8192)
del x
gs = Searcher(ix, router).graph(qn, q, a.R, k=10)
for _ in range(a.warmup + a.steps):
    gs.run()
torch.cuda.synchronize()
print("done", flush=True)
