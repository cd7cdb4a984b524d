"""Per-kernel durations of the search step from a rocprofv3 kernel trace:
dispatches of lmi:: kernels grouped by (name, grid), median/mean/count, so the
10M build's big launches (router argmax over the corpus) separate from the
per-step ones.  usage: python tools/trace_summary.py <run_kernel_trace.csv>"""
import csv, re, statistics, sys
from collections import defaultdict

rows = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if "lmi::" not in name:
        continue
    short = re.sub(r"\(.*", "", name.replace("void ", "").replace("lmi::(anonymous namespace)::", ""))
    grid = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
    rows[(short, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':48s} {'WGs':>8s} {'calls':>6s} {'median us':>10s} {'mean us':>10s}")
for (k, g), v in sorted(rows.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    print(f"{k:48s} {g:8d} {len(v):6d} {statistics.median(v):10.1f} {statistics.mean(v):10.1f}")

# idle time of the GPU between consecutive dispatches (all kernels, in start order), over the
# last third of the trace (steady state): the host gaps a captured graph removes
ev = []
for r in csv.DictReader(open(sys.argv[1])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
ev.sort()
ev = ev[2 * len(ev) // 3:]
if len(ev) > 1:
    busy_end, idle, gaps = ev[0][1], 0, []
    for a, b in ev[1:]:
        if a > busy_end:
            idle += a - busy_end
            gaps.append((a - busy_end) / 1e3)
        busy_end = max(busy_end, b)
    span = (ev[-1][1] - ev[0][0]) / 1e3
    gaps.sort(reverse=True)
    print(f"steady-state window {span:.1f} us: GPU idle {idle / 1e3:.1f} us "
          f"({100 * idle / 1e3 / span:.1f}%), largest gaps us {[round(g, 1) for g in gaps[:8]]}")
