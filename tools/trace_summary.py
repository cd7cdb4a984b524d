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
