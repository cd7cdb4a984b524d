"""Per-kernel breakdown of the timed bound + collect calls in a rocprofv3
kernel trace of tools/wide_bench.py (the second call of each k: after the
warm-up).  python tools/wide_trace.py <trace dir>"""
import csv
import glob
import os
import re
import sys


def main(root):
    f = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    nm = lambda r: re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")) \
        .replace("void ", "").replace("lmi::", "")
    starts = [i for i, r in enumerate(rows) if "wide_init_kernel" in r["Kernel_Name"]]
    # per k: warm-up, timed, then (after the passes) the no-fix-up call
    for n, i0 in enumerate(starts[1::3]):
        i1 = next((i for i in range(i0, len(rows)) if "fix_combine" in rows[i]["Kernel_Name"]), None)
        if i1 is None:
            break
        i1 += 1
        span = (int(rows[i1 - 1]["End_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e6
        agg = {}
        for r in rows[i0:i1]:
            a = agg.setdefault(nm(r), [0, 0.0])
            a[0] += 1
            a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        print(f"call {n}: {span:.3f} ms, {i1 - i0} kernels")
        for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"  {t:8.3f} ms {c:4d}  {k[:90]}")


if __name__ == "__main__":
    main(sys.argv[1])
