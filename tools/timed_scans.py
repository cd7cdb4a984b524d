"""Per-launch durations of the scan kernel inside bench.py's timed region, from
a rocprofv3 run with --kernel-trace --marker-trace (tools/gpu_profile.sh).

bench.py brackets each timed loop with a ROCTx range ("bench timed stream f32",
...); this picks the scan3_kernel dispatches whose start lies inside each range
and reports their durations with mean and median, so the profile's figure for
the roofline kernel is the timed launches' own (warm-up, checks and the other
passes of the bench are outside the ranges).

    python tools/timed_scans.py <rocprofv3 output dir> [out.json]
"""
import csv
import glob
import json
import os
import statistics
import sys


def rows(pattern, root):
    out = []
    for f in glob.glob(os.path.join(root, "**", pattern), recursive=True):
        out.extend(csv.DictReader(open(f)))
    return out


def main(root, out_path=None, kernel="scan3_kernel"):
    kern = rows("*kernel_trace.csv", root)
    marks = rows("*marker_api_trace.csv", root)
    ranges = []
    for m in marks:
        text = " ".join(str(v) for v in m.values())
        if "bench timed" in text:
            name = next((str(v) for v in m.values() if "bench timed" in str(v)), text)
            ranges.append((name, int(m["Start_Timestamp"]), int(m["End_Timestamp"])))
    res = {"source": os.path.relpath(root), "kernel": kernel, "ranges": []}
    for name, a, b in sorted(ranges, key=lambda r: r[1]):
        d = sorted(((int(k["Start_Timestamp"]), (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e6,
                     k["Kernel_Name"]) for k in kern
                    if kernel in k["Kernel_Name"] and a <= int(k["Start_Timestamp"]) <= b))
        ms = [x[1] for x in d]
        r = {"range": name, "range_ms": round((b - a) / 1e6, 3), "launches": len(ms)}
        if ms:
            r.update(mean_ms=round(statistics.mean(ms), 4), median_ms=round(statistics.median(ms), 4),
                     min_ms=round(min(ms), 4), max_ms=round(max(ms), 4),
                     durations_ms=[round(x, 4) for x in ms],
                     kernel_names=sorted({x[2].replace("(anonymous namespace)::", "").split("(")[0]
                                          .replace("void ", "") for x in d}))
        res["ranges"].append(r)
    s = json.dumps(res, indent=1)
    print(s)
    if out_path:
        open(out_path, "w").write(s + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
