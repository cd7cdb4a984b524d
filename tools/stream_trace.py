"""Overlap of the batch stream's branches with the scan, from a rocprofv3 kernel
trace: for each of the last scan3_kernel launches, the scan's duration, the gap to
the next scan, and how much of the other kernels' busy time falls inside the scan.
usage: python tools/stream_trace.py <run_kernel_trace.csv> [n_last]"""
import csv, re, sys

ev = []
for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("lmi::(anonymous namespace)::", ""))
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
ev.sort()
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
scans = [e for e in ev if e[2].startswith("scan3_kernel")][-n_last - 1:]
for (s0, e0, _), (s1, _, _) in zip(scans, scans[1:]):
    others = [e for e in ev if e[0] >= s0 - 2_000_000 and e[0] < s1 and not e[2].startswith("scan3_kernel")]
    inside = sum(max(0, min(e, e0) - max(s, s0)) for s, e, _ in others)
    after = [e for e in others if e[0] >= e0]
    first_after = min((e[0] for e in after), default=s1)
    last_end = max((e[1] for e in others), default=e0)
    names = sorted({n.split("<")[0] for _, _, n in after})
    print(f"scan {(e0 - s0) / 1e3:8.1f} us | next scan +{(s1 - e0) / 1e3:7.1f} us after | other kernels "
          f"busy {sum(e - s for s, e, _ in others) / 1e3:7.1f} us, {inside / 1e3:6.1f} us inside the scan | "
          f"last other kernel ends +{(last_end - e0) / 1e3:6.1f} us | after: {names[:8]}")

# one representative launch in detail: every other kernel between a scan's start
# and the next scan's start, as (start, end) relative to the scan's start, in us
if len(scans) >= 3:
    (s0, e0, _), (s1, _, _) = scans[-3], scans[-2]
    print(f"detail: scan 0 .. {(e0 - s0) / 1e3:.1f} us, next scan at {(s1 - s0) / 1e3:.1f} us")
    for s, e, n in ev:
        if s0 - 500_000 <= s < s1 and not n.startswith("scan3_kernel"):
            print(f"  {(s - s0) / 1e3:9.1f} {(e - s0) / 1e3:9.1f}  {n[:70]}")
