"""Summarise tools/pmc_sq.sh's passes: per-dispatch means of every counter
for the product scan (scan3_kernel<10, 0, false, 0>), and the derived
fractions (MICROARCH.md "rocprofv3 PMC slots", "DVFS give-back"):
  clock_ghz      GRBM_GUI_ACTIVE / 8 XCDs / the kernel's HIP-event time
  mfma_busy      SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles)
  wait/issue/active  SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over
                 SQ_WAVE_CYCLES (disjoint; quad-cycles)
Usage: python tools/pmc_sq_summary.py gpurun_out/pmc_sq"""
import collections
import csv
import glob
import json
import re
import sys

d = sys.argv[1]
KEY = "<10, 0, false, 0>"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if KEY in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
ms = []
for f in sorted(glob.glob(f"{d}/p*.log")):
    for line in open(f):
        m = re.search(r"scan ms: median ([0-9.]+)", line)
        if m:
            ms.append(float(m.group(1)))
mean = {k: sum(v) / len(v) for k, v in vals.items()}
out = {"kernel": f"scan3_kernel{KEY} (product, configs[2]: 10M, R=4, 10k queries)",
       "dispatches_per_counter": {k: len(v) for k, v in vals.items()},
       "counters_mean_per_dispatch": mean,
       "kernel_ms_under_profiler": ms}
if ms and "GRBM_GUI_ACTIVE" in mean:
    t = sum(ms) / len(ms) * 1e-3
    cyc = mean["GRBM_GUI_ACTIVE"] / 8
    out["clock_ghz"] = round(cyc / t / 1e9, 3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
        out["mfma_busy_of_simd_cycles"] = round(mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 4)
        # 6.18 TFLOP per launch at 32 cycles per 32x32x16 MFMA (32768 flop)
        out["mfma_count_from_busy"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / 32
if "SQ_WAVE_CYCLES" in mean:
    w = mean["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
              "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA",
              "SQ_INST_CYCLES_VMEM", "SQ_ACTIVE_INST_FLAT"):
        if k in mean:
            out[f"{k}_of_wave_cycles"] = round(mean[k] / w, 4)
if "SQ_LDS_IDX_ACTIVE" in mean and "SQ_LDS_BANK_CONFLICT" in mean:
    out["lds_bank_conflict_of_lds_active"] = round(mean["SQ_LDS_BANK_CONFLICT"] /
                                                   max(mean["SQ_LDS_IDX_ACTIVE"], 1), 4)
print(json.dumps(out, indent=1))
