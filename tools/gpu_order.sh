#!/bin/bash
# tile order A/B: LMI_SCAN_ORDER 0 (queue order), 1 (heavy-first per tile), 2 (heavy-first per chunk,
# sibling tiles adjacent): scan time (diagnostic build, clocks) and FETCH_SIZE per order
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 400 python tools/prof_scan.py --no-subcluster --check --reps 10 --abl 0 \
   --variants "LMI_SCAN_ORDER=1|LMI_SCAN_ORDER=2|LMI_SCAN_ORDER=0|LMI_SCAN_ORDER=1|LMI_SCAN_ORDER=2|LMI_SCAN_ORDER=0" > gpurun_out/order.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/order.log; [ $rc -ne 0 ] && exit $rc
for O in 0 1 2; do
  LMI_SCAN_ORDER=$O timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex scan3_kernel --output-format csv \
     -d gpurun_out/ord_pmc$O -o run -- python3 tools/prof_scan.py --no-subcluster --reps 3 > gpurun_out/ord_pmc$O.log 2>&1
  rc=$?; echo "pmc order $O rc=$rc"; [ $rc -ne 0 ] && { tail -3 gpurun_out/ord_pmc$O.log; exit $rc; }
  python3 - $O <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(f"gpurun_out/ord_pmc{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
print(f"order {sys.argv[1]}: FETCH_SIZE launches {len(v)}, mean {sum(v)/max(len(v),1)/1e6:.3f} GB (x2 on gfx950 -> {2*sum(v)/max(len(v),1)/1e6:.2f} GB)")
PY
done
