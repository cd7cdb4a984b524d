#!/bin/bash
# PMC passes over the scan kernel alone (tools/prof_scan.py, 10M workload).
# Usage: ABL=0 bash tools/pmc_scan.sh   (diagnostic ablation library when ABL != 0)
# One counter group per rocprofv3 run (gpurun refuses mixing --pmc with tracing).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ABL=${ABL:-0}
LIB=liblmi_hip.so; [ "$ABL" != "0" ] && LIB=liblmi_hip_abl.so
KRE=${KRE:-scan3_kernel}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  LMI_LIB_NAME=$LIB timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" \
     -d gpurun_out/pmc/p${ABL}_$i -o run --output-format csv -- python3 tools/prof_scan.py --abl $ABL --reps 3 \
     > gpurun_out/pmc/p${ABL}_$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p${ABL}_$i.log; exit $rc; fi
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
GROUPS
python3 - <<'PY'
import csv, glob, collections, os
abl = os.environ.get("ABL", "0")
tot = collections.defaultdict(float); n = collections.Counter()
for f in sorted(glob.glob(f"gpurun_out/pmc/p{abl}_*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:32s} {tot[k]:.4g}  (records {n[k]})")
PY
