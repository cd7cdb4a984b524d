#!/bin/bash
# SQ / GRBM counter passes over the PRODUCT scan kernel at configs[2] (10M,
# R = 4, the bench's layout: no sub-clustering), one rocprofv3 run per pass
# (tools/prof_scan.py: 2 warm-up + REPS timed launches), then
# tools/pmc_sq_summary.py -> gpurun_out/pmc_sq/summary.json.
# Usage: bash tools/pmc_sq.sh   (KRE: kernel regex, REPS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_sq
mkdir -p $OUT
export TMPDIR=/tmp
KRE=${KRE:-scan3_kernel}
REPS=${REPS:-3}
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
have() { grep -qw "$1" $OUT/counters.txt; }
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU"
have SQ_INSTS_MFMA && B="$B SQ_INSTS_MFMA"
C="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
i=0
for grp in "$A" "$B" "$C"; do
  i=$((i+1))
  cs=""
  for c in $grp; do have $c && cs="$cs $c"; done
  echo "pass $i:$cs"
  timeout -s KILL 150 rocprofv3 --pmc $cs --kernel-include-regex "$KRE" --output-format csv \
     -d $OUT/p$i -o run -- python3 tools/prof_scan.py --no-subcluster --reps $REPS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; grep "scan ms" $OUT/p$i.log
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_sq_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
