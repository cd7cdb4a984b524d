#!/bin/bash
# round 4, session e: candidates and time with the union-of-halves bound
# (diagnostic ABL 81 = ABL 7's counters + the bound) vs the product (ABL 7)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4e
for W in 8 1; do
  ck=8192; [ $W = 8 ] && ck=2048
  LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 300 python3 tools/prof_scan.py --abl 0,7,81,0,7,81 --reps 5 --world $W --rank 0 \
      --chunk-rows $ck --check > gpurun_out/r4e/w$W.log 2>&1 || { tail -5 gpurun_out/r4e/w$W.log; exit 1; }
  echo "W=$W:"; grep "scan ms\|per launch\|identical" gpurun_out/r4e/w$W.log
done
