#!/bin/bash
# round 4, session f: bound-exchange period at rank 0 of W = 8 and at W = 1
# (diagnostic ABL 41 / 42 / 43: every 4 / 8 / 16 blocks; 0: every 32)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4f
for W in 8 1; do
  ck=8192; [ $W = 8 ] && ck=2048
  LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 300 python3 tools/prof_scan.py --abl 0,41,42,43,0,41,42,43 --reps 7 --world $W --rank 0 \
      --chunk-rows $ck > gpurun_out/r4f/w$W.log 2>&1 || { tail -5 gpurun_out/r4f/w$W.log; exit 1; }
  echo "W=$W:"; grep "scan ms" gpurun_out/r4f/w$W.log
done
