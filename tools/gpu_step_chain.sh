#!/bin/bash
# Kernel trace of rank 0's pipelined step graph at W = 8 (and 1): every kernel between two
# consecutive scans, to see the step's non-scan dependency chain (tools/stream_trace.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/chain
for W in ${WORLDS:-8 1}; do
  echo "== W=$W $ENVS"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chain/w$W -o run -- \
      python3 tools/stream_steps.py --worlds $W --steps 12 --modes graph-pipe > gpurun_out/chain/w$W.log 2>&1
  rc=$?; echo "W=$W trace rc=$rc"; grep world gpurun_out/chain/w$W.log; [ $rc -ne 0 ] && exit $rc
  python3 tools/stream_trace.py $(find gpurun_out/chain/w$W -name "run_kernel_trace.csv" | head -1) 6 > gpurun_out/chain/w${W}_chain.txt
  cat gpurun_out/chain/w${W}_chain.txt | cut -c1-120
done
