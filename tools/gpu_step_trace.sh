#!/bin/bash
# Kernel trace of the per-rank step at W = 1 and W = 8 (rank 0's shard on one GPU, tools/shard_step.py):
# per-kernel times and the GPU idle time between dispatches (host gaps)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for W in ${WORLDS:-1 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st$W -o run -- \
      python3 tools/shard_step.py --worlds $W --steps ${STEPS:-20} > gpurun_out/st$W.log 2>&1
  rc=$?; echo "W=$W trace rc=$rc"; grep -v amdgpu.ids gpurun_out/st$W.log | tail -2
  [ $rc -ne 0 ] && exit $rc
  python3 tools/trace_summary.py $(find gpurun_out/st$W -name "run_kernel_trace.csv" | head -1) | tee gpurun_out/st${W}_summary.txt
done
