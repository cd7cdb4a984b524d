#!/bin/bash
# kernel trace of the W=8 shard step (per-kernel fixed costs), and the GPU idle
# gap between steps with one synchronised graph vs two batches in flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
WORLDS=8 STEPS=20 bash tools/gpu_step_trace.sh || exit $?
for P in 0 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gg$P -o run -- \
      python3 tools/graph_gap.py --pipeline $P > gpurun_out/gg$P.log 2>&1
  rc=$?; echo "gap P=$P rc=$rc"; [ $rc -ne 0 ] && { tail -3 gpurun_out/gg$P.log; exit $rc; }
  python3 tools/graph_gap.py --trace $(find gpurun_out/gg$P -name "run_kernel_trace.csv" | head -1) | tee gpurun_out/gg${P}_summary.json | cut -c1-200
done
