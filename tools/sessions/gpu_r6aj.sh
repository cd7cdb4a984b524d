#!/bin/bash
# Round 6, call aj: rank 0's W = 8 batch-stream launch traces on the current tree,
# float32 then float64 (tools/gpu_stream_trace.sh), for the float64 finish chain.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
for dd in f32 f64; do
  WGSS=0 WORLDS=8 EXTRA="--dist $dd --steps 12" timeout -k 10 400 bash tools/gpu_stream_trace.sh > gpurun_out/r6aj_trace_$dd.log 2>&1
  rc=$?; tail -3 gpurun_out/r6aj_trace_$dd.log; [ $rc -ne 0 ] && exit $rc
  cp gpurun_out/strace/w0_overlap.txt gpurun_out/r6aj_w8_${dd}_trace.txt
  cp $(find gpurun_out/strace/w0 -name "run_kernel_trace.csv" | head -1) gpurun_out/r6aj_w8_${dd}_kernel_trace.csv
  rm -rf gpurun_out/strace
done
exit 0
