#!/bin/bash
# round 4, session b: the float64 mode's scan lists, 11-entry (product) vs 15
# (liblmi_hip_kl15.so), per launch of the batch stream at W = 1 and rank 0 of
# W = 8, f32 beside; then a kernel trace of the W = 8 float64 stream.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/r4b
for rep in 1 2; do
  for lib in liblmi_hip.so liblmi_hip_kl15.so; do
    LMI_LIB_NAME=$lib timeout -k 10 400 python3 tools/stream_steps.py --worlds 1,8 --dist f64 --steps 20 --modes stream \
        > gpurun_out/r4b/f64_${lib}_$rep.log 2>&1 || { tail -5 gpurun_out/r4b/f64_${lib}_$rep.log; exit 1; }
    echo "$lib rep $rep:"; grep world gpurun_out/r4b/f64_${lib}_$rep.log
  done
done
timeout -k 10 400 python3 tools/stream_steps.py --worlds 1,8 --dist f32 --steps 20 --modes stream > gpurun_out/r4b/f32.log 2>&1 || exit 1
echo "f32:"; grep world gpurun_out/r4b/f32.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b/trace -o run -- \
    python3 tools/stream_steps.py --worlds 8 --dist f64 --steps 12 --modes stream > gpurun_out/r4b/trace.log 2>&1 || exit 1
python3 tools/trace_summary.py $(find gpurun_out/r4b/trace -name "run_kernel_trace.csv" | head -1) > gpurun_out/r4b/trace_summary.txt 2>&1
head -30 gpurun_out/r4b/trace_summary.txt
