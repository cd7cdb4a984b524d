#!/bin/bash
# Round 6, call c: kernel traces of rank 0's W = 8 stream launch in float32,
# float64 with the W-rank band (ABI 10) and float64 with each rank's own band
# (round 5's form), and the sampled-MIN cross-rank bound study.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6c
for v in f32 f64 f64local; do
  dd=${v:0:3}; extra=""; envs=""
  [ "$v" = "f64local" ] && { extra="--local-band"; export LMI_F64_LOCAL_BAND=1; }
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6c/$v -o run -- \
      python3 tools/stream_steps.py --worlds 8 --steps 12 --modes stream --dist $dd $extra > gpurun_out/r6c/$v.log 2>&1
  rc=$?; unset LMI_F64_LOCAL_BAND; echo "$v trace rc=$rc"; grep world gpurun_out/r6c/$v.log
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r6c/$v.log; exit $rc; }
  python3 tools/stream_trace.py $(find gpurun_out/r6c/$v -name "run_kernel_trace.csv" | head -1) 8 > gpurun_out/r6c/${v}_overlap.txt
  head -3 gpurun_out/r6c/${v}_overlap.txt
done
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 600 python3 tools/bound_study.py --sampled --abl7 > gpurun_out/r6c/bound_sampled.txt 2>&1
rc=$?; cat gpurun_out/r6c/bound_sampled.txt | grep -v Warning | tail -12; exit $rc
