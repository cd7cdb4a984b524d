#!/bin/bash
# Round 6, call ad: the bound exchange (every 32 blocks) in the float64 band
# scan (scan3_kernel MODE 3) too -- the float64 GPU tests, then the W = 8
# rank-0 float64 launches and the W = 1 bench line against the previous build
# (li/liblmi_hip_base.so), alternated.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f64_global.py tests/test_gpu_parity.py tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py \
  tests/test_gpu_seed.py tests/test_gpu_dist.py > gpurun_out/r6ad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6ad_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in liblmi_hip_base.so liblmi_hip.so; do
    LMI_LIB_NAME=$lib timeout -k 10 300 python -u tools/stream_steps.py --worlds 1,8 --steps 40 --dist f64 > gpurun_out/r6ad_${lib}_$i.txt 2>&1
    rc=$?; echo "$lib $(grep -h ms/step gpurun_out/r6ad_${lib}_$i.txt | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
  done
done
for lib in liblmi_hip_base.so liblmi_hip.so; do
  LMI_LIB_NAME=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-single \
    > gpurun_out/r6ad_bench_$lib.json 2> gpurun_out/r6ad_bench_$lib.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6ad_bench_$lib.json')); print('bench $lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist'])"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
