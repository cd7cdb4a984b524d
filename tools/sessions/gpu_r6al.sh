#!/bin/bash
# Round 6, call al: the chunk merges as bitonic merges over 16 register slots
# (chunk_merge_kernel, chunk_merge_band_kernel) -- the merge-path GPU tests, then
# rank 0's W = 8 launches (float32, float64) and the W = 1 bench against the
# previous build (li/liblmi_hip_base.so), alternated.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f64_global.py tests/test_gpu_dist.py tests/test_gpu_rccl.py tests/test_gpu_parity.py \
  tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_edges.py tests/test_gpu_stream.py \
  tests/test_gpu_split_mode.py tests/test_gpu_graph.py > gpurun_out/r6al_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6al_tests.log; [ $rc -ne 0 ] && exit $rc
run() {  # name dist lib
  LMI_LIB_NAME=$3 timeout -k 10 300 python -u tools/stream_steps.py --worlds 8 --steps 30 --dist $2 \
    > gpurun_out/r6al_$1.txt 2>&1
  local rc=$?; echo "== $1 rc=$rc"; grep "ms/step" gpurun_out/r6al_$1.txt; return $rc
}
for i in 1 2; do
  for lib in liblmi_hip_base.so liblmi_hip.so; do
    run w8_f32_${lib}_$i f32 $lib || exit $?
    run w8_f64_${lib}_$i f64 $lib || exit $?
  done
done
for i in 1 2; do
  for lib in liblmi_hip_base.so liblmi_hip.so; do
    LMI_LIB_NAME=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 \
      > gpurun_out/r6al_w1_${lib}_$i.json 2> gpurun_out/r6al_w1_${lib}_$i.err
    rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6al_w1_${lib}_$i.json')); print('w1 $lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['other_dist']['ms_per_step'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
