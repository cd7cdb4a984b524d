#!/bin/bash
# Round 6, call ak: the global band's refine four pairs a wave (refine_packed_kernel)
# -- the float64 GPU tests, then rank 0's W = 8 float64 launches with it and
# without (LMI_REFINE_UNPACKED=1), alternated, and float32 beside them.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f64_global.py tests/test_gpu_dist.py tests/test_gpu_rccl.py tests/test_gpu_parity.py \
  tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_edges.py tests/test_gpu_stream.py \
  > gpurun_out/r6ak_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6ak_tests.log; [ $rc -ne 0 ] && exit $rc
run() {  # name dist unpacked
  LMI_REFINE_UNPACKED=$3 timeout -k 10 300 python -u tools/stream_steps.py --worlds 8 --steps 30 --dist $2 \
    > gpurun_out/r6ak_$1.txt 2>&1
  local rc=$?; echo "== $1 rc=$rc"; grep "ms/step" gpurun_out/r6ak_$1.txt; return $rc
}
run f32 f32 0 || exit $?
run f64_unpacked f64 1 || exit $?
run f64_packed f64 0 || exit $?
run f64_unpacked_b f64 1 || exit $?
run f64_packed_b f64 0 || exit $?
run f32_b f32 0 || exit $?
exit 0
