#!/bin/bash
# Round 6, call r: the float64 global band's k-th per pair in its own kernel
# (band_kth_kernel) and the sliced fallback's merge folded into fallback_kernel --
# the float64 GPU tests, the W = 8 rank-0 float64 / float32 launches with
# LMI_REFINE_KB 1 / 2 / 4, and a kernel trace of the float64 W = 8 launch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f64_global.py tests/test_gpu_dist.py tests/test_gpu_rccl.py tests/test_gpu_parity.py \
  tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_edges.py tests/test_gpu_stream.py \
  > gpurun_out/r6r_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6r_tests.log; [ $rc -ne 0 ] && exit $rc
run() {  # name dist kb
  LMI_REFINE_KB=$3 timeout -k 10 300 python -u tools/stream_steps.py --worlds 8 --steps 30 --dist $2 \
    > gpurun_out/r6r_$1.txt 2>&1
  local rc=$?; echo "== $1 rc=$rc"; grep "ms/step" gpurun_out/r6r_$1.txt; return $rc
}
run f32 f32 1 || exit $?
run f64_kb1 f64 1 || exit $?
run f64_kb2 f64 2 || exit $?
run f64_kb4 f64 4 || exit $?
run f32b f32 1 || exit $?
run f64_kb1b f64 1 || exit $?
WGSS=0 WORLDS=8 EXTRA="--dist f64 --steps 12" timeout -k 10 400 bash tools/gpu_stream_trace.sh > gpurun_out/r6r_trace.log 2>&1
rc=$?; tail -5 gpurun_out/r6r_trace.log; exit $rc
