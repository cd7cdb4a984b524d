#!/bin/bash
# Round 6, call q: the finish enqueued ahead of the route (LMI_STREAM_FINISH_FIRST=1)
# -- stream / RCCL tests under it, then W = 1 / W = 8 rank-0 launches against the
# product order, float32 and float64; then the split mode's PMC traffic passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
LMI_STREAM_FINISH_FIRST=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_stream.py tests/test_gpu_rccl.py > gpurun_out/r6q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6q_tests.log; [ $rc -ne 0 ] && exit $rc
run() {  # name dist ff
  LMI_STREAM_FINISH_FIRST=$3 timeout -k 10 300 python -u tools/stream_steps.py --worlds 1,8 --steps 30 --dist $2 \
    > gpurun_out/r6q_$1.txt 2>&1
  local rc=$?; echo "== $1 rc=$rc"; grep "ms/step" gpurun_out/r6q_$1.txt; return $rc
}
run f32_a f32 0 || exit $?
run f32_ff_a f32 1 || exit $?
run f64_a f64 0 || exit $?
run f64_ff_a f64 1 || exit $?
run f32_b f32 0 || exit $?
run f32_ff_b f32 1 || exit $?
run f64_b f64 0 || exit $?
run f64_ff_b f64 1 || exit $?
timeout -k 10 900 bash tools/pmc_split.sh > gpurun_out/r6q_pmc_split.log 2>&1; rc=$?; tail -3 gpurun_out/r6q_pmc_split.log; exit $rc
