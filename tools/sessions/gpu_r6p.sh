#!/bin/bash
# Round 6, call p: the W = 1 bench line with CUs left to the finish chain
# (StreamedSearch reserve_cus via LMI_STREAM_RESERVE; ABI 12) against none,
# alternated on one box; then the stream tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_stream.py \
  > gpurun_out/r6p_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6p_tests.log; [ $rc -ne 0 ] && exit $rc
run() {  # name reserve
  LMI_STREAM_RESERVE=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-single \
     > gpurun_out/r6p_$1.json 2> gpurun_out/r6p_$1.err
  local rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r6p_$1.json')); print('$1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['other_dist']['ms_per_step'], d['parity'].get('stream_answers_f32'))" || tail -3 gpurun_out/r6p_$1.err
  return $rc
}
run r0a 0 || exit $?
run r4a 4 || exit $?
run r8 8 || exit $?
run r0b 0 || exit $?
run r4b 4 || exit $?
run r2 2 || exit $?
