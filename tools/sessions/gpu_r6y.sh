#!/bin/bash
# Round 6, call y: the split sample halved (max(chunk_rows / 2, n_c / 16) rows) on top of
# the LDS-staged collect -- the split-mode / wide (k > 16) /
# golden GPU tests, then the split-mode bench line twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_split_mode.py tests/test_gpu_split_stream.py tests/test_gpu_split.py tests/test_gpu_wide.py \
  tests/test_gpu_golden_r2.py tests/test_gpu_golden.py > gpurun_out/r6y_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6y_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --corpus f32 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6y_split_$i.json 2> gpurun_out/r6y_split_$i.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6y_split_$i.json')); print('split', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist'], d['single_batch']['ms'], d['parity']['lists_f32']['mismatches'], d['parity'].get('stream_answers_f32'))"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
