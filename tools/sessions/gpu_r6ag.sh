#!/bin/bash
# Round 6, call ag: the split mode's collect scan skips every bucket's sample
# (under a quarter of it) and takes the sample scan's own list for those rows
# (ABI 13), the sample fallback sliced over workgroups -- the split GPU tests, then the split bench line with the skip off
# (LMI_X_SKIP_SHARE=0) and on, alternated, and its kernel stats under rocprofv3.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_split_mode.py tests/test_gpu_split_stream.py tests/test_gpu_split.py tests/test_gpu_stream.py \
  > gpurun_out/r6ag_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6ag_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for sk in 0 4; do
    LMI_X_SKIP_SHARE=$sk timeout -k 10 300 python -u bench.py --corpus f32 --no-cpu-baseline --steps 20 --warmup 5 \
      > gpurun_out/r6ag_split_${sk}_$i.json 2> gpurun_out/r6ag_split_${sk}_$i.err
    rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6ag_split_${sk}_$i.json')); print('split skip $sk', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['other_dist']['ms_per_step'], d['single_batch']['ms'], d['parity']['lists_f32']['mismatches'], d['parity']['stream_answers_f32'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ag_prof -o run -- \
  python3 bench.py --corpus f32 --no-cpu-baseline --no-single --steps 10 --warmup 3 > gpurun_out/r6ag_prof.json 2> gpurun_out/r6ag_prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
