#!/bin/bash
# Round 6, call aq: the split mode's skip threshold -- a bucket's sample skipped
# by the collect when it is at most 1/2, 1/3 or 1/4 (default) of the bucket
# (LMI_X_SKIP_SHARE): the split tests at 2, then the split bench alternated.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
LMI_X_SKIP_SHARE=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_split_mode.py tests/test_gpu_split_stream.py > gpurun_out/r6aq_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6aq_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for sk in 4 2 3; do
    LMI_X_SKIP_SHARE=$sk timeout -k 10 300 python -u bench.py --corpus f32 --no-cpu-baseline --no-single --steps 20 --warmup 5 \
      > gpurun_out/r6aq_split_${sk}_$i.json 2> gpurun_out/r6aq_split_${sk}_$i.err
    rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6aq_split_${sk}_$i.json')); print('split share $sk', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['parity']['lists_f32']['mismatches'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
