#!/bin/bash
# Round 6, call u: the merge phase on the scan's stream right behind the scan
# (LMI_STREAM_MERGE_ON_SCAN=1) -- the stream / split-stream / RCCL / dist tests
# under it, then W = 1 / W = 8 rank-0 launches and the W = 1 bench line,
# alternated against the product order.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
LMI_STREAM_MERGE_ON_SCAN=1 timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_stream.py tests/test_gpu_split_stream.py tests/test_gpu_rccl.py tests/test_gpu_dist.py \
  > gpurun_out/r6u_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6u_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for m in 0 1; do
    for dd in f32 f64; do
      LMI_STREAM_MERGE_ON_SCAN=$m timeout -k 10 300 python -u tools/stream_steps.py --worlds 1,8 --steps 40 --dist $dd \
        > gpurun_out/r6u_m${m}_${dd}_$i.txt 2>&1
      rc=$?; echo "mos=$m $(grep -h ms/step gpurun_out/r6u_m${m}_${dd}_$i.txt | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
    done
  done
done
for i in 1 2; do
  for m in 0 1; do
    LMI_STREAM_MERGE_ON_SCAN=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-single \
      > gpurun_out/r6u_bench_m${m}_$i.json 2> gpurun_out/r6u_bench_m${m}_$i.err
    rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6u_bench_m${m}_$i.json')); print('bench mos=$m', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['other_dist']['ms_per_step'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
