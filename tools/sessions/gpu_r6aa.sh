#!/bin/bash
# Round 6, call aa: the answer's D2H as a graph of its own after the finish,
# which the next scan does not wait for (LMI_STREAM_D2H_BESIDE=1) -- the stream /
# RCCL / split-stream tests under it, then the W = 1 bench line and the W = 8
# rank-0 launches, alternated against the product.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
LMI_STREAM_D2H_BESIDE=1 timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_stream.py tests/test_gpu_rccl.py tests/test_gpu_split_stream.py > gpurun_out/r6aa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6aa_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for m in 0 1; do
    LMI_STREAM_D2H_BESIDE=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-single \
      > gpurun_out/r6aa_bench_m${m}_$i.json 2> gpurun_out/r6aa_bench_m${m}_$i.err
    rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6aa_bench_m${m}_$i.json')); print('bench d2h_beside=$m', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['other_dist']['ms_per_step'], d['parity']['stream_answers_f32'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
for i in 1 2; do
  for m in 0 1; do
    LMI_STREAM_D2H_BESIDE=$m timeout -k 10 300 python -u tools/stream_steps.py --worlds 8 --steps 40 --dist f32 > gpurun_out/r6aa_w8_m${m}_$i.txt 2>&1
    rc=$?; echo "d2h_beside=$m $(grep -h ms/step gpurun_out/r6aa_w8_m${m}_$i.txt)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
