#!/bin/bash
# Round 6, call ar: the batch stream's answer D2H after a kdone event (the
# lookahead scan waits for the finish's kernels only, the copy runs beside its
# start) -- the stream / RCCL / split-stream GPU tests, then against
# LMI_STREAM_WAIT_D2H=1 (the previous order), alternated: rank 0's W = 8
# launches in both arithmetics and the W = 1 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_stream.py tests/test_gpu_rccl.py tests/test_gpu_split_stream.py tests/test_gpu_dist.py \
  tests/test_gpu_graph.py > gpurun_out/r6ar_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6ar_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for w in 1 0; do
    for dd in f32 f64; do
      LMI_STREAM_WAIT_D2H=$w timeout -k 10 300 python -u tools/stream_steps.py --worlds 8 --steps 30 --dist $dd \
        > gpurun_out/r6ar_w8_${dd}_${w}_$i.txt 2>&1
      rc=$?; echo "wait_d2h=$w $dd run $i: $(grep 'ms/step' gpurun_out/r6ar_w8_${dd}_${w}_$i.txt)"; [ $rc -ne 0 ] && exit $rc
    done
  done
done
for i in 1 2; do
  for w in 1 0; do
    LMI_STREAM_WAIT_D2H=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 \
      > gpurun_out/r6ar_w1_${w}_$i.json 2> gpurun_out/r6ar_w1_${w}_$i.err
    rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6ar_w1_${w}_$i.json')); print('w1 wait_d2h=$w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['other_dist']['ms_per_step'], d['parity'].get('stream_answers_f32', d['parity'].get('stream_answers')))"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
