#!/bin/bash
# Batch stream with / without the next scan enqueued ahead: stream tests, then same-box A/B at W = 1 / 8
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 250 --timeout-method thread > gpurun_out/s3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s3_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 tools/stream_steps.py --worlds 1,8 --steps 20 --modes stream-la,stream-nola,stream-fin,graph-pipe 2>&1 | grep world || exit 1
done
