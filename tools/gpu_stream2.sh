#!/bin/bash
# Batch stream on four streams (per-branch graphs, SDMA upload): stream tests, then the same-box
# A/B against the pipelined step graph at W = 1 / 8 (rank 0), twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_dist.py -x -q --timeout 250 --timeout-method thread > gpurun_out/s2_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 tools/stream_steps.py --worlds 1,8 --steps 20 --modes graph-pipe,stream,stream-eager 2>&1 | grep world || exit 1
done
