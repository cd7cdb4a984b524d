#!/bin/bash
# Tail split with S row parts (LMI_SCAN_SPLIT_PARTS): split tests, then the step at
# W = 1 and 8 (rank 0; pipelined step graph) for S = 2, 4, 8, twice, same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_replay.py tests/test_gpu_parity.py tests/test_gpu_seed.py tests/test_gpu_stream.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/sp_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for S in 2 4 8; do
    LMI_SCAN_SPLIT_PARTS=$S timeout -k 10 300 python3 tools/stream_steps.py --worlds 1,8 --steps 20 --modes graph-pipe 2>&1 | grep world | sed "s/^/S=$S /" || exit 1
  done
done
