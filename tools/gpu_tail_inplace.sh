#!/bin/bash
# In-place tail split: parity tests, then the step-chain trace at W = 8 and the pipelined
# step at W = 1 / 8
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_seed.py tests/test_gpu_graph.py tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_stream.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/tip_tests.log 2>&1; rc=$?; tail -3 gpurun_out/tip_tests.log; [ $rc -ne 0 ] && exit $rc
WORLDS=8 bash tools/gpu_step_chain.sh 2>&1 | grep -A24 detail | head -26
for rep in 1 2; do
  timeout -k 10 300 python3 tools/stream_steps.py --worlds 1,8 --steps 20 --modes graph-pipe 2>&1 | grep world || exit 1
done
