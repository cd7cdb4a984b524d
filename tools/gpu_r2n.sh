#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_golden.py tests/test_gpu_golden_r2.py tests/test_gpu_graph.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/t2n.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t2n.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_replay_abl.sh
