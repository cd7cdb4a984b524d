#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py -x -q -rf --timeout 600 --timeout-method thread > gpurun_out/t2p.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t2p.log; [ $rc -ne 0 ] && exit $rc
WORLDS=8 STEPS=20 bash tools/gpu_step_trace.sh
