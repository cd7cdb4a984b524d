#!/bin/bash
# k > 16 bound + collect path: its own tests, then the existing k > 16 / float64
# parity tests that now run through it.  Logs under gpurun_out/wide/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wide
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_wide.py > gpurun_out/wide/wide.log 2>&1
rc=$?; echo "wide rc=$rc"; tail -5 gpurun_out/wide/wide.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_golden_r2.py tests/test_gpu_split.py tests/test_gpu_parity.py > gpurun_out/wide/k16.log 2>&1
rc=$?; echo "k16 rc=$rc"; tail -5 gpurun_out/wide/k16.log; exit $rc
