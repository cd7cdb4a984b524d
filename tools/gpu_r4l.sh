#!/bin/bash
# round 4: the float64 refinement's batched row loads -- its parity tests, then
# the bench line + kernel trace (tools/gpu_profile.sh without PMC)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4l
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_wide.py tests/test_gpu_stream.py \
   tests/test_gpu_fullsize.py > gpurun_out/r4l/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4l/tests.log; [ $rc -ne 0 ] && exit $rc
NO_PMC=1 bash tools/gpu_profile.sh
