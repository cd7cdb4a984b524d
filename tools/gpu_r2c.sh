#!/bin/bash
# GPU parity suite (all -m gpu tests but the slow full-size module), then the float64 probe at 10M
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
    --deselect tests/test_gpu_fullsize.py > gpurun_out/t2c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/t2c.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python tools/f64_error.py --scale 10M > gpurun_out/f64_10M.json 2> gpurun_out/f64_10M.err
rc=$?; echo "f64 10M rc=$rc"; cat gpurun_out/f64_10M.json; tail -3 gpurun_out/f64_10M.err
exit $rc
