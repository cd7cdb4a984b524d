#!/bin/bash
# round 2: GPU parity suite (incl. float64 fixtures), then the float64 error/speed probe at 1M and 10M
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
# timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/t2a.log 2>&1
rc=0
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/f64_error.py --scale 1M > gpurun_out/f64_1M.json 2> gpurun_out/f64_1M.err
rc=$?; echo "f64 1M rc=$rc"; cat gpurun_out/f64_1M.json; tail -3 gpurun_out/f64_1M.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python tools/f64_error.py --scale 10M > gpurun_out/f64_10M.json 2> gpurun_out/f64_10M.err
rc=$?; echo "f64 10M rc=$rc"; cat gpurun_out/f64_10M.json; tail -3 gpurun_out/f64_10M.err
exit $rc
