#!/bin/bash
# GPU parity suite then a short 10M bench (no CPU baseline); stops at the first failure
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/tq.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/tq.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bq.json 2> gpurun_out/bq.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bq.json; tail -3 gpurun_out/bq.err
exit $rc
