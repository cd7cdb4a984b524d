#!/bin/bash
# GPU session: parity tests, then a short bench; stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/t1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/t1.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --scale 300K --R 7 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b1.json 2> gpurun_out/b1.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b1.json; tail -5 gpurun_out/b1.err
exit $rc
