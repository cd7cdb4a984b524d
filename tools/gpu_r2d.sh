#!/bin/bash
# GPU suite (minus the full-size module) + the default bench line (with its CPU baseline)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
    --deselect tests/test_gpu_fullsize.py > gpurun_out/t2d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t2d.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python bench.py > gpurun_out/b2d.json 2> gpurun_out/b2d.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b2d.json; grep -v amdgpu.ids gpurun_out/b2d.err | tail -3
exit $rc
