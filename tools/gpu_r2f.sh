#!/bin/bash
# Round-2 re-entry check: the whole GPU suite, smoke(), the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
    > gpurun_out/t2f.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t2f.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2f.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/s2f.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py > gpurun_out/b2f.json 2> gpurun_out/b2f.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b2f.json; grep -v amdgpu.ids gpurun_out/b2f.err | tail -3
exit $rc
