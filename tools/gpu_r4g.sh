#!/bin/bash
# round 4: smoke() and the whole GPU suite at the current tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4g
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4g/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; grep -v amdgpu.ids gpurun_out/r4g/smoke.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4g/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r4g/tests.log; exit $rc
