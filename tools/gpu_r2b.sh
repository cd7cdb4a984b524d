#!/bin/bash
# round 2: full-size parity (configs[1], configs[2]) + the two-rank launcher rehearsal
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -x -v -rf --timeout 600 --timeout-method thread > gpurun_out/t2b.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/t2b.log | head -30; tail -5 gpurun_out/t2b.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_two_ranks.sh
