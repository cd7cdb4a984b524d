#!/bin/bash
# GPU suite (packed K3 path included), smoke, the two-rank launcher rehearsal, rank-0 shard steps at W=1, 8
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/t2l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t2l.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2l.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/s2l.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_two_ranks.sh || exit $?
timeout -k 10 400 python tools/shard_step.py --worlds 1,8 > gpurun_out/shard_step.txt 2> gpurun_out/shard_step.err
rc=$?; echo "shard_step rc=$rc"; cat gpurun_out/shard_step.txt; exit $rc
