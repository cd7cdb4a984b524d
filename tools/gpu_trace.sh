#!/bin/bash
# GPU parity suite, a short bench, and a kernel trace of the bench summarised per kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$TRACE_ONLY" ] || bash tools/gpu_quick.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/tr.log 2>&1
rc=$?; echo "trace rc=$rc"
if [ $rc -ne 0 ]; then tail -5 gpurun_out/tr.log; exit $rc; fi
python3 tools/trace_summary.py $(find gpurun_out/tr -name "run_kernel_trace.csv" | head -1) | tee gpurun_out/tr_summary.txt
