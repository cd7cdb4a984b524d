#!/bin/bash
# parity tests -> 10M bench -> rocprofv3 kernel stats (csv); stop on crash/timeout
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/t3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/t3.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b3.json 2> gpurun_out/b3.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b3.json; tail -4 gpurun_out/b3.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --recall-sample 20 > gpurun_out/p3.json 2> gpurun_out/p3.err
rc=$?; echo "rocprof rc=$rc"
f=$(find gpurun_out/prof3 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-200 "$f" | head -20
exit $rc
