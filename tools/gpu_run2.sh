#!/bin/bash
# 10M bench (default config) + rocprofv3 kernel-trace stats of a short run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/b2.json 2> gpurun_out/b2.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b2.json; tail -8 gpurun_out/b2.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --recall-sample 20 > gpurun_out/p2.json 2> gpurun_out/p2.err
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof2 -name "*stats*" | head; 
f=$(find gpurun_out/prof2 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-220 "$f" | head -20
exit $rc
