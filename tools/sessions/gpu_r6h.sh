#!/bin/bash
# Round 6, call h: per-kernel times of the split mode (both arithmetics are
# timed by one bench run), to price the reference-order float32 re-score.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6h_split 500 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6h -o run -- python3 bench.py --corpus f32 --no-cpu-baseline --no-single --steps 5 --warmup 2"
rc=$?
s=$(ls gpurun_out/r6h/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$s" ] && cut -d, -f1-5 "$s" | cut -c1-200 | head -30
exit $rc
