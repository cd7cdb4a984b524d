#!/bin/bash
# round 5, session aa: configs[1] (300K, R = 7) at chunk_rows 1024 / 2048 / 4096 / 8192
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
for c in 1024 2048 4096 8192; do
  bash tools/gpu_steps.sh r5aa_$c 300 "python -u bench.py --scale 300K --R 7 --no-cpu-baseline --no-single --steps 20 --warmup 5 --chunk-rows $c > gpurun_out/r5aa_300K_$c.json" || exit $?
done
