#!/bin/bash
# round 5, session cc: the configs[1] line at the size-aware default (4096-row chunks at 300K)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5cc_300k 300 'python -u bench.py --scale 300K --R 7 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5cc_300K_R7_bench.json'
