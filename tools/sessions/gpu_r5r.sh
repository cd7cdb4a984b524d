#!/bin/bash
# round 5, session r: configs[1] (300K, R = 7) and configs[4] on one GPU
# (100M random unit vectors, 154 GB fp16) with the round-5 tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5r_300k 600 'python -u bench.py --scale 300K --R 7 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5r_300K_R7_bench.json' \
  r5r_100m 900 'python -u bench.py --scale 100M --no-cpu-baseline --steps 5 --warmup 2 --recall-sample 50 > gpurun_out/r5r_100M_bench.json'
