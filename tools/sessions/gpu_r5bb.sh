#!/bin/bash
# round 5, session bb: size-aware default chunk rows -- whole GPU suite, the
# configs[1] line at its new default (1024-row chunks)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5bb_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  r5bb_300k 300 'python -u bench.py --scale 300K --R 7 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5bb_300K_R7_bench.json'
