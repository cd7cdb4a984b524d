#!/bin/bash
# round 5, session q: split-mode tests with k = 12 (the sampled chunk-list bound), golden r5
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5q_tests 900 "$T tests/test_gpu_split_mode.py"
