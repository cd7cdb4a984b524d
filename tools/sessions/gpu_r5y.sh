#!/bin/bash
# round 5, session y: split-mode tests with multi-chunk samples
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5y_tests 900 "$T tests/test_gpu_split_mode.py"
