#!/bin/bash
# round 5, session l: achievable HBM bandwidth on the box (copy / read peak)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh r5l_peak 300 'python -u tools/hbm_peak.py && python -u tools/hbm_peak.py'
