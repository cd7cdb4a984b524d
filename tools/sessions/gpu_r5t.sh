#!/bin/bash
# round 5, session t: the float64 band lists' fallbacks at 300K (R = 7)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh r5t_diag 300 'python -u tools/band_diag10m.py --n 300000 --R 7'
