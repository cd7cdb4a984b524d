#!/bin/bash
# round 5, session f: band-list diagnostic on the failing test workload
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh r5f_diag 300 'python -u tools/band_diag.py'
