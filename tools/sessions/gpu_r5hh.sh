#!/bin/bash
# round 5, session hh: the one-GPU W = 8 projection with the stream-queue change (every rank's stripe in turn;
# round 4's ranks spread 1.21-1.42 ms per launch), float32 and float64
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5hh_steps 700 'python -u tools/stream_steps.py --worlds 1,8 --all-ranks --steps 30 --modes stream' \
  r5hh_steps64 500 'python -u tools/stream_steps.py --worlds 8 --steps 30 --modes stream --dist f64'
