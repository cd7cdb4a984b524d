#!/bin/bash
# round 5, session z: the stream with the finish and the next scan enqueued
# before the launch's route and plan (scan_first) -- its tests, A/B at W = 1 / 8
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5z_tests 600 "$T tests/test_gpu_stream.py" \
  r5z_steps 900 'python -u tools/stream_steps.py --worlds 1,8 --steps 30 --modes stream,stream-sf,stream,stream-sf,stream,stream-sf'
