#!/bin/bash
# round 5, session ff: the batch stream's streams on distinct hardware queues (li.stream.queue_streams) --
# stream / graph / multi-process tests, then the default bench line and its kernel trace (no PMC)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5ff_focus 900 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream.py tests/test_gpu_graph.py tests/test_gpu_dist.py' \
  && NO_PMC=1 timeout -k 10 900 bash tools/gpu_profile.sh > gpurun_out/r5ff_profile.log 2>&1
rc=$?; tail -8 gpurun_out/r5ff_profile.log; exit $rc
