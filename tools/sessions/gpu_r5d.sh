#!/bin/bash
# round 5, session d: the committed tree's smoke, whole GPU suite and round
# artefacts (tools/gpu_profile.sh: bench line, kernel trace + stats, PMC traffic)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5d_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r5d_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  && timeout -k 10 1500 bash tools/gpu_profile.sh > gpurun_out/r5d_profile.log 2>&1
rc=$?; tail -12 gpurun_out/r5d_profile.log; exit $rc
