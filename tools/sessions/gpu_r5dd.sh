#!/bin/bash
# round 5, session dd: the committed tree after the size-aware chunk default -- smoke, whole GPU
# suite, round artefacts (tools/gpu_profile.sh: default bench line, kernel trace, PMC traffic)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5dd_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r5dd_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  && timeout -k 10 1500 bash tools/gpu_profile.sh > gpurun_out/r5dd_profile.log 2>&1
rc=$?; tail -8 gpurun_out/r5dd_profile.log; exit $rc
