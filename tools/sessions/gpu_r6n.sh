#!/bin/bash
# Round 6, call n (a new session of the round): the committed tree after the
# split-mode batch stream -- smoke, the whole GPU suite with the tie-window
# report, the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6n_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r6n_tests 900 "LMI_TIE_REPORT=gpurun_out/r6n_ties.json python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/" \
  r6n_bench 400 "python -u bench.py > gpurun_out/r6n_bench.json"
rc=$?; tail -12 gpurun_out/r6n_tests.log; cut -c1-400 gpurun_out/r6n_bench.json; exit $rc
