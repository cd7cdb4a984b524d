#!/bin/bash
# The committed tree's round artefacts in one gpurun call (rounds 5-6): smoke,
# the whole GPU suite (tie-window report), the default bench line with its
# kernel trace, timed-scan durations and PMC traffic passes
# (tools/gpu_profile.sh), the split-mode line, and the SQ counter passes of the
# product scan (tools/pmc_sq.sh).  TAG names the outputs (default r06).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T=${TAG:-r06}
bash tools/gpu_steps.sh \
  ${T}_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  ${T}_tests 1500 "LMI_TIE_REPORT=gpurun_out/${T}_ties.json python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/" \
  ${T}_split 400 "python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${T}_bench_split.json" \
  && timeout -k 10 1200 bash tools/gpu_profile.sh > gpurun_out/${T}_profile.log 2>&1
rc=$?; tail -8 gpurun_out/${T}_profile.log; exit $rc
