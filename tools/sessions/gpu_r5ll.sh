#!/bin/bash
# round 5, session ll: the committed tree after the refine occupancy change -- smoke, the whole GPU suite, the
# default bench line with its kernel trace (tools/gpu_profile.sh, no PMC), configs[1] (300K, R=7)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5ll_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r5ll_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  r5ll_300k 400 'python -u bench.py --scale 300K --R 7 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5ll_300K_R7_bench.json' \
  && NO_PMC=1 timeout -k 10 900 bash tools/gpu_profile.sh > gpurun_out/r5ll_profile.log 2>&1
rc=$?; tail -8 gpurun_out/r5ll_profile.log; exit $rc
