#!/bin/bash
# round 5, session oo: the final committed tree -- smoke, the whole GPU suite, the default bench line with its kernel
# trace (tools/gpu_profile.sh, no PMC), the split-mode line
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5oo_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r5oo_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  r5oo_split 400 'python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r5oo_bench_split.json' \
  && NO_PMC=1 timeout -k 10 900 bash tools/gpu_profile.sh > gpurun_out/r5oo_profile.log 2>&1
rc=$?; tail -8 gpurun_out/r5oo_profile.log; exit $rc
