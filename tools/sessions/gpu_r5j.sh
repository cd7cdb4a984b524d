#!/bin/bash
# round 5, session j: the tree with the float64 band lists -- smoke, whole GPU
# suite, round artefacts (tools/gpu_profile.sh), the float64 and split-mode
# bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5j_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r5j_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  r5j_bench64 600 'python -u bench.py --dist f64 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5j_bench64.json' \
  && NO_PMC=1 timeout -k 10 1200 bash tools/gpu_profile.sh > gpurun_out/r5j_profile.log 2>&1
rc=$?; tail -8 gpurun_out/r5j_profile.log; exit $rc
