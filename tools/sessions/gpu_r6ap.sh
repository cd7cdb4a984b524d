#!/bin/bash
# Round 6, call ap (the final tree with the bitonic chunk merges, part 1): smoke, the whole GPU suite with the
# tie-window report, the default bench line and the split-mode line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6ap_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r6ap_tests 900 "LMI_TIE_REPORT=gpurun_out/r6ap_ties.json python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/" \
  r6ap_bench 400 "python -u bench.py > gpurun_out/r6ap_bench.json" \
  r6ap_split 400 "python -u bench.py --corpus f32 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6ap_bench_split.json"
rc=$?; tail -12 gpurun_out/r6ap_tests.log; cut -c1-300 gpurun_out/r6ap_bench.json; echo; cut -c1-300 gpurun_out/r6ap_bench_split.json; exit $rc
