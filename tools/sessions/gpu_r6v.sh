#!/bin/bash
# Round 6, call v (final tree, part 1): smoke, the whole GPU suite with the
# tie-window report, the default bench line and the split-mode line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6v_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r6v_tests 900 "LMI_TIE_REPORT=gpurun_out/r6v_ties.json python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/" \
  r6v_bench 400 "python -u bench.py > gpurun_out/r6v_bench.json" \
  r6v_split 400 "python -u bench.py --corpus f32 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6v_bench_split.json"
rc=$?; tail -12 gpurun_out/r6v_tests.log; cut -c1-300 gpurun_out/r6v_bench.json; echo; cut -c1-300 gpurun_out/r6v_bench_split.json; exit $rc
