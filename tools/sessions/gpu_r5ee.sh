#!/bin/bash
# round 5, session ee: GraphedSearch.stream (batch i + 1 staged and uploaded beside batch i's step) and
# the one-wave-per-pair x_select for the split mode -- their tests first, smoke, the split-mode bench
# line (graph step), then the whole GPU suite and the round artefacts (tools/gpu_profile.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5ee_focus 600 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_graph.py tests/test_gpu_split_mode.py' \
  && bash tools/gpu_steps.sh \
  r5ee_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r5ee_split 600 'python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r5ee_bench_split.json' \
  r5ee_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  && timeout -k 10 1500 bash tools/gpu_profile.sh > gpurun_out/r5ee_profile.log 2>&1
rc=$?; tail -8 gpurun_out/r5ee_profile.log; exit $rc
