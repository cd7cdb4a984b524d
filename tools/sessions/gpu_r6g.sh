#!/bin/bash
# Round 6, call g: the split mode's float32 order with the ballot tail flags:
# its GPU tests and the split bench line (both arithmetics).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6g_tests 600 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_split_mode.py tests/test_gpu_split.py tests/test_gpu_golden_r2.py" \
  r6g_split 500 "python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r6g_bench_split.json"
rc=$?; grep -A6 "by (side" gpurun_out/r6g_tests.log; cut -c1-300 gpurun_out/r6g_bench_split.json; exit $rc
