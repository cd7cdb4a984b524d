#!/bin/bash
# Round 6, call j: the split mode, a lane per K block on the normalised rows
# (ABI 11, corpus32n): its GPU tests, the split bench line, and the kernel
# trace of the same run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6j_tests 600 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_split_mode.py tests/test_gpu_split.py" \
  r6j_split 500 "python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r6j_bench_split.json" \
  r6j_trace 500 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6j -o run -- python3 bench.py --corpus f32 --no-cpu-baseline --no-single --steps 5 --warmup 2"
rc=$?; grep -A8 "by (side" gpurun_out/r6j_tests.log; cut -c1-300 gpurun_out/r6j_bench_split.json; exit $rc
