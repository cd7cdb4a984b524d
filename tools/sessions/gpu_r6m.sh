#!/bin/bash
# Round 6, call m: the split mode's phases and batch stream (ABI 11) -- the
# split / stream GPU tests, the split bench line (now the batch stream), and
# the kernel trace of the same run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6m_tests 600 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_split_stream.py tests/test_gpu_split_mode.py tests/test_gpu_split.py tests/test_gpu_stream.py" \
  r6m_split 500 "python -u bench.py --corpus f32 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6m_bench_split.json" \
  r6m_trace 500 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6m -o run -- python3 bench.py --corpus f32 --no-cpu-baseline --no-single --steps 5 --warmup 2"
rc=$?; grep -A8 "by (side" gpurun_out/r6m_tests.log; cut -c1-300 gpurun_out/r6m_bench_split.json; exit $rc
