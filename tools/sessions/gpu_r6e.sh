#!/bin/bash
# Round 6, call e: the chunk merge at 8 lanes per pair and thread-local
# captures -- the GPU tests that cover the merge (parity, fixtures, stream,
# dist, graph, fullsize, f64 global, rccl), the default bench (W = 1), and the
# W = 8 projection in both arithmetics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6e_tests 900 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_stream.py tests/test_gpu_dist.py tests/test_gpu_graph.py tests/test_gpu_f64_global.py tests/test_gpu_rccl.py tests/test_gpu_fullsize.py tests/test_gpu_split_mode.py tests/test_gpu_seed.py" \
  r6e_bench 500 "python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6e_bench.json" \
  r6e_steps32 600 "python tools/stream_steps.py --worlds 8 --all-ranks --dist f32 --steps 20 > gpurun_out/r6e_steps_f32.txt" \
  r6e_steps64 600 "python tools/stream_steps.py --worlds 8 --all-ranks --dist f64 --steps 20 > gpurun_out/r6e_steps_f64.txt"
rc=$?; grep -h "ms/step" gpurun_out/r6e_steps_f*.txt; cut -c1-200 gpurun_out/r6e_bench.json; exit $rc
