#!/bin/bash
# Round 6, call f: the split mode in the reference's float32 order (its GPU
# tests, the split bench line, its PMC traffic), and kernel traces of rank 0's
# W = 8 stream launch (the 8-lane chunk merge) in both arithmetics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6f
bash tools/gpu_steps.sh \
  r6f_tests 600 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_split_mode.py tests/test_gpu_split.py" \
  r6f_split 500 "python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r6f_bench_split.json" || exit $?
for v in f32 f64; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6f/$v -o run -- \
      python3 tools/stream_steps.py --worlds 8 --steps 12 --modes stream --dist $v > gpurun_out/r6f/$v.log 2>&1
  rc=$?; echo "$v trace rc=$rc"; grep world gpurun_out/r6f/$v.log
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r6f/$v.log; exit $rc; }
  python3 tools/stream_trace.py $(find gpurun_out/r6f/$v -name "run_kernel_trace.csv" | head -1) 8 > gpurun_out/r6f/${v}_overlap.txt
  head -3 gpurun_out/r6f/${v}_overlap.txt
done
timeout -k 10 900 bash tools/pmc_split.sh
