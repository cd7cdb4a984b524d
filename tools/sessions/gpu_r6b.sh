#!/bin/bash
# Round 6, call b: the new GPU tests (forced RCCL exchange, float64 global
# band, stream lifetime, split-mode sub-clusters, the gloo ranks), the bench
# under LMI_FORCE_EXCHANGE=1, the W = 8 projection (f32 / f64 global band),
# and the SQ counter passes of the product scan.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_rccl.py tests/test_gpu_f64_global.py tests/test_gpu_stream.py tests/test_gpu_dist.py \
  tests/test_gpu_split_mode.py tests/test_gpu_graph.py > gpurun_out/r6b_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6b_tests.log; [ $rc -ne 0 ] && exit $rc
LMI_FORCE_EXCHANGE=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r6b_bench_fx.json 2> gpurun_out/r6b_bench_fx.err
rc=$?; cut -c1-300 gpurun_out/r6b_bench_fx.json; tail -3 gpurun_out/r6b_bench_fx.err; [ $rc -ne 0 ] && exit $rc
for dd in f32 f64; do
  timeout -k 10 600 python tools/stream_steps.py --worlds 8 --all-ranks --dist $dd --steps 20 \
    > gpurun_out/r6b_steps_$dd.txt 2>&1
  rc=$?; grep "ms/step" gpurun_out/r6b_steps_$dd.txt; [ $rc -ne 0 ] && { tail -5 gpurun_out/r6b_steps_$dd.txt; exit $rc; }
done
bash tools/pmc_sq.sh
