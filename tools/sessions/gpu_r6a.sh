#!/bin/bash
# Round 6, call a: the new GPU tests (forced RCCL exchange, stream lifetime,
# split-mode sub-clusters), the bench under LMI_FORCE_EXCHANGE=1, and the SQ
# counter passes of the product scan.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_rccl.py tests/test_gpu_stream.py tests/test_gpu_split_mode.py > gpurun_out/r6a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6a_tests.log; [ $rc -ne 0 ] && exit $rc
LMI_FORCE_EXCHANGE=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r6a_bench_fx.json 2> gpurun_out/r6a_bench_fx.err
rc=$?; cut -c1-300 gpurun_out/r6a_bench_fx.json; tail -3 gpurun_out/r6a_bench_fx.err; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_sq.sh
