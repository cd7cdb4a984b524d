#!/bin/bash
# Round 6, call s: kth_send folded into the band chunk merge (+ band_kth_kernel,
# the fallback merge in fallback_kernel) -- the float64 / stream / RCCL / full-size
# GPU tests, then W = 8 rank-0 launches alternated float32 / float64, 60 steps each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f64_global.py tests/test_gpu_dist.py tests/test_gpu_rccl.py tests/test_gpu_parity.py \
  tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_edges.py tests/test_gpu_stream.py \
  tests/test_gpu_fullsize.py tests/test_gpu_graph.py > gpurun_out/r6s_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6s_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for dd in f32 f64; do
    timeout -k 10 300 python -u tools/stream_steps.py --worlds 8 --steps 60 --dist $dd > gpurun_out/r6s_${dd}_$i.txt 2>&1
    rc=$?; grep "ms/step" gpurun_out/r6s_${dd}_$i.txt; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
