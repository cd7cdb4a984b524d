#!/bin/bash
# Round 6, call am: after the bitonic merges, the global band's refine four pairs a
# wave again (refine_packed_kernel) against one pair a wave (LMI_REFINE_UNPACKED=1):
# rank 0's W = 8 float64 launches alternated, then the kernel stats of both.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f64_global.py tests/test_gpu_dist.py tests/test_gpu_rccl.py > gpurun_out/r6am_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6am_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for u in 1 0; do
    LMI_REFINE_UNPACKED=$u timeout -k 10 300 python -u tools/stream_steps.py --worlds 8 --steps 30 --dist f64 \
      > gpurun_out/r6am_u${u}_$i.txt 2>&1
    rc=$?; echo "unpacked=$u run $i: $(grep 'ms/step' gpurun_out/r6am_u${u}_$i.txt)"; [ $rc -ne 0 ] && exit $rc
  done
done
for u in 1 0; do
  LMI_REFINE_UNPACKED=$u timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6am_prof_u$u -o run -- \
    python3 tools/stream_steps.py --worlds 8 --steps 30 --dist f64 > gpurun_out/r6am_prof_u$u.txt 2>&1
  rc=$?; echo "prof unpacked=$u rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
