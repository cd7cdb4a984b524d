#!/bin/bash
# Round 6, call an: the packed refine A/B again, longer and in both orders
# (p u u p p u u p): rank 0's W = 8 float64 launches, 40 steps each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for u in 0 1 1 0 0 1 1 0; do
  i=$((i+1))
  LMI_REFINE_UNPACKED=$u timeout -k 10 300 python -u tools/stream_steps.py --worlds 8 --steps 40 --dist f64 \
    > gpurun_out/r6an_${i}_u$u.txt 2>&1
  rc=$?; echo "unpacked=$u run $i: $(grep 'ms/step' gpurun_out/r6an_${i}_u$u.txt)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
