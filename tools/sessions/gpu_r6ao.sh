#!/bin/bash
# Round 6, call ao (final tree: split sample skip, bitonic chunk merges; part 2): the round's profile artefacts
# (tools/gpu_profile.sh: bench line, kernel trace + timed scans, PMC traffic),
# the W = 8 projection of every rank's stripe in both arithmetics, and rank 0's
# W = 8 launch traces (float32, float64).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 bash tools/gpu_profile.sh > gpurun_out/r6ao_profile.log 2>&1
rc=$?; tail -8 gpurun_out/r6ao_profile.log; [ $rc -ne 0 ] && exit $rc
for dd in f32 f64; do
  timeout -k 10 600 python -u tools/stream_steps.py --worlds 8 --all-ranks --steps 30 --dist $dd > gpurun_out/r6ao_steps_$dd.txt 2>&1
  rc=$?; grep "ms/step" gpurun_out/r6ao_steps_$dd.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
