#!/bin/bash
# Control-flow rehearsal of the multi-rank bench on a 1-GPU box: bench.py
# launches its own two ranks (bench.launch_ranks), both on device 0, over gloo
# (RCCL refuses two ranks on one device; collectives stage through host
# memory), 1M workload.  Checks the launcher, the barriers, the all-gathers and
# the max-over-ranks clock line up: one JSON line with n_gpus 2.  The per-rank
# times are not a scaling measurement.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
LMI_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --scale 1M --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/two_ranks.json 2> gpurun_out/two_ranks.err
rc=$?
echo "two-rank bench rc=$rc"; cut -c1-600 gpurun_out/two_ranks.json; grep -v amdgpu.ids gpurun_out/two_ranks.err | tail -5
exit $rc
