#!/bin/bash
# Control-flow rehearsal of the multi-rank bench on a 1-GPU box: two ranks,
# both on device 0 (RANK 0/1, WORLD_SIZE 2, LOCAL_RANK 0), gloo (RCCL refuses
# two ranks on one device; collectives stage through host memory),
# 1M workload.  Checks the collectives line up (barriers, all-gathers, the
# max-over-ranks clock); the per-rank times are not a scaling measurement.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 WORLD_SIZE=2 LOCAL_RANK=0 LMI_DIST_BACKEND=gloo
RANK=1 timeout -k 10 300 python -u bench.py --gpus 2 --scale 1M --steps 3 --warmup 1 \
    > gpurun_out/r1.json 2> gpurun_out/r1.err &
p1=$!
RANK=0 timeout -k 10 300 python -u bench.py --gpus 2 --scale 1M --steps 3 --warmup 1 \
    > gpurun_out/r0.json 2> gpurun_out/r0.err
rc0=$?
wait $p1; rc1=$?
echo "rank0 rc=$rc0 rank1 rc=$rc1"
cut -c1-400 gpurun_out/r0.json; grep -v amdgpu.ids gpurun_out/r0.err | tail -5; grep -v amdgpu.ids gpurun_out/r1.err | tail -5
[ $rc0 -eq 0 ] && [ $rc1 -eq 0 ]
