#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
LMI_LIB_NAME=liblmi_hip_abl.so ABLS=0,1,2,3,0 timeout -k 10 300 python tools/replay_bench.py --bench-lists > gpurun_out/rabl.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/rabl.log; exit $rc
