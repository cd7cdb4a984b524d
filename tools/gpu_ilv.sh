#!/bin/bash
# A/B of the DMA placement variants (diagnostic build, one box, calibration first and last)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 400 python tools/prof_scan.py --no-subcluster --check --reps 10 \
   --abl ${ABLS:-0,54,55,56,0} > gpurun_out/ilv.log 2>&1
rc=$?; cat gpurun_out/ilv.log | grep -v amdgpu.ids; exit $rc
