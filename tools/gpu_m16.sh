#!/bin/bash
# MFMA shape probe: 6 / 66 (MFMA + A-reads, 32x32x16 / 16x16x32), 67 / 68 (full kernel minus the epilogue)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 400 python tools/prof_scan.py --no-subcluster --reps 10 --abl 6,66,67,68,0,6,66,67,68 > gpurun_out/m16.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/m16.log; exit $rc
