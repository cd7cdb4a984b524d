#!/bin/bash
# seeding ceiling: scan time / candidate counters with fresh vs kept (near-final) per-pair bounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 300 python -u tools/prof_scan.py --no-subcluster --abl 0,7,1 --variants "LMI_SCAN_GROUPS=8|LMI_SCAN_KEEP_THR=1" 2>&1 | grep -v amdgpu.ids
