#!/bin/bash
# tail-only light-tile moves: LMI_SCAN_ORDER 3 (tiles under 1/4 of a full one to the queue tail), 4 (under 1/8) vs 0
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 400 python tools/prof_scan.py --no-subcluster --check --reps 10 --abl 0 \
   --variants "LMI_SCAN_ORDER=0|LMI_SCAN_ORDER=3|LMI_SCAN_ORDER=4|LMI_SCAN_ORDER=0|LMI_SCAN_ORDER=3|LMI_SCAN_ORDER=4" > gpurun_out/order2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/order2.log; exit $rc
