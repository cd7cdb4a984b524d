#!/bin/bash
# scan tuning sweep: tile groups x ring lag (ablation lib), after the GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/t6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t6.log
if [ $rc -ne 0 ]; then exit $rc; fi
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 500 python tools/prof_scan.py --abl ${ABL:-0,1,2} \
  --variants "${VARIANTS:-LMI_SCAN_GROUPS=8,LMI_SCAN_LAG=0|LMI_SCAN_GROUPS=1,LMI_SCAN_LAG=0|LMI_SCAN_GROUPS=8,LMI_SCAN_LAG=1|LMI_SCAN_GROUPS=1,LMI_SCAN_LAG=1}"
