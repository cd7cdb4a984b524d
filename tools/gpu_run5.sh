#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/t5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t5.log
if [ $rc -ne 0 ]; then exit $rc; fi
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 400 python tools/prof_scan.py --abl 0,1,2,3
