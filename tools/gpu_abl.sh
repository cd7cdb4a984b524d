#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 400 python tools/prof_scan.py --abl 0,1,2,3
