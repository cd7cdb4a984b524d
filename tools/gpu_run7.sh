#!/bin/bash
# parity tests -> 10M bench -> scan ablations (v3 and the v2 ring); stop on crash/timeout
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/t7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/t7.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b7.json 2> gpurun_out/b7.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b7.json; tail -3 gpurun_out/b7.err
if [ $rc -ne 0 ]; then exit $rc; fi
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 400 python tools/prof_scan.py --abl ${ABL:-0,1,2,3} --variants "${VARIANTS:-LMI_SCAN_GROUPS=8}"
