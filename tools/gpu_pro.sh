#!/bin/bash
# tile prologue A/B: block 0's DMA before (new) vs after (prev) the query-fragment loads, chunks 8192 / 4096
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for CK in 8192 4096; do
  for L in liblmi_hip_prev.so liblmi_hip_abl.so liblmi_hip_prev.so liblmi_hip_abl.so; do
    LMI_LIB_NAME=$L timeout -k 10 300 python tools/prof_scan.py --no-subcluster --chunk-rows $CK --reps 10 --abl 0 > gpurun_out/pro.log 2>&1
    rc=$?; echo "chunk $CK $L rc=$rc"; grep -v amdgpu.ids gpurun_out/pro.log | grep -v "^\[gpurun"; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_codeobj.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tpro.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tpro.log; exit $rc
