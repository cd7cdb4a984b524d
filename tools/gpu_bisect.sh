#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for L in liblmi_hip.so liblmi_hip_A.so liblmi_hip_B.so; do
  LMI_LIB_NAME=$L timeout -k 10 200 python -u -m pytest "tests/test_gpu_parity.py::test_bucket_topk_matches_oracle" -q -rf --timeout 120 --timeout-method thread > gpurun_out/bis_$L.log 2>&1
  echo "$L rc=$?"; tail -3 gpurun_out/bis_$L.log
done
