#!/bin/bash
# rank 0's W=8 shard scan: chunk rows x tile order (diagnostic build: clocks, workgroup life)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for CK in 2048 1024; do
  LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 300 python tools/prof_scan.py --no-subcluster --world 8 --rank 0 \
     --chunk-rows $CK --reps 20 --abl 0 --variants "LMI_SCAN_ORDER=0|LMI_SCAN_ORDER=1|LMI_SCAN_ORDER=2|LMI_SCAN_ORDER=0|LMI_SCAN_ORDER=1" > gpurun_out/w8_$CK.log 2>&1
  rc=$?; echo "chunk $CK rc=$rc"; grep -v amdgpu.ids gpurun_out/w8_$CK.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
