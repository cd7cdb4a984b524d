#!/bin/bash
# Kernel traces of the batch stream at W = 1 and W = 8 (rank 0's stripe): do the plan / finish
# branches run inside the scan?  (tools/stream_trace.py), for scan grids of all CUs and fewer
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/strace
for WGS in ${WGSS:-0 248}; do
  if [ "$WGS" = "0" ]; then unset LMI_SCAN_WGS; else export LMI_SCAN_WGS=$WGS; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/strace/w$WGS -o run -- \
      python3 tools/stream_steps.py --worlds ${WORLDS:-1,8} --steps 12 --modes stream $EXTRA > gpurun_out/strace/w$WGS.log 2>&1
  rc=$?; echo "WGS=$WGS trace rc=$rc"; grep world gpurun_out/strace/w$WGS.log
  [ $rc -ne 0 ] && exit $rc
  python3 tools/stream_trace.py $(find gpurun_out/strace/w$WGS -name "run_kernel_trace.csv" | head -1) 30 > gpurun_out/strace/w${WGS}_overlap.txt
  tail -4 gpurun_out/strace/w${WGS}_overlap.txt; sed -n 1,3p gpurun_out/strace/w${WGS}_overlap.txt
done
