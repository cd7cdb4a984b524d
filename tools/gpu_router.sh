#!/bin/bash
# router parity tests + K1 kernel durations (MFMA form by query groups vs the FMA-chain form)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/rt; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -k "router or predict" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
for v in "LMI_ROUTER_QG=1" "LMI_ROUTER_QG=2" "LMI_ROUTER_QG=4" "LMI_ROUTER_FMA=1"; do
  rm -rf gpurun_out/rt/t
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rt/t -o run -- python3 tools/router_bench.py > gpurun_out/rt/out.txt 2>&1 || exit 1
  echo "== $v"; python3 tools/trace_summary.py $(find gpurun_out/rt/t -name "*kernel_trace.csv" | head -1) | grep -v calls
done
rm -rf gpurun_out/rt/t
