#!/bin/bash
# Round 6, call o: the finish chain beside the next scan -- the W = 1 / W = 8
# (rank 0) stream launches with the scan's grid at every CU (the product) and
# with CUs left free for the finish (LMI_SCAN_WGS) and the lookahead scan not
# waiting for the finish (LMI_STREAM_OVERLAP=1), float32 and float64.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u tools/stream_steps.py --worlds 1,8 --steps 30 --dist $DD > gpurun_out/r6o_$n.txt 2>&1
  local rc=$?; echo "== $n rc=$rc"; grep "ms/step" gpurun_out/r6o_$n.txt; return $rc
}
DD=f32 run f32_base LMI_STREAM_OVERLAP=0 || exit $?
DD=f32 run f32_ov240 LMI_STREAM_OVERLAP=1 LMI_SCAN_WGS=240 || exit $?
DD=f32 run f32_ov248 LMI_STREAM_OVERLAP=1 LMI_SCAN_WGS=248 || exit $?
DD=f32 run f32_ov224 LMI_STREAM_OVERLAP=1 LMI_SCAN_WGS=224 || exit $?
DD=f64 run f64_base LMI_STREAM_OVERLAP=0 || exit $?
DD=f64 run f64_ov240 LMI_STREAM_OVERLAP=1 LMI_SCAN_WGS=240 || exit $?
