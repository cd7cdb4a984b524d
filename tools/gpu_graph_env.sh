#!/bin/bash
# Same-box A/B of the step forms at W = 1 and 8 (rank 0): per-batch graph with the upload
# pipelined on a copy stream, the batch stream as captured branches and as eager launches on
# three streams, with the scan on all CUs and on 248 (8 left to the side branches); twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  timeout -k 10 300 python3 tools/stream_steps.py --worlds 1,8 --steps 20 --modes graph-pipe,stream,stream-eager 2>&1 | grep world || exit 1
  LMI_SCAN_WGS=248 timeout -k 10 300 python3 tools/stream_steps.py --worlds 1,8 --steps 20 --modes graph-pipe,stream-eager 2>&1 | grep world || exit 1
done
