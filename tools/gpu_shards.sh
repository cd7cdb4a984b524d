#!/bin/bash
# per-rank scan time of a G-GPU striped index, timed on one GPU (rank 0's shard), by chunk size
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for w in 8 4 2; do
  for ck in 8192 4096 2048 1024; do
    echo "== world $w chunk $ck"
    timeout -k 10 200 python -u tools/prof_scan.py --no-subcluster --world $w --chunk-rows $ck 2>&1 | grep "scan ms" || exit 1
  done
done
