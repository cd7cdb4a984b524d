#!/bin/bash
# Batch stream (StreamedSearch) vs the per-batch step graph: the bench line both ways,
# the scan grid at 256 / 248 / 240 workgroups (LMI_SCAN_WGS: CUs left to the plan and
# finish branches), and rank 0's W = 1 / 8 steps (tools/shard_step.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/stream
for v in default no-stream wgs248 wgs240; do
  case $v in
    default) env="";; no-stream) env=""; extra="--no-stream";;
    wgs248) env="LMI_SCAN_WGS=248"; extra="";; wgs240) env="LMI_SCAN_WGS=240"; extra="";;
  esac
  [ "$v" = "default" ] && extra=""
  env $env timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --recall-sample 20 $extra \
     > gpurun_out/stream/b_$v.json 2> gpurun_out/stream/b_$v.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/stream/b_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['parity'].get('stream_vs_eager_f32'), d['step'][:40])"
done
timeout -k 10 400 python tools/shard_step.py --worlds 1,8 > gpurun_out/stream/shard.txt 2>&1 || exit $?
grep world gpurun_out/stream/shard.txt
