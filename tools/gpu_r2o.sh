#!/bin/bash
# r2l (suite, smoke, two ranks, shard steps) + the default bench line without the CPU baseline
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash tools/gpu_r2l.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b2o.json 2> gpurun_out/b2o.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/b2o.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['breakdown_ms'])"; exit $rc
