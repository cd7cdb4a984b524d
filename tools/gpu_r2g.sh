#!/bin/bash
# pipelined graphs (tests + bench) and the fixed DMA-interleave A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/t2g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t2g.log
[ $rc -ne 0 ] && exit $rc
ABLS=0,54,56,0,54,56 bash tools/gpu_ilv.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b2g.json 2> gpurun_out/b2g.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/b2g.json'));print(d['value'],d['step'],d['ms_per_step'],d['ms_per_step_serial'],d['roofline']['kernel_ms'],d['other_dist'],d['breakdown_ms'])"; grep -v amdgpu.ids gpurun_out/b2g.err | tail -3
exit $rc
