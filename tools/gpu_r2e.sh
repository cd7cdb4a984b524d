#!/bin/bash
# graph tests + bench (graph replay) + eager bench for comparison
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_golden_r2.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/t2e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/t2e.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b2e.json 2> gpurun_out/b2e.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/b2e.json; python3 -c "import json;d=json.load(open('gpurun_out/b2e.json'));print(d['step'],d['ms_per_step'],d['roofline']['kernel_ms'],d['other_dist'],d['breakdown_ms'])"; grep -v amdgpu.ids gpurun_out/b2e.err | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph > gpurun_out/b2e_eager.json 2> gpurun_out/b2e_eager.err
rc=$?; python3 -c "import json;d=json.load(open('gpurun_out/b2e_eager.json'));print(d['step'],d['ms_per_step'],d['roofline']['kernel_ms'],d['other_dist'])"
exit $rc
