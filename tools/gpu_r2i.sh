#!/bin/bash
# GPU suite, the zeroed-dead-column A/B (ABL 57 = round 1's query-0 fragments),
# the W=8 step trace (fixed costs) and the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/t2i.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t2i.log; [ $rc -ne 0 ] && exit $rc
ABLS=0,57,0,57 bash tools/gpu_ilv.sh || exit $?
WORLDS=8 STEPS=20 bash tools/gpu_step_trace.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b2i.json 2> gpurun_out/b2i.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/b2i.json'));print(d['value'],d['ms_per_step'],d['ms_per_step_serial'],d['roofline']['kernel_ms'],d['other_dist'],d['breakdown_ms'])"; grep -v amdgpu.ids gpurun_out/b2i.err | tail -3
exit $rc
