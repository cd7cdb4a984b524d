#!/bin/bash
# replay tests + W=8 step trace (replay_group after the 16-entry register share) + bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_golden.py tests/test_gpu_graph.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/t2j.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t2j.log; [ $rc -ne 0 ] && exit $rc
WORLDS=8 STEPS=20 bash tools/gpu_step_trace.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --pipeline > gpurun_out/b2j.json 2> gpurun_out/b2j.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/b2j.json'));print(d['value'],d['ms_per_step'],d['ms_per_step_serial'],d['roofline']['kernel_ms'],d['breakdown_ms'])"
exit $rc
