#!/bin/bash
# round 4, session a: the stream / graph / multi-process tests, the float64
# tests (scan lists of kF64KL entries), the two-rank gloo rehearsal of the
# bench, then the default 10M bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_codeobj.py tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_parity.py \
    tests/test_gpu_stream.py tests/test_gpu_graph.py tests/test_gpu_dist.py > gpurun_out/r4a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r4a_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_two_ranks.sh || exit $?
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-1500 gpurun_out/r4a_bench.json; tail -3 gpurun_out/r4a_bench.err; exit $rc
