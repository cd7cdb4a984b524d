#!/bin/bash
# round 4, session a: the stream / graph / multi-process tests, the two-rank
# gloo rehearsal of the bench, then the default 10M bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_stream.py tests/test_gpu_graph.py tests/test_gpu_dist.py > gpurun_out/r4a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r4a_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_two_ranks.sh || exit $?
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-1500 gpurun_out/r4a_bench.json; tail -3 gpurun_out/r4a_bench.err; exit $rc
