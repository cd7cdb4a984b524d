#!/bin/bash
# round 4, session a: the stream / graph / multi-process tests, the float64
# tests (scan lists of kF64KL entries), the two-rank gloo rehearsal of the
# bench, the default 10M bench line + its kernel trace (gpu_profile.sh without
# the PMC passes), and the memset-node repro.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_codeobj.py tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_parity.py \
    tests/test_gpu_stream.py tests/test_gpu_graph.py tests/test_gpu_dist.py > gpurun_out/r4a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r4a_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_two_ranks.sh || exit $?
NO_PMC=1 bash tools/gpu_profile.sh || exit $?
timeout -k 10 120 python -u tools/memset_graph_repro.py --rounds 10 --out gpurun_out/memset_repro.json > gpurun_out/memset_repro.log 2>&1
rc=$?; echo "memset repro rc=$rc"; cat gpurun_out/memset_repro.log; exit $rc
