#!/bin/bash
# Round 6, call z: the replay's group kernel with one fused workgroup reduction
# (sum, min, max) and its first-pass list entries kept in registers for the B_q
# writes -- the replay / golden / stream GPU tests, then the replay alone on the
# bench's lists (tools/replay_bench.py --bench-lists) against the previous
# build (li/liblmi_hip_base.so), and the 300K R = 7 bench line, alternated.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_replay.py tests/test_gpu_golden.py tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py \
  tests/test_gpu_stream.py tests/test_gpu_edges.py > gpurun_out/r6z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6z_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in liblmi_hip_base.so liblmi_hip.so; do
    LMI_LIB_NAME=$lib timeout -k 10 300 python -u tools/replay_bench.py --bench-lists > gpurun_out/r6z_replay_${lib}_$i.txt 2>&1
    rc=$?; grep "us$" gpurun_out/r6z_replay_${lib}_$i.txt; [ $rc -ne 0 ] && exit $rc
  done
done
for i in 1 2; do
  for lib in liblmi_hip_base.so liblmi_hip.so; do
    LMI_LIB_NAME=$lib timeout -k 10 300 python -u bench.py --scale 300K --R 7 --no-cpu-baseline --steps 30 --warmup 5 \
      > gpurun_out/r6z_300K_${lib}_$i.json 2> gpurun_out/r6z_300K_${lib}_$i.err
    rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6z_300K_${lib}_$i.json')); print('300K $lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['other_dist']['ms_per_step'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
