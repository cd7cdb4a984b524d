#!/bin/bash
# round 5, session k: the replay's group kernels with 256-thread workgroups
# (was 1024) against the previous build -- replay tests, replay_bench, the
# stream at W = 1 / 8
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5k_tests 600 "$T tests/test_gpu_replay.py tests/test_gpu_golden.py tests/test_gpu_golden_r2.py tests/test_gpu_stream.py" \
  r5k_rb 600 'python -u tools/replay_bench.py --bench-lists && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/replay_bench.py --bench-lists' \
  r5k_steps 600 'python -u tools/stream_steps.py --worlds 1,8 --steps 30 && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/stream_steps.py --worlds 1,8 --steps 30 && python -u tools/stream_steps.py --worlds 1,8 --steps 30 && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/stream_steps.py --worlds 1,8 --steps 30'
