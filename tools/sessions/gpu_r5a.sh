#!/bin/bash
# round 5, session a: the split mode's parity tests; the phased / fused replay
# and the batch stream on it (one process and 2-3 gloo ranks); search.py
# --gpus G through the reference interface; the cross-rank bound study
# (diagnostic build); the W = 8 stream trace and the step times at W = 1 / 8
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5a_tests 900 "$T tests/test_gpu_split_mode.py tests/test_gpu_replay.py tests/test_gpu_stream.py tests/test_gpu_dist.py" \
  r5a_cli 900 'python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_cli_dist.py' \
  r5a_bound 600 'LMI_LIB_NAME=liblmi_hip_abl.so python -u tools/bound_study.py --abl7' \
  r5a_steps 600 'python -u tools/stream_steps.py --worlds 1,8 --steps 30 --modes stream' \
  r5a_strace 600 'WGSS=0 WORLDS=8 bash tools/gpu_stream_trace.sh'
