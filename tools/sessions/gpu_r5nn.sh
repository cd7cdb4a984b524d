#!/bin/bash
# round 5, session nn: replay_merge_kernel without its by-reference lambda (40 B of stack per thread -> none): replay
# tests, then the W = 8 rank-0 stream step and the default bench line, against the previous build (liblmi_hip_prev.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5nn_tests 600 "$T tests/test_gpu_replay.py tests/test_gpu_stream.py" \
  r5nn_ab 900 'for lib in liblmi_hip_prev.so liblmi_hip.so liblmi_hip_prev.so liblmi_hip.so; do LMI_LIB_NAME=$lib python -u tools/stream_steps.py --worlds 1,8 --steps 40 --modes stream | grep ms/step | sed "s/^/$lib /" || exit 1; done'
