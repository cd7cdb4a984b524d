#!/bin/bash
# round 5, session a: the split mode's parity tests; search.py --gpus G through
# the reference interface (gloo ranks on the box's GPU); the cross-rank bound
# study (diagnostic build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_steps.sh \
  r5a_split 600 'python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_split_mode.py' \
  r5a_cli 900 'python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_cli_dist.py' \
  r5a_bound 600 'LMI_LIB_NAME=liblmi_hip_abl.so python -u tools/bound_study.py --abl7'
