#!/bin/bash
# round 5, session c: the replay group kernel (distances kept in LDS, one
# block reduction) against the previous build on the bench's own lists; its
# tests; the W = 8 step and trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5c_tests 600 "$T tests/test_gpu_replay.py tests/test_gpu_golden.py tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py" \
  r5c_rb 600 'python -u tools/replay_bench.py --bench-lists && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/replay_bench.py --bench-lists && python -u tools/replay_bench.py --bench-lists' \
  r5c_rbtrace 600 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5c_rbtrace -o run -- python3 tools/replay_bench.py --bench-lists' \
  r5c_steps 600 'python -u tools/stream_steps.py --worlds 1,8 --steps 30 --modes stream && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/stream_steps.py --worlds 8 --steps 30 --modes stream && python -u tools/stream_steps.py --worlds 8 --steps 30 --modes stream'
