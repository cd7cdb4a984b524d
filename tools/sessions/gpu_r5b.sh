#!/bin/bash
# round 5, session b: the replay (last merge writes the answer, groups beside
# the scan) through its tests and the stream / dist tests; search.py --gpus G;
# the W = 8 stream trace and step times; the default bench line; the split
# mode's 10M bench line (--corpus f32)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5b_tests 900 "$T tests/test_gpu_replay.py tests/test_gpu_stream.py tests/test_gpu_dist.py tests/test_h5.py" \
  r5b_cli 900 'python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_cli_dist.py' \
  r5b_steps 600 'python -u tools/stream_steps.py --worlds 1,8 --steps 30 --modes stream' \
  r5b_strace 600 'WGSS=0 WORLDS=8 bash tools/gpu_stream_trace.sh' \
  r5b_bench 600 'python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5b_bench.json' \
  r5b_split 900 'python -u bench.py --corpus f32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5b_split.json'
