#!/bin/bash
# round 5, session p: the split mode's first scan on a per-bucket sample (k <= 10; sampled chunk lists for k <= 15) --
# its tests, the split-mode bench line against the previous build
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5p_tests 900 "$T tests/test_gpu_split_mode.py tests/test_gpu_golden_r2.py tests/test_gpu_wide.py" \
  r5p_bench 900 'python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r5p_bench_split.json && LMI_LIB_NAME=liblmi_hip_prev.so python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r5p_bench_split_prev.json'
