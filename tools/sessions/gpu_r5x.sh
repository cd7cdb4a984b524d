#!/bin/bash
# round 5, session x: the split mode's sample scaled with the bucket (n_c / 16
# rows past one chunk) -- its tests and bench line (roofline over both scans)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5x_tests 900 "$T tests/test_gpu_split_mode.py" \
  r5x_bench 600 'python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r5x_bench_split.json'
