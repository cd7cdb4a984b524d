#!/bin/bash
# round 5, session h: seeded fallbacks of the float64 band lists at 10M (with
# the refine's seeded limit), K2 in float64 against the previous build; the
# batch stream with its route / plan behind the finish
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5h_diag 300 'python -u tools/band_diag10m.py' \
  r5h_f64 600 'python -u tools/f64_band_stats.py && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/f64_band_stats.py' \
  r5h_tests 600 "$T tests/test_gpu_stream.py tests/test_gpu_golden_r2.py tests/test_gpu_seed.py" \
  r5h_side 600 'python -u tools/stream_steps.py --worlds 1,8 --steps 30 --modes stream,stream-route,stream-plan,stream,stream-route,stream-plan'
