#!/bin/bash
# round 5, session v: the float64 fallback in row slices over many workgroups
# -- float64 tests, K2 in float64 at 300K / 10M
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5v_tests 900 "$T tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_seed.py tests/test_gpu_parity.py tests/test_gpu_wide.py" \
  r5v_f64 600 'python -u tools/f64_band_stats.py --n 300000 --R 7 && python -u tools/f64_band_stats.py'
