#!/bin/bash
# round 5, session u: band lists with each lane's smallest dropped distance as
# its bound (instead of its 10th) -- float64 tests, K2 in float64 at 300K and
# 10M against the pre-band build
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5u_tests 900 "$T tests/test_codeobj.py tests/test_gpu_golden_r2.py tests/test_gpu_golden_r3.py tests/test_gpu_seed.py tests/test_gpu_parity.py tests/test_gpu_stream.py" \
  r5u_f64 600 'python -u tools/f64_band_stats.py --n 300000 --R 7 && LMI_LIB_NAME=liblmi_hip_preband.so python -u tools/f64_band_stats.py --n 300000 --R 7 && python -u tools/f64_band_stats.py && LMI_LIB_NAME=liblmi_hip_preband.so python -u tools/f64_band_stats.py'
