#!/bin/bash
# round 5, session ii: the float64 refine with 8 fp16 rows in flight per wave (LMI_REFINE_KB=8, 4 waves per SIMD)
# against 4 (5 waves per SIMD): float64 tests under KB=8, then K2-in-float64 times at 10M and 300K, alternated
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5ii_tests 600 "LMI_REFINE_KB=8 $T tests/test_gpu_golden_r2.py tests/test_gpu_parity.py tests/test_gpu_seed.py tests/test_gpu_fullsize.py" \
  r5ii_ab 700 'for kb in 4 8 4 8; do LMI_REFINE_KB=$kb python -u tools/f64_band_stats.py --n 300000 --R 7 --chunk-rows 4096 | sed "s/^/KB=$kb /" || exit 1; done; for kb in 4 8 4 8; do LMI_REFINE_KB=$kb python -u tools/f64_band_stats.py | sed "s/^/KB=$kb /" || exit 1; done'
