#!/bin/bash
# round 5, session jj: the float64 refine with 2 fp16 rows in flight per wave at 6 waves per SIMD (LMI_REFINE_KB=2)
# against 4 rows at 5 waves (the default; 8 rows at 4 waves measured slower in session ii)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5jj_tests 600 "LMI_REFINE_KB=2 $T tests/test_gpu_golden_r2.py tests/test_gpu_parity.py tests/test_gpu_seed.py" \
  r5jj_ab 700 'for kb in 4 2 4 2; do LMI_REFINE_KB=$kb python -u tools/f64_band_stats.py --n 300000 --R 7 --chunk-rows 4096 | sed "s/^/KB=$kb /" || exit 1; done; for kb in 4 2 4 2; do LMI_REFINE_KB=$kb python -u tools/f64_band_stats.py | sed "s/^/KB=$kb /" || exit 1; done'
