#!/bin/bash
# round 5, session kk: the float64 refine with one list slot per lane (lists <= 64 entries) and 1 / 2 / 4 fp16 rows in
# flight per wave (LMI_REFINE_KB; 8 / 7 / 5 waves per SIMD) -- float64 tests under the default (2), then K2 in
# float64 at 300K and 10M, alternated
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5kk_tests 600 "$T tests/test_gpu_golden_r2.py tests/test_gpu_parity.py tests/test_gpu_seed.py tests/test_gpu_stream.py" \
  r5kk_tests1 600 "LMI_REFINE_KB=1 $T tests/test_gpu_golden_r2.py tests/test_gpu_seed.py" \
  r5kk_ab 700 'for kb in 4 2 1 4 2 1; do LMI_REFINE_KB=$kb python -u tools/f64_band_stats.py --n 300000 --R 7 --chunk-rows 4096 | sed "s/^/KB=$kb /" || exit 1; done; for kb in 4 2 1 4 2 1; do LMI_REFINE_KB=$kb python -u tools/f64_band_stats.py | sed "s/^/KB=$kb /" || exit 1; done'
