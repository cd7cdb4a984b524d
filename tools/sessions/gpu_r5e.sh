#!/bin/bash
# round 5, session e: the float64 mode's band lists (10-entry lane lists, the
# filter widened by 2 eps, 15 entries + a bound per pair) -- whole GPU suite,
# K2-in-float64 time and fallback count against the previous build; the
# batch stream with the answer's D2H on the copy engine and the finish at high priority
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5e_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  r5e_f64 600 'python -u tools/f64_band_stats.py && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/f64_band_stats.py' \
  r5e_sdma 600 'python -u tools/stream_steps.py --worlds 1,8 --steps 30 --modes stream,stream-sdma,stream-prio,stream-sdma-prio,stream,stream-sdma-prio' \
  r5e_bench64 600 'python -u bench.py --dist f64 --no-cpu-baseline --steps 20 --warmup 5 && LMI_LIB_NAME=liblmi_hip_prev.so python -u bench.py --dist f64 --no-cpu-baseline --steps 20 --warmup 5'
