#!/bin/bash
# round 5, session g: the float64 band lists (fixed) -- whole GPU suite, K2 in
# float64 against the previous build, the f64 bench line, a kernel trace of
# the float64 scan
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5g_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  r5g_f64 600 'python -u tools/f64_band_stats.py && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/f64_band_stats.py' \
  r5g_bench64 600 'python -u bench.py --dist f64 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5g_bench64.json' \
  r5g_trace64 600 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g_trace64 -o run -- python3 tools/f64_band_stats.py'
