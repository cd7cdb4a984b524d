#!/bin/bash
# round 5, session s: K2 in float64 at 300K (R = 7) and 10M: band lists
# against the pre-band build (liblmi_hip_preband.so, commit 78edc47)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5s_f64 600 'python -u tools/f64_band_stats.py --n 300000 --R 7 && LMI_LIB_NAME=liblmi_hip_preband.so python -u tools/f64_band_stats.py --n 300000 --R 7' \
  r5s_trace 600 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5s_trace -o run -- python3 tools/f64_band_stats.py --n 300000 --R 7'
