#!/bin/bash
# round 5, session i: the scan's candidate stash (KL = 10 lane lists: four
# unsorted slots flushed into the list together) -- whole GPU suite; K2 and
# the stream step against the previous build (liblmi_hip_prev.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5i_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  r5i_f64 600 'python -u tools/f64_band_stats.py && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/f64_band_stats.py && python -u tools/f64_band_stats.py' \
  r5i_steps 600 'python -u tools/stream_steps.py --worlds 1,8 --steps 30 && LMI_LIB_NAME=liblmi_hip_prev.so python -u tools/stream_steps.py --worlds 1,8 --steps 30 && python -u tools/stream_steps.py --worlds 1,8 --steps 30'
