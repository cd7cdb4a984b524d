#!/bin/bash
# round 5, session o: kernel breakdown of the split mode (sampled bound scan +
# collect + select) under rocprofv3
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5o_trace 600 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5o_trace -o run -- python3 bench.py --corpus f32 --no-cpu-baseline --steps 5 --warmup 2 --no-single --recall-sample 20'
