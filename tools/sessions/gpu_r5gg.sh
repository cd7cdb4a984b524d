#!/bin/bash
# round 5, session gg: the committed tree after the stream-queue change -- smoke, the whole GPU suite,
# configs[1] (300K, R=7) bench line (float32 + float64), the split-mode line
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r5gg_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r5gg_tests 1500 'python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/' \
  r5gg_300k 400 'python -u bench.py --scale 300K --R 7 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5gg_300K_R7_bench.json' \
  r5gg_split 400 'python -u bench.py --corpus f32 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r5gg_bench_split.json'
