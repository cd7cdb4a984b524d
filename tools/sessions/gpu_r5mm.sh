#!/bin/bash
# round 5, session mm: the split mode's one-wave select with 1 / 2 / 4 float32 rows in flight per wave
# (LMI_XSEL_KB; 7 / 5 / 4 waves per SIMD) -- split-mode tests under 1 and 2, then the split bench line, alternated
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T='python -u -m pytest -x -v --timeout 300 --timeout-method thread'
bash tools/gpu_steps.sh \
  r5mm_tests 600 "LMI_XSEL_KB=1 $T tests/test_gpu_split_mode.py && LMI_XSEL_KB=2 $T tests/test_gpu_split_mode.py" \
  r5mm_ab 900 'for kb in 4 1 2 4 1 2; do LMI_XSEL_KB=$kb python -u bench.py --corpus f32 --no-cpu-baseline --no-single --steps 10 --warmup 3 > gpurun_out/r5mm_split_kb$kb.json || exit 1; python3 -c "import json;d=json.load(open(\"gpurun_out/r5mm_split_kb$kb.json\"));print(\"KB=$kb\", d[\"value\"], d[\"ms_per_step\"], d[\"other_dist\"][\"value\"], d[\"breakdown_ms\"])"; done'
