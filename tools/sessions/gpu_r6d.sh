#!/bin/bash
# Round 6, call d: smoke and the whole GPU suite (with the per-mode tie-window
# report), then the W = 8 projection, every rank, in both arithmetics (the
# refine's early exit for pairs with no band rows).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  r6d_smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  r6d_tests 1500 "LMI_TIE_REPORT=gpurun_out/r6d_ties.json python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/" \
  r6d_steps32 600 "python tools/stream_steps.py --worlds 8 --all-ranks --dist f32 --steps 20 > gpurun_out/r6d_steps_f32.txt" \
  r6d_steps64 600 "python tools/stream_steps.py --worlds 8 --all-ranks --dist f64 --steps 20 > gpurun_out/r6d_steps_f64.txt"
rc=$?; grep -h "ms/step" gpurun_out/r6d_steps_f*.txt; exit $rc
