#!/bin/bash
# Round 6, call ah: the split mode's own PMC traffic on the sample-skipping
# collect (tools/pmc_split.sh), then the split bench line reading it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_split.sh || exit $?
cp gpurun_out/prof_split/split_pmc_traffic.json profiles/r06ah_split_pmc_traffic.json
cp gpurun_out/prof_split/split_pmc_traffic.json gpurun_out/r06ah_split_pmc_traffic.json
timeout -k 10 300 python -u bench.py --corpus f32 --steps 20 --warmup 5 \
  > gpurun_out/r6ah_split_bench.json 2> gpurun_out/r6ah_split_bench.err
rc=$?; cut -c1-400 gpurun_out/r6ah_split_bench.json; exit $rc
