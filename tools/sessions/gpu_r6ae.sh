#!/bin/bash
# Round 6, call ae: the split mode's workgroup select walks only the pairs the
# wave select lists (instead of every grouped pair) -- the split GPU tests, then
# the split bench line against the previous build (li/liblmi_hip_base.so),
# alternated, and its kernel stats under rocprofv3.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_split_mode.py tests/test_gpu_split_stream.py tests/test_gpu_split.py tests/test_gpu_stream.py \
  > gpurun_out/r6ae_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6ae_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in liblmi_hip_base.so liblmi_hip.so; do
    LMI_LIB_NAME=$lib timeout -k 10 300 python -u bench.py --corpus f32 --no-cpu-baseline --steps 20 --warmup 5 \
      > gpurun_out/r6ae_split_${lib}_$i.json 2> gpurun_out/r6ae_split_${lib}_$i.err
    rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r6ae_split_${lib}_$i.json')); print('split $lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['other_dist']['value'], d['other_dist']['ms_per_step'], d['single_batch']['ms'], d['parity']['lists_f32']['mismatches'], d['parity']['stream_answers_f32'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ae_prof -o run -- \
  python3 bench.py --corpus f32 --no-cpu-baseline --no-single --steps 10 --warmup 3 > gpurun_out/r6ae_prof.json 2> gpurun_out/r6ae_prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
