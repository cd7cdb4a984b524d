#!/bin/bash
# parity tests (gpu) -> 10M bench (no cpu baseline); stop on crash/timeout
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/t4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t4.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/b4.json 2> gpurun_out/b4.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/b4.json')); r=d['roofline']
print('QPS', d['value'], 'ms/step', d['ms_per_step'], 'scan_ms', r['kernel_ms'], 'HBMfrac', r['frac'], 'TF', r['mfma_tflops'], 'recall', d['recall'], d['breakdown_ms'])"
exit $rc
