#!/bin/bash
# chunk rows vs scan time and FETCH_SIZE at W=1 (plan tile order: sibling tiles adjacent; shorter
# tiles start siblings closer together in time)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for CK in 8192 4096 2048 8192; do
  LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 300 python tools/prof_scan.py --no-subcluster --chunk-rows $CK --reps 10 --abl 0 > gpurun_out/ck_$CK.log 2>&1
  rc=$?; echo "chunk $CK rc=$rc"; grep -v amdgpu.ids gpurun_out/ck_$CK.log; [ $rc -ne 0 ] && exit $rc
done
for CK in 8192 4096 2048; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex scan3_kernel --output-format csv \
     -d gpurun_out/ckp$CK -o run -- python3 tools/prof_scan.py --no-subcluster --chunk-rows $CK --reps 3 > gpurun_out/ckp$CK.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "pmc $CK rc=$rc"; tail -3 gpurun_out/ckp$CK.log; exit $rc; }
  python3 - $CK <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(f"gpurun_out/ckp{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
print(f"chunk {sys.argv[1]}: FETCH_SIZE x2 = {2*sum(v)/max(len(v),1)/1e6:.2f} GB per launch ({len(v)} launches)")
PY
done
