#!/bin/bash
# round 4, session c: which ingredient breaks captured memset nodes; the scan's
# candidate counts and clock at W = 1 and at rank 0 of W = 8 (diagnostic
# library: ABL 7 = the full kernel + event counters); the PMC traffic passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4c
timeout -k 10 180 python -u tools/memset_graph_repro.py --quick --rounds 6 --out gpurun_out/r4c/memset_quick.json \
    > gpurun_out/r4c/memset_quick.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4c/memset_quick.log; [ $rc -ne 0 ] && exit $rc
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 300 python3 tools/prof_scan.py --abl 0,7,0 --reps 5 \
    > gpurun_out/r4c/w1.log 2>&1 || { tail -5 gpurun_out/r4c/w1.log; exit 1; }
grep -v "^\[bench\]\|amdgpu.ids" gpurun_out/r4c/w1.log
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 300 python3 tools/prof_scan.py --abl 0,7,0 --reps 5 --world 8 --rank 0 \
    --chunk-rows 2048 > gpurun_out/r4c/w8.log 2>&1 || { tail -5 gpurun_out/r4c/w8.log; exit 1; }
grep -v "^\[bench\]\|amdgpu.ids" gpurun_out/r4c/w8.log
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex scan3_kernel --output-format csv \
     -d gpurun_out/prof/pmc_$c -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-single --recall-sample 20 \
     > gpurun_out/prof/pmc_$c.json 2> gpurun_out/prof/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 - <<'PY'
import collections, csv, glob, json
out = {"by_kernel": {}}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/prof/pmc_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                agg[r["Kernel_Name"].split("(lmi::")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out["by_kernel"].setdefault(k, {})[c] = {"launches": len(v), "mean_kb": sum(v) / len(v)}
        if "<10," in k:
            out[c] = {"launches": len(v), "mean_kb": sum(v) / len(v), "kernel": k}
print(json.dumps(out))
json.dump(out, open("gpurun_out/prof/pmc_traffic.json", "w"), indent=1)
PY
