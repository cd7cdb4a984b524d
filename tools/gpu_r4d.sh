#!/bin/bash
# round 4, session d: the walk's share of the scan at W = 1 and rank 0 of W = 8
# (diagnostic library: ABL 1 = no insertion, ABL 80 = the list held in
# registers across a block's walk), the hold-list product build, and the PMC
# traffic passes of the default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4d gpurun_out/prof
for W in 8 1; do
  ck=8192; [ $W = 8 ] && ck=2048
  LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 300 python3 tools/prof_scan.py --abl 0,1,80,0,1,80 --reps 5 --world $W --rank 0 \
      --chunk-rows $ck > gpurun_out/r4d/w$W.log 2>&1 || { tail -5 gpurun_out/r4d/w$W.log; exit 1; }
  echo "W=$W abl lib:"; grep "scan ms" gpurun_out/r4d/w$W.log
  LMI_LIB_NAME=liblmi_hip_hl.so timeout -k 10 300 python3 tools/prof_scan.py --abl 0 --reps 5 --world $W --rank 0 \
      --chunk-rows $ck --check > gpurun_out/r4d/hl_w$W.log 2>&1 || { tail -5 gpurun_out/r4d/hl_w$W.log; exit 1; }
  LMI_LIB_NAME=liblmi_hip.so timeout -k 10 300 python3 tools/prof_scan.py --abl 0 --reps 5 --world $W --rank 0 \
      --chunk-rows $ck > gpurun_out/r4d/base_w$W.log 2>&1 || { tail -5 gpurun_out/r4d/base_w$W.log; exit 1; }
  echo "W=$W hold-list build:"; grep "scan ms\|identical" gpurun_out/r4d/hl_w$W.log; echo "W=$W product:"; grep "scan ms" gpurun_out/r4d/base_w$W.log
done
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
