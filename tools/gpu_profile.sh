#!/bin/bash
# Round artefacts: the default bench line (with cpu_baseline); rocprofv3 kernel
# trace + stats of the same command with the ROCTx ranges bench.py puts around
# its timed loops (tools/timed_scans.py: the timed scan launches' own
# durations); the PMC traffic passes of the scan kernel (FETCH_SIZE and
# WRITE_SIZE each in its own run).  Outputs under gpurun_out/prof/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
KRE=${KRE:-scan3_kernel}
STEPS=${STEPS:-20}
WARM=${WARM:-5}
timeout -k 10 500 python bench.py --steps $STEPS --warmup $WARM > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/prof/bench.json; tail -2 gpurun_out/prof/bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/prof/trace -o run \
   -- python3 bench.py --steps $STEPS --warmup $WARM --no-cpu-baseline --recall-sample 20 > gpurun_out/prof/trace.json 2> gpurun_out/prof/trace.err
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/timed_scans.py gpurun_out/prof/trace gpurun_out/prof/timed_scans.json > /dev/null
echo "timed scans:"; python3 -c "import json;[print(r['range'],r['launches'],r.get('mean_ms'),r.get('median_ms')) for r in json.load(open('gpurun_out/prof/timed_scans.json'))['ranges']]"
[ -n "$NO_PMC" ] && exit 0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv \
     -d gpurun_out/prof/pmc_$c -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-single --recall-sample 20 \
     > gpurun_out/prof/pmc_$c.json 2> gpurun_out/prof/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 - <<'PY'
# per kernel template (the f32 bench launches scan3_kernel<10,...>, its f64
# block scan3_kernel<15,...>); the top-level FETCH_SIZE / WRITE_SIZE are the
# f32 step's kernel (what bench.py's roofline.traffic reads)
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
        if "<10, 0, false, 0>" in k:  # (the f32 product scan; MODE 3 is the float64 band scan)
            out[c] = {"launches": len(v), "mean_kb": sum(v) / len(v), "kernel": k}
print(json.dumps(out))
json.dump(out, open("gpurun_out/prof/pmc_traffic.json", "w"), indent=1)
PY
