#!/bin/bash
# PMC traffic of the split mode's step (bench.py --corpus f32): FETCH_SIZE and
# WRITE_SIZE, each in its own rocprofv3 run, over its two scans -- the sample
# scan (scan3_kernel<10, 0, false, 0> on the sample descriptor) and the collect
# scan (scan3_kernel<10, 0, false, 2>) -- per step, summed (what the bench
# line's kernel_ms sums too) -> gpurun_out/prof_split/split_pmc_traffic.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/prof_split; mkdir -p $O; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex "scan3_kernel" --output-format csv \
     -d $O/pmc_$c -o run -- python3 bench.py --corpus f32 --steps 5 --warmup 1 --no-cpu-baseline --no-single \
     --recall-sample 20 > $O/pmc_$c.json 2> $O/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && { tail -3 $O/pmc_$c.err; exit $rc; }
done
python3 - <<'PY'
import collections, csv, glob, json
O = "gpurun_out/prof_split"
out = {"by_kernel": {}, "how": "per dispatch means; a split step launches one sample scan (MODE 0 over "
       "the sample descriptor) and one collect scan (MODE 2); FETCH_SIZE / WRITE_SIZE below are their sums"}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{O}/pmc_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                agg[r["Kernel_Name"].split("(lmi::")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    tot = 0.0
    for k, v in agg.items():
        out["by_kernel"].setdefault(k, {})[c] = {"launches": len(v), "mean_kb": sum(v) / len(v)}
        if "<10, 0, false, 0>" in k or "<10, 0, false, 2>" in k:
            tot += sum(v) / len(v)
    out[c] = {"mean_kb": tot, "kernels": "scan3_kernel<10, 0, false, 0> (sample) + <10, 0, false, 2> (collect)"}
print(json.dumps(out))
json.dump(out, open(f"{O}/split_pmc_traffic.json", "w"), indent=1)
PY
