#!/bin/bash
# One SQ counter pass per ablation variant (diagnostic library), scan kernel only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
for A in ${ABLS:-1 4}; do
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"; do
    tag=$(echo $grp | cut -c1-6)
    LMI_LIB_NAME=liblmi_hip_abl.so timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex scan3_kernel \
      -d gpurun_out/pmc2/a${A}_$tag -o run --output-format csv -- python3 tools/prof_scan.py --abl $A --reps 3 \
      > gpurun_out/pmc2/a${A}_$tag.log 2>&1
    rc=$?; echo "abl $A [$grp] rc=$rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc2/a${A}_$tag.log; exit $rc; fi
  done
done
python3 - <<'PY'
import csv, glob, collections, os, re
for d in sorted(set(re.sub(r"_[^_/]*$", "", x) for x in glob.glob("gpurun_out/pmc2/a*_*") if os.path.isdir(x))):
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(d + "_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(d, " ".join(f"{k}={tot[k]/max(n[k],1):.4g}" for k in sorted(tot)))
PY
