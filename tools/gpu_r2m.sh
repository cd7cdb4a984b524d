#!/bin/bash
# bench's graph-capture fallback (Searcher.graph patched to raise) and the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python - > gpurun_out/fb.json 2> gpurun_out/fb.err <<'PY'
import sys
sys.argv = ["bench.py", "--no-cpu-baseline", "--steps", "3", "--warmup", "1", "--scale", "1M"]
sys.path.insert(0, ".")
import bench
from li import index
def boom(*a, **k):
    raise RuntimeError("capture refused (test)")
index.Searcher.graph = boom
bench.main()
PY
rc=$?; echo "fallback rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/fb.json'));print(d['step'],d['value'])" || { tail -5 gpurun_out/fb.err; exit 1; }
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py > gpurun_out/b2m.json 2> gpurun_out/b2m.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b2m.json; exit $rc
