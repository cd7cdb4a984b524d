"""GraphedSearch(pipeline=True) regression probe: capture, one replay, eager work between replays
(searches, clones, allocations), then replays and a restaged batch.  Round 3 found the two
captured graphs answering wrong lists after such eager work while the library initialised its
workspace with hipMemsetAsync (memset nodes in the graphs); with fill kernels every sequence
here answers like the eager search."""
import sys, os
for p in ("tests", "oracle", "sisap23-laion-challenge-learned-index_amd"):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", p))
import numpy as np, torch
import workloads
from li.index import DeviceIndex, DeviceRouter, Searcher

w = workloads.clustered(n=6000, nq=300, C=16, seed=51, label_mode="near")
s = Searcher(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda"),
             DeviceRouter(w["layers"], device="cuda"))
perm = np.random.default_rng(1).permutation(w["q"].shape[0])
qn2, q2 = w["qn"][perm], w["q"][perm]
T = lambda a: torch.from_numpy(a).cuda()
A0 = s.search(T(w["qn"]), T(w["q"]), 4, k=10)[1]
B0 = s.search(T(qn2), T(q2), 4, k=10)[1]

def tensors(obj):
    return {k: v for k, v in vars(obj).items() if isinstance(v, torch.Tensor) and v.is_cuda}

def snap():
    out = {}
    for name, o in (("index", s.index), ("router", s.router), ("searcher", s)):
        for k, v in tensors(o).items():
            out[f"{name}.{k}"] = v.clone()
    for i, t in enumerate(getattr(s, "_dev_tables", ()) or ()):
        out[f"devtab{i}"] = t.clone()
    return out

def case(name, pipeline=True, d0=True, e0=True, between="search_perm", restage=True):
    g = s.graph(w["qn"], w["q"], 4, k=10, dist="f32", pipeline=pipeline)
    if d0: s.search(T(w["qn"]), T(w["q"]), 4, k=10)
    if e0: s.search(T(qn2), T(q2), 4, k=10)
    g.run()
    torch.cuda.synchronize()
    before = snap()
    if between == "search_perm": s.search(T(qn2), T(q2), 4, k=10)
    elif between == "search_orig": s.search(T(w["qn"]), T(w["q"]), 4, k=10)
    elif between == "lists_perm": s.lists(T(qn2), T(q2), 4, 10)
    elif between == "router_perm": s.router.topr(T(qn2), 4)
    elif between == "alloc": x = torch.full((1 << 22,), 7, dtype=torch.int32, device="cuda"); del x
    torch.cuda.synchronize()
    after = snap()
    changed = [k for k in before if not torch.equal(before[k], after[k])]
    res = []
    for i in range(3):
        try:
            a = g.run(qn2, q2)[1] if (restage and i == 0) else g.run()[1]
            res.append("ok" if np.array_equal(a, B0 if restage else A0) else "DIFF")
        except Exception:
            res.append("RAISE")
    blk = ""
    if pipeline:
        hb = g.h_blk[0].cuda()
        blk = " d_blk==h_blk " + str([bool(torch.equal(db, hb)) for db in g.d_blks])
    print(f"{name}: {res} changed={changed}{blk}", flush=True)
    del g
    torch.cuda.synchronize()

case("V0 control")
case("V1 no d0", d0=False)
case("V2 no e0", e0=False)
case("V1+2 no d0 e0", d0=False, e0=False)
case("V3 between orig", between="search_orig")
case("V4 between alloc", between="alloc")
case("V4b between none", between="none")
case("V5 no restage", restage=False)
case("V6 non-pipeline", pipeline=False)
case("V7 between lists", between="lists_perm")
case("V8 between router", between="router_perm")
case("V0 control again")
