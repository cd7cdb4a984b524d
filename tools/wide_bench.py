"""k > 16 lists at the bench's workload (10M, R = 4, 10k queries): the bound +
collect path (bucket_topk_wide) against the lower-bound passes alone
(LMI_WIDE_PASSES=1) -- ms per lmi_bucket_topk call (HIP events), the lists
bitwise equal, and how many pairs took the fix-up passes (the pairs whose
lists change under LMI_WIDE_NO_FIXUP).  Float64 mode too (k + 5 entries).

    python tools/wide_bench.py [--scale 10M] [--ks 20,50,100,250] [--out path]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd")]
import bench  # noqa: E402
from li import _lib  # noqa: E402
from li import index as I  # noqa: E402


def run(ix, q, cls, k, dist, env, reps):
    for var in ("LMI_WIDE_PASSES", "LMI_WIDE_NO_FIXUP"):
        os.environ.pop(var, None)
    os.environ.update(env)
    _lib.load().lmi_config_reload()
    fn = I.bucket_topk_f64 if dist == "f64" else I.bucket_topk
    out = fn(ix, q, cls, k)  # warm-up (workspace, kernel attributes)
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn(ix, q, cls, k)
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    for var in env:
        os.environ.pop(var, None)
    _lib.load().lmi_config_reload()
    return sorted(ms)[len(ms) // 2], out[0], out[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="10M")
    ap.add_argument("--ks", default="20,50,100,250")
    ap.add_argument("--f64-ks", default="11,45")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/wide/bench.json")
    a = ap.parse_args()
    args = argparse.Namespace(scale=a.scale, nq=10_000, n_buckets=122, arch="MLP-5", centres=400,
                              train_steps=200, chunk_rows=8192)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    x, q, qn, router, ix, labels = bench.build_workload(args, dev, 0, 1)
    del x
    cls, _ = router.topr(qn, 4, with_probs=True)
    res = {"workload": f"{a.scale}, R=4, nq=10000, chunk_rows=8192", "runs": []}
    cases = [(int(k), "f32") for k in a.ks.split(",") if k] + \
            [(int(k), "f64") for k in a.f64_ks.split(",") if k]
    for k, dist in cases:
        t_w, d_w, p_w = run(ix, q, cls, k, dist, {}, a.reps)
        t_p, d_p, p_p = run(ix, q, cls, k, dist, {"LMI_WIDE_PASSES": "1"}, a.reps)
        _, d_n, p_n = run(ix, q, cls, k, dist, {"LMI_WIDE_NO_FIXUP": "1"}, 1)
        equal = bool(torch.equal(p_w, p_p) and torch.equal(d_w, d_p))
        fixed = int((p_n != p_w).reshape(p_w.shape[0] * p_w.shape[1], -1).any(dim=1).sum())
        r = {"k": k, "dist": dist, "wide_ms": round(t_w, 3), "passes_ms": round(t_p, 3),
             "speedup": round(t_p / t_w, 2), "bitwise_equal": equal,
             "fixup_pairs": fixed, "pairs": int(p_w.shape[0] * p_w.shape[1])}
        print(json.dumps(r), flush=True)
        res["runs"].append(r)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
