#!/usr/bin/env python3
"""Float64 parity mode on the bench workload (measurement, not a test):

  * the fp32 scan's error against float64: max |d32 - d64| over every entry of
    the fp32 16-entry lists (d64 recomputed here with torch in float64 from the
    stored fp16 rows, sklearn's normalize-then-dot) — the margin behind
    LMI_REFINE_EPS;
  * how many (query, probe) top-10 lists differ between fp32 and float64
    ordering (the id flips the float64 mode exists to avoid);
  * how many pairs took the whole-bucket fallback;
  * step time of Searcher.search with dist='f32' and dist='f64'.

    python tools/f64_error.py [--scale 1M] [--R 4]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
sys.path.insert(0, ROOT)

from bench import SCALES  # noqa: E402
from li import synth  # noqa: E402
from li.index import DeviceIndex, DeviceRouter, Searcher, bucket_topk, bucket_topk_f64  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="1M")
    ap.add_argument("--R", type=int, default=4)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = SCALES[args.scale]
    x, q, qn, xn, layers = synth.build_lmi_workload(n, args.nq, 122, "MLP-5", dev)
    router = DeviceRouter(layers, device=dev)
    labels = router.argmax(xn)
    del xn
    index = DeviceIndex(x, labels, 122, device=dev)
    del x
    s = Searcher(index, router)
    classes = router.topr(qn, args.R)[0]
    torch.set_grad_enabled(False)
    d32, p32, _ = bucket_topk(index, q, classes, 16)
    d64, p64, _, nfb = bucket_topk_f64(index, q, classes, 10, fallback_count=True)
    # float64 distance of every fp32 list entry
    gpos = index.gpos.long()
    row_of = torch.empty(index.n_total, dtype=torch.long, device=dev)
    row_of[gpos] = torch.arange(index.n_rows, device=dev)
    qh = q.double() / q.double().norm(dim=1, keepdim=True)
    nq, R, K = p32.shape
    err = 0.0
    for a in range(0, nq, 1000):
        pp = p32[a:a + 1000]
        m = pp >= 0
        rows = row_of[pp.clamp(min=0).long()]
        y = index.corpus[rows.view(-1), : index.d].double().view(pp.shape + (index.d,))
        yh = y / y.norm(dim=-1, keepdim=True)
        dd = 1.0 - (qh[a:a + 1000, None, None, :] * yh).sum(-1)
        e = (dd - d32[a:a + 1000].double()).abs()[m]
        err = max(err, float(e.max()))
    flips = int((p32[..., :10] != p64).any(dim=-1).sum())
    times = {}
    for dist in ("f32", "f64"):
        for _ in range(3):
            s.search(qn, q, args.R, dist=dist)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            s.search(qn, q, args.R, dist=dist)
        torch.cuda.synchronize()
        times[dist] = (time.perf_counter() - t0) / args.steps * 1e3
    out = {"scale": args.scale, "R": args.R, "nq": nq, "pairs": nq * R,
           "max_abs_err_d32_vs_d64": err, "eps": 2.0 ** -16, "eps_over_max_err": 2.0 ** -16 / err,
           "pairs_with_fp32_vs_f64_list_difference": flips, "fallback_pairs": nfb,
           "step_ms": {k: round(v, 3) for k, v in times.items()},
           "qps": {k: round(nq / (v * 1e-3), 1) for k, v in times.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
