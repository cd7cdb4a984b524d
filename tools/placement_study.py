"""Study: whole buckets per rank instead of stripes.
For the bench workload (10M, 122 buckets, R = 4) and four 10k-query batches:
the scan work of each rank, sum over its buckets of pairs_c * N_c, when the
buckets are placed on W ranks by longest-processing-time on a weight known at
index build (N_c, N_c^2, or batch 0's pairs_c * N_c); max / mean over ranks
per batch (1.0 = the stripes' balance).  python tools/placement_study.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
from li import synth  # noqa: E402
from li.index import DeviceRouter  # noqa: E402


def lpt(weights, W):
    load = np.zeros(W)
    owner = np.zeros(len(weights), np.int64)
    for c in np.argsort(-weights, kind="stable"):
        r = int(np.argmin(load))
        owner[c] = r
        load[r] += weights[c]
    return owner


def main():
    dev = torch.device("cuda", 0)
    x, q, qn, xn, layers = synth.build_lmi_workload(10_000_000, 10_000, 122, "MLP-5", dev)
    router = DeviceRouter(layers)
    labels = router.argmax(xn).cpu().numpy()
    del x, xn
    N = np.bincount(labels, minlength=122).astype(np.float64)
    batches = synth.query_batches(4, 10_000, dev)
    pairs = []
    for b_q, b_qn in batches:
        cls, _ = router.topr(b_qn, 4, with_probs=True)
        pairs.append(np.bincount(cls.cpu().numpy().ravel(), minlength=122).astype(np.float64))
    out = {"bucket_rows": {"min": int(N.min()), "median": int(np.median(N)), "max": int(N.max())},
           "pairs_per_bucket_batch0": {"min": int(pairs[0].min()), "median": int(np.median(pairs[0])),
                                       "max": int(pairs[0].max())},
           "max_over_mean": {}}
    for W in (2, 4, 8):
        for name, w in (("N", N), ("N^2", N * N), ("batch0 work", pairs[0] * N)):
            own = lpt(w, W)
            ratios = []
            for p in pairs:
                work = np.bincount(own, weights=p * N, minlength=W)
                ratios.append(round(float(work.max() / work.mean()), 3))
            out["max_over_mean"][f"W={W} by {name}"] = ratios
    s = json.dumps(out, indent=1)
    print(s)
    os.makedirs("gpurun_out", exist_ok=True)
    open("gpurun_out/placement_study.json", "w").write(s + "\n")


if __name__ == "__main__":
    main()
