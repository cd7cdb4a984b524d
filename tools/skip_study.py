"""How much of K2 could exact chunk skipping remove?  

For every (query, probe) pair and every chunk of its bucket, the cosine
distance of any row of the chunk is at least

    lb = 1 - cos(max(0, angle(q, c) - theta)),   theta = max_x angle(x, c)

(c = the chunk's unit centroid, x over the chunk's rows).  A chunk whose lb
exceeds the pair's final k-th distance in that bucket cannot change the pair's
list; a scan tile (<= 256 pairs x one chunk) can be skipped only when that holds
for every pair of its query block.  This prints the best case (the final k-th
known in advance) per pair and per tile, with pairs blocked in query order (the
plan's order) and, as an upper bound for a re-ordering plan, blocked by
nearest chunk.

    python tools/skip_study.py [--n 10000000] [--R 4]
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import numpy as np
import torch

from li import synth
from li.index import DeviceIndex, DeviceRouter, bucket_topk

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--nq", type=int, default=10_000)
ap.add_argument("--R", type=int, default=4)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--chunk-rows", type=int, default=8192)
ap.add_argument("--block", type=int, default=256)
a = ap.parse_args()
dev = torch.device("cuda")
x, q, qn, xn, layers = synth.build_lmi_workload(a.n, a.nq, 122, "MLP-5", dev)  # trains the router
torch.set_grad_enabled(False)
router = DeviceRouter(layers)
labels = router.argmax(xn)
del xn
ix = DeviceIndex(x, labels, 122, chunk_rows=a.chunk_rows, subcluster=True)
del x
classes, _ = router.topr(qn, a.R)
d, _, _ = bucket_topk(ix, q, classes, a.k)
kth = d[:, :, a.k - 1].reshape(-1)                       # [P]
cf = ix.chunk_first.cpu().numpy()
off = ix.bucket_off_local.cpu().numpy()
cent = ix.chunk_centroid[:, : ix.d]
# angular radius of every chunk: min over rows of cos(x^, c)
cos_min = torch.empty(ix.n_chunks, device=dev)
for c in range(ix.n_buckets):
    for j in range(int(cf[c + 1] - cf[c])):
        ra = int(off[c]) + j * a.chunk_rows
        rb = min(int(off[c + 1]), ra + a.chunk_rows)
        xr = ix.corpus[ra:rb, : ix.d].float() * ix.inv_norm[ra:rb, None]
        cos_min[int(cf[c]) + j] = (xr @ cent[int(cf[c]) + j]).min()
qh = q.float() / q.float().norm(dim=1, keepdim=True)
cls = classes.reshape(-1).long()
qi = torch.arange(a.nq, device=dev).repeat_interleave(a.R)
pairs = chunks = skip_pairs = 0
tiles = skip_tiles = skip_tiles_sorted = 0
for c in range(ix.n_buckets):
    nch = int(cf[c + 1] - cf[c])
    sel = (cls == c).nonzero().flatten()
    if nch == 0 or sel.numel() == 0:
        continue
    cc = cent[int(cf[c]): int(cf[c + 1])]
    cq = (qh[qi[sel]] @ cc.T).clamp(-1, 1)                 # [p, nch]
    alpha = torch.acos(cq)
    theta = torch.acos(cos_min[int(cf[c]): int(cf[c + 1])].clamp(-1, 1))
    lb = 1 - torch.cos((alpha - theta[None, :]).clamp(min=0))
    skip = lb > kth[sel][:, None] + 1e-5                   # [p, nch]
    pairs += sel.numel()
    chunks += skip.numel()
    skip_pairs += int(skip.sum())
    for order, name in ((torch.arange(sel.numel(), device=dev), "q"), (cq.argmax(dim=1).argsort(), "s")):
        sk = skip[order]
        for b0 in range(0, sel.numel(), a.block):
            blk = sk[b0: b0 + a.block].all(dim=0)          # [nch]
            if name == "q":
                tiles += nch
                skip_tiles += int(blk.sum())
            else:
                skip_tiles_sorted += int(blk.sum())
out = {"n": a.n, "nq": a.nq, "R": a.R, "k": a.k, "chunk_rows": a.chunk_rows, "n_chunks": ix.n_chunks,
       "cos_min_median": float(cos_min.median()), "theta_median_deg": math.degrees(math.acos(float(cos_min.median()))),
       "pair_chunks": chunks, "pair_chunks_skippable": skip_pairs, "pair_frac": skip_pairs / max(chunks, 1),
       "tiles": tiles, "tiles_skippable_query_order": skip_tiles, "tile_frac_query_order": skip_tiles / max(tiles, 1),
       "tiles_skippable_nearest_chunk_order": skip_tiles_sorted,
       "tile_frac_nearest_chunk_order": skip_tiles_sorted / max(tiles, 1)}
print(json.dumps(out), flush=True)
