"""How often the split mode's sample scan alone covers its own rows (a study for
DESIGN §8 item 4): on the bench's 10M --corpus f32 workload, for every (query,
bucket) pair, the fp16 distances of the rounded query to the bucket's rows
(1 - cos, fp32 arithmetic on the fp16 values), d~_k over the whole bucket and
over its sample (the first s_c = min(n_c, max(chunk_rows, n_c / 16)) rows,
x_sample_desc_kernel), and the count of sample rows at or under d~_k + 2 eps.
When that count is below k, the sample scan's own top-k list holds every
sample row the select needs, so the collect scan could skip the sample rows.
Prints the failing fraction by the bucket's sample share and the rows the
collect would skip."""
import argparse, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--chunk-rows", type=int, default=8192)
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
from li import synth, _lib
from li.index import DeviceIndex, DeviceRouter
from bench import not_fp16

x, q, qn, xn, layers = synth.build_lmi_workload(a.n, 10_000, 122, "MLP-5", dev)
router = DeviceRouter(layers, device=dev)
labels = router.argmax(xn); del xn
x, q = not_fp16(x, 11), not_fp16(q, 12)
ix = DeviceIndex(x, labels, 122, device=dev, chunk_rows=a.chunk_rows)
del x
assert ix.storage == "f32x", ix.storage
two_eps = 2.0 * _lib.load().lmi_split_eps(ix.d_pad)
cls = router.topr(qn, 4)[0].to(torch.int64)
qh = q.float()
qh = (qh / qh.norm(dim=1, keepdim=True)).half().float()
qh = torch.nn.functional.pad(qh, (0, ix.d_pad - qh.shape[1]))
off = ix.layout.bucket_off
k = a.k
tot_pairs = fail = 0
rows_all = rows_skip = 0
by_share = {}
hist = np.zeros(k + 2, dtype=np.int64)
for c in range(122):
    n_c = int(off[c + 1] - off[c])
    qi, r = torch.nonzero(cls == c, as_tuple=True)
    if n_c == 0 or qi.numel() == 0:
        continue
    want = max(a.chunk_rows, (n_c // 16 + 31) // 32 * 32)
    s_c = min(n_c, want)
    xc = ix.corpus[int(off[c]):int(off[c + 1])].float()
    xc = xc * ix.inv_norm[int(off[c]):int(off[c + 1]), None]
    for b in range(0, qi.numel(), 512):
        qq = qh[qi[b:b + 512]]
        d = 1.0 - qq @ xc.T
        kk = min(k, n_c)
        dk = torch.topk(d, kk, dim=1, largest=False).values[:, -1]
        ns = (d[:, :s_c] <= (dk.double() + two_eps).float()[:, None]).sum(dim=1)
        bad = (ns >= k) & (s_c < n_c)
        share = "whole" if s_c == n_c else f"{min(9, int(10 * s_c / n_c))}/10"
        e = by_share.setdefault(share, [0, 0])
        e[0] += qq.shape[0]; e[1] += int(bad.sum())
        tot_pairs += qq.shape[0]; fail += int(bad.sum())
        rows_all += qq.shape[0] * n_c
        if s_c < n_c:
            rows_skip += qq.shape[0] * s_c
        hist += np.bincount(ns.clamp(max=k + 1).cpu().numpy(), minlength=k + 2)
        del d
print(f"pairs {tot_pairs}: sample rows at or under d~_k + 2 eps >= k (not covered) in {fail} "
      f"({100.0 * fail / tot_pairs:.2f}%); 2 eps = {two_eps:.3e}")
print("by sample share of the bucket (pairs, not covered):",
      {s: tuple(v) for s, v in sorted(by_share.items())})
print("histogram of sample rows in band (0..k, >k):", hist.tolist())
print(f"probed rows {rows_all}, sample rows of split buckets {rows_skip} ({100.0 * rows_skip / rows_all:.1f}%)")
