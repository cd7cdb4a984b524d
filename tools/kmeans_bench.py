"""Timing of the k-means kernels at the 10M build shape (pca96, 122 centroids):
lmi_kmeans_assign over all rows (kmeans.index.search(X, 1), LearnedIndex.py:282)
and one training iteration on faiss's 122·256-row sample."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import torch
from li import kmeans as K

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d, k = 96, 122
g = torch.Generator(device="cuda"); g.manual_seed(0)
x = torch.randn(n, d, device="cuda", generator=g)
x /= x.norm(dim=1, keepdim=True)
cent = x[:k].clone()
for _ in range(2):
    K.assign(x, cent)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 10
e0.record()
for _ in range(reps):
    K.assign(x, cent)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
flops = 3.0 * n * k * d  # sub, mul, add per (point, centroid, dim)
t = time.time()
km = K.Kmeans(d, k, niter=25, seed=2023)
km.train(x)
torch.cuda.synchronize()
out = {"assign_ms": round(ms, 3), "n": n, "d": d, "k": k,
       "assign_GBps": round(n * d * 4 / ms / 1e6, 1), "assign_valu_Tops": round(flops / ms / 1e9, 2),
       "train_25it_s": round(time.time() - t, 3)}
print(json.dumps(out))
