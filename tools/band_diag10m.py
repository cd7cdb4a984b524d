"""Diagnostic: pairs of the 10M bench workload that the float64 band lists
send to the whole-shard fallback under LMI_Q_SEED_ROUND0 -- their listed d32,
the bound of their unlisted rows, the band, the round-0 pair's 10th, and the
pair's true d32 order (torch over the bucket's fp16 rows)."""
import argparse, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import numpy as np
import torch
from li import synth
from li.index import DeviceIndex, DeviceRouter, bucket_topk_f64

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--R", type=int, default=4)
args = ap.parse_args()
dev = torch.device("cuda", 0)
x, q, qn, xn, layers = synth.build_lmi_workload(args.n, 10_000, 122, "MLP-5", dev)
router = DeviceRouter(layers)
labels = router.argmax(xn)
del xn
ix = DeviceIndex(x, labels, 122, chunk_rows=8192)
del x
cls, _ = router.topr(qn, args.R)
R, kl = args.R, 15
P = cls.numel()
ws = torch.zeros(1 << 29, dtype=torch.uint8, device=dev)
for seed in (False, True):
    d, pos, st, nfb = bucket_topk_f64(ix, q, cls, 10, fallback_count=True, ws=ws, seed_round0=seed)
    al = lambda b: (b + 255) // 256 * 256
    o_lb = 3 * al(P * kl * 4)
    ld = ws[:P * kl * 4].view(torch.float32).view(P, kl).cpu().numpy()
    lb = ws[o_lb:o_lb + P * 4].view(torch.float32).cpu().numpy()
    eps = 2.0 ** -16
    t = np.where(np.isfinite(ld[:, 9]), ld[:, 9].astype(np.float64) + 2 * eps, np.inf)
    bad = np.nonzero(np.isfinite(lb) & (lb <= t))[0]
    print(f"seed {int(seed)}: fallbacks {nfb}, flagged {bad.size}, rounds {np.bincount(bad % R, minlength=R)}", flush=True)
    off = ix.bucket_off_local.cpu().numpy()
    cl = cls.cpu().numpy()
    for p in bad[:6]:
        qi, r = divmod(int(p), R)
        c = int(cl[qi, r])
        a, b = int(off[c]), int(off[c + 1])
        y = ix.corpus[a:b, :768].double() * ix.inv_norm[a:b, None].double()
        qq = q[qi].double()
        dd = 1 - (y @ qq) / qq.norm()
        srt, idx = torch.sort(dd)
        print(f" pair {p} r {r} bucket {c} ({b - a} rows): lbound {lb[p]:.7f} t {t[p]:.7f} "
              f"round-0 10th {ld[qi * R, 9]:.7f}\n  listed {np.array2string(ld[p], precision=6)}\n"
              f"  true   {np.array2string(srt[:16].cpu().numpy(), precision=6)}\n"
              f"  rows of the true top-12 (local) {idx[:12].cpu().numpy()}, lanes (row % 8 < 4) {(idx[:12].cpu().numpy() % 8 < 4).astype(int)}", flush=True)
