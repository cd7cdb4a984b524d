"""Debug: v1 vs v2 vs oracle on the failing skewed case; prints mismatching rows."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("sisap23-laion-challenge-learned-index_amd", "oracle", "tests")]
import numpy as np, torch
import lmi_oracle as O, workloads
from li.index import DeviceIndex, bucket_topk
for mode, chunk in [("skewed", 512), ("skewed", 8192), ("router", 512)]:
    w = workloads.clustered(n=6000, nq=257, C=16, seed=5, label_mode=mode)
    R, k = 4, 10
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, k, w["C"])
    ix = DeviceIndex(w["x"], w["labels"], w["C"], storage="f16", chunk_rows=chunk)
    q = torch.from_numpy(w["q"]).cuda(); c = torch.from_numpy(classes.astype(np.int32)).cuda()
    d2, p2, _ = bucket_topk(ix, q, c, k); d2, p2 = d2.cpu().numpy(), p2.cpu().numpy()
    os.environ["LMI_SCAN_V1"] = "1"
    d1, p1, _ = bucket_topk(ix, q, c, k); d1, p1 = d1.cpu().numpy(), p1.cpu().numpy()
    del os.environ["LMI_SCAN_V1"]
    sizes = np.bincount(w["labels"], minlength=16)
    print(mode, chunk, "sizes", sizes.tolist())
    print("  v1 bad", O.compare_lists(ref_d, ref_p, d1, p1), " v2 bad", O.compare_lists(ref_d, ref_p, d2, p2))
    bad = [(qq, r) for qq in range(257) for r in range(R)
           if O.compare_lists(ref_d[qq, r][None], ref_p[qq, r][None], d2[qq, r][None], p2[qq, r][None])]
    print("  v2 bad (q,r):", bad[:12], "buckets:", sorted({int(classes[qq, r]) for qq, r in bad}))
    for qq, r in bad[:3]:
        print("   q", qq, "r", r, "c", classes[qq, r], "size", sizes[classes[qq, r]])
        print("    ref", np.round(ref_d[qq, r], 4).tolist(), ref_p[qq, r].tolist())
        print("    v2 ", np.round(d2[qq, r], 4).tolist(), p2[qq, r].tolist())
