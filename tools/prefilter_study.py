#!/usr/bin/env python3
"""Would an exact low-precision prefilter cut K2's MFMA work?  (VERDICT r2,
next-round item 3c.)  Measured on the bench's own 10M workload, no kernel
written: for sampled (query, probe) pairs, the int8 distance of every row of
the probed bucket with a RIGOROUS bound on its error, and how many rows the
bound cannot exclude.

An int8 scan (v_mfma_i32_32x32x32_i8: 2x the fp16 MFMA rate, exact int32
accumulation) of rows quantised per row, y~ = round(y / s_y) * s_y with
s_y = max|y| / 127, and of queries quantised per query the same way, gives
dot~ = <q~, y~> exactly; with e_y = y - y~ (|e_y,i| <= s_y / 2) and e_q:
    |<q, y> - dot~| <= sum |q_i| |e_y,i| + sum |y~_i| |e_q,i|
                    <= (s_y / 2) ||q||_1 + (s_q / 2) ||y~||_1     (bound_abs)
so |d - d~| <= bound_abs / (||q|| ||y||) with d~ = 1 - dot~ / (||q|| ||y||).
A row can be dropped exactly only when d~ - bound > the pair's final k-th
distance (the best case for the prefilter: the final threshold known from
the start).  The survivors must then be rescored in fp16; a tile of 256
pairs re-reads every row that survives for ANY of its pairs.  (fp8 e4m3
carries 3 mantissa bits against int8's 7 at the row's largest element: its
bound is wider still.)

    python tools/prefilter_study.py [--pairs 256] [--scale 10M]
Writes profiles/r03_prefilter_study.json (run on the GPU box: torch on the
device for the float64 distances)."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))


def main():
    import numpy as np
    import torch
    from li import synth
    from li.index import BucketLayout, DeviceRouter
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_prefilter_study.json"))
    a = ap.parse_args()
    dev = torch.device(a.device)
    t0 = time.time()
    x, q, qn, xn, layers = synth.build_lmi_workload(a.n, 10_000, 122, "MLP-5", dev)
    if dev.type == "cuda":
        router = DeviceRouter(layers, device=dev)
        labels = router.argmax(xn).cpu().numpy()
        classes = router.topr(qn, 4)[0].cpu().numpy()
    else:   # CPU rehearsal at a small n: the same MLP (Linear/ReLU) in torch
        def logits(v):
            for i, (w, b) in enumerate(layers):
                v = v @ w.T + b
                if i + 1 < len(layers):
                    v = torch.relu(v)
            return v
        labels = torch.cat([logits(xn[i:i + 65536]).argmax(1) for i in range(0, xn.shape[0], 65536)]).numpy()
        classes = torch.topk(logits(qn), 4, dim=1).indices.numpy()
    del xn
    lay = BucketLayout.from_labels(labels, 122)
    order = torch.from_numpy(lay.order).to(dev)
    rng = np.random.default_rng(1)
    # the pairs of one popular bucket (a tile's worth) and random pairs
    c_pop = int(np.bincount(classes.ravel(), minlength=122).argmax())
    qs_pop = np.nonzero((classes == c_pop).any(axis=1))[0][: a.pairs]
    res = {"what": __doc__.split("\n\n")[0], "n": a.n, "k": a.k, "workload": "bench.py synthetic workload at n rows", "device": str(dev),
           "build_s": round(time.time() - t0, 1)}

    def study(q_idx, c_of):
        stats = {"pairs": 0, "rows": 0, "int8_survivors": 0, "int8_survivors_self_threshold": 0,
                 "int8_survivors_cs": 0, "int8_survivors_cs_self_threshold": 0,
                 "bound_median": [], "bound_cs_median": [], "kth_gap_median": [],
                 "wave_blocks": 0, "wave_blocks_with_survivor": 0}
        union8 = {}
        wave, wave_n = {}, {}
        cache = {}
        for qi in q_idx:
            c = int(c_of(qi))
            a0, b0 = int(lay.bucket_off[c]), int(lay.bucket_off[c + 1])
            if c not in cache:
                cache.clear()
                y = x[order[a0:b0]].double()                  # fp16 values, exact
                sy = y.abs().amax(dim=1) / 127                # int8 per-row scale
                yi = torch.round(y / sy[:, None])
                y8 = yi * sy[:, None]
                cache[c] = (y, y.norm(dim=1), sy, yi, y8.abs().sum(dim=1), (y - y8).norm(dim=1), y8.norm(dim=1))
            y, ny, sy, yi, y8l1, ey2, y8n = cache[c]
            qq = q[qi].double()
            nq_ = qq.norm()
            d = 1 - (y @ qq) / (ny * nq_)
            thr = torch.topk(d, a.k, largest=False).values[-1]
            # int8 per-row / per-query quantisation, exact integer dot
            sq = qq.abs().max() / 127
            qi8 = torch.round(qq / sq)
            dot8 = (yi @ qi8) * sy * sq
            bound = (sy / 2) * qq.abs().sum() + (sq / 2) * y8l1
            d8 = 1 - dot8 / (ny * nq_)
            bnd = bound / (ny * nq_)
            surv8 = (d8 - bnd) <= thr
            # one-pass variant: the threshold an int8 scan can know by itself,
            # the k-th smallest upper bound d~ + bound (>= the true k-th distance)
            thr_up = torch.topk(d8 + bnd, a.k, largest=False).values[-1]
            surv_up = (d8 - bnd) <= thr_up
            # Cauchy-Schwarz form: |<q, e_y>| + |<e_q, y~>| <= ||q|| ||e_y|| + ||e_q|| ||y~||
            # (||e_y|| stored per row, ||e_q|| per query: exact quantities, no sign info needed)
            bnd_cs = (nq_ * ey2 + (qq - qi8 * sq).norm() * y8n) / (ny * nq_)
            stats["int8_survivors_cs"] += int(((d8 - bnd_cs) <= thr).sum())
            thr_cs = torch.topk(d8 + bnd_cs, a.k, largest=False).values[-1]
            stats["int8_survivors_cs_self_threshold"] += int(((d8 - bnd_cs) <= thr_cs).sum())
            stats["bound_cs_median"].append(float(bnd_cs.median()))
            stats["pairs"] += 1
            stats["rows"] += b0 - a0
            stats["int8_survivors"] += int(surv8.sum())
            stats["int8_survivors_self_threshold"] += int(surv_up.sum())
            stats["bound_median"].append(float(bnd.median()))
            stats["kth_gap_median"].append(float((d.median() - thr)))
            u = union8.setdefault(c, torch.zeros(b0 - a0, dtype=torch.bool, device=dev))
            u |= surv8
            # a wave's 32 pairs (consecutive pairs of the sample): the 32-row
            # blocks where at least one of them keeps a survivor (C-S bound,
            # the final threshold) are the blocks the wave would rescore in fp16
            wv = wave.setdefault(c, torch.zeros(b0 - a0, dtype=torch.bool, device=dev))
            wv |= (d8 - bnd_cs) <= thr
            wave_n[c] = wave_n.get(c, 0) + 1
            if wave_n[c] == 32:
                m = wv[: wv.numel() // 32 * 32].view(-1, 32).any(dim=1)
                stats["wave_blocks"] += int(m.numel())
                stats["wave_blocks_with_survivor"] += int(m.sum())
                wave_n[c] = 0
                wv.zero_()
        stats["int8_survivor_frac"] = stats["int8_survivors"] / max(stats["rows"], 1)
        stats["int8_survivor_frac_self_threshold"] = stats["int8_survivors_self_threshold"] / max(stats["rows"], 1)
        for key in ("int8_survivors_cs", "int8_survivors_cs_self_threshold"):
            stats[key + "_frac"] = stats[key] / max(stats["rows"], 1)
        for key in ("bound_median", "bound_cs_median", "kth_gap_median"):   # median over pairs of the per-pair medians
            stats[key] = float(np.median(stats[key])) if stats[key] else None
        # 32-row blocks holding a survivor of any pair of the sample (what a tile re-reads in fp16)
        nb = nbs = 0
        for v in union8.values():
            m = v[: v.numel() // 32 * 32].view(-1, 32).any(dim=1)
            nb += int(m.numel()); nbs += int(m.sum())
        stats["blocks32_with_any_survivor_frac"] = nbs / max(nb, 1)
        stats["wave32_blocks32_with_survivor_frac"] = (stats["wave_blocks_with_survivor"] /
                                                       max(stats["wave_blocks"], 1))
        tot = sum(int(v.numel()) for v in union8.values())
        stats["rows_surviving_for_any_pair_of_the_sample"] = sum(int(v.sum()) for v in union8.values())
        stats["union_frac"] = stats["rows_surviving_for_any_pair_of_the_sample"] / max(tot, 1)
        return stats

    res["tile_of_popular_bucket"] = {"bucket": c_pop, **study(qs_pop, lambda qi: c_pop)}
    rnd = rng.choice(10_000, a.pairs, replace=False)
    rr = rng.integers(0, 4, a.pairs)
    res["random_pairs"] = study(rnd, lambda qi: classes[qi, rr[list(rnd).index(qi)]])
    print(json.dumps(res, indent=1))
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
