"""Seeded small workloads shared by the CPU and GPU tests (numpy PCG64)."""
import numpy as np

from li import synth
import lmi_oracle as O


def clustered(n=6000, d=768, nq=200, C=16, arch="MLP", seed=7, label_mode="router",
              n_centres=48):
    """Corpus, nav vectors, queries, router layers and object labels.

    label_mode: 'router'  labels = router argmax (LearnedIndex.py:240)
                'skewed'  Dirichlet-skewed labels with empty and tiny buckets
                'dup'     'skewed' plus exact duplicate vectors in the same
                          bucket (tied distances)
                'near'    'skewed' plus near-duplicates: 10% of the rows are
                          copies of another row of their bucket with one or two
                          components moved by one fp16 ulp (distances that
                          differ by 1e-9..1e-6, below fp32 rounding of a
                          768-term dot), 2.5% exact duplicates, and 10% of the
                          queries one ulp away from a corpus row
    """
    if label_mode == "near":
        w = clustered(n=n, d=d, nq=nq, C=C, arch=arch, seed=seed, label_mode="skewed",
                      n_centres=n_centres)
        x, xn, q, labels = w["x"], w["xn"], w["q"], w["labels"]
        rng = np.random.Generator(np.random.PCG64(seed + 6))
        perm = rng.permutation(n)
        n_near, n_dup = n // 10, n // 40
        src, dst = perm[:n_near + n_dup], perm[n_near + n_dup:2 * (n_near + n_dup)]
        x16 = x.astype(np.float16)
        for j, (s, t) in enumerate(zip(src, dst)):
            x16[t] = x16[s]
            xn[t] = xn[s]
            labels[t] = labels[s]
            if j < n_near:
                for e in rng.choice(d, 1 + (j & 1), replace=False):
                    x16[t, e] = np.nextafter(x16[t, e], np.float16(np.inf if (j >> 1) & 1 else -np.inf))
        q16 = q.astype(np.float16)
        for i in rng.choice(nq, nq // 10, replace=False):
            q16[i] = x16[rng.integers(n)]
            e = rng.integers(d)
            q16[i, e] = np.nextafter(q16[i, e], np.float16(np.inf))
        w.update(x=x16.astype(np.float32), xn=xn, q=q16.astype(np.float32), labels=labels)
        return w
    x, cen = synth.np_mixture(n, d, n_centres, seed)
    q, _ = synth.np_mixture(nq, d, n_centres, seed + 1, centres=cen)
    P = synth.np_projection(d, 96, seed + 2)
    xn, qn = synth.np_nav(x, P), synth.np_nav(q, P)
    layers = synth.np_router_layers(synth.ARCHS[arch], C, seed + 3)
    if label_mode == "router":
        labels = O.predict(xn, layers)
    elif label_mode not in ("skewed", "dup"):
        raise ValueError(label_mode)
    else:
        rng = np.random.Generator(np.random.PCG64(seed + 4))
        p = rng.dirichlet(np.full(C, 0.3))
        p[rng.choice(C, 2, replace=False)] = 0.0       # empty buckets
        p /= p.sum()
        labels = rng.choice(C, n, p=p)
        big = int(np.argmax(p))
        live = [c for c in np.nonzero(p > 0)[0] if c != big]
        tiny = rng.choice(live, 2, replace=False)
        for j, c in enumerate(tiny):                    # buckets with < k objects
            labels[labels == c] = big
            labels[rng.choice(np.nonzero(labels == big)[0], 3 + 2 * j, replace=False)] = c
    labels = np.asarray(labels, np.int64)
    if label_mode == "dup":
        rng = np.random.Generator(np.random.PCG64(seed + 5))
        src = rng.choice(n, n // 20, replace=False)
        dst = rng.choice(np.setdiff1d(np.arange(n), src), n // 20, replace=False)
        x[dst] = x[src]
        xn[dst] = xn[src]
        labels[dst] = labels[src]
    return dict(x=x, xn=xn, q=q, qn=qn, layers=layers, labels=labels, C=C)


def float64_inputs(w, seed, rel=2e-10):
    """Float64 corpus and queries for the reference's float64 branch on float64
    inputs (utils.py:11: sklearn computes in float64 unless both operands are
    float32): the float32 values plus a seeded relative perturbation below
    half a float32 ulp, so rounding them to float32 gives back w['x'] / w['q']
    exactly -- rows that are exact duplicates in float32 differ in float64,
    and any float32 shortcut orders them by position instead of by the float64
    distances the reference sees."""
    rng = np.random.Generator(np.random.PCG64(seed + 64))
    x64 = w["x"].astype(np.float64)
    q64 = w["q"].astype(np.float64)
    x64 *= 1.0 + rel * rng.standard_normal(x64.shape)
    q64 *= 1.0 + rel * rng.standard_normal(q64.shape)
    assert np.array_equal(x64.astype(np.float32), w["x"]) and np.array_equal(q64.astype(np.float32), w["q"])
    return x64, q64


def float32_inputs(w, seed, rel=2e-5, rel_q=None):
    """Float32 corpus and queries that are NOT fp16-exact, for the split mode
    (lmi_index_desc.corpus32): the workload's fp16-exact values times
    (1 + rel N(0, 1)).  rel = 2e-5 is below half an fp16 ulp (2^-12), so the
    normalised fp16 rounding the split mode scans maps most rows back onto
    their fp16 originals: near-duplicates and exact duplicates of the
    workload become ties of the fp16 scan that only the exact float32
    distances order -- the step the split mode has to get right."""
    rng = np.random.Generator(np.random.PCG64(seed + 32))
    rel_q = rel if rel_q is None else rel_q
    x32 = (w["x"].astype(np.float64) * (1.0 + rel * rng.standard_normal(w["x"].shape))).astype(np.float32)
    q32 = (w["q"].astype(np.float64) * (1.0 + rel_q * rng.standard_normal(w["q"].shape))).astype(np.float32)
    assert not np.array_equal(x32.astype(np.float16).astype(np.float32), x32)
    return x32, q32
