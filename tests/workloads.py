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
    """
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
