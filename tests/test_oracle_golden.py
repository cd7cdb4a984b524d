"""Pin the oracle (and the host replay of the product) to the reference's own
outputs: tests/golden/reference_outputs.npz was produced by running the
reference (search/li/*.py) on these seeded inputs (tests/golden/gen_golden.py)."""
import hashlib
import os

import numpy as np
import pytest

import lmi_oracle as O
import workloads

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "reference_outputs.npz"))
SEARCH = sorted({k.split("__")[0][len("search_"):] for k in G.files if k.startswith("search_")})
ROUTERS = sorted({k.split("__")[0] for k in G.files if k.startswith("router_")})

# label_mode / arch of each case (the generator's table)
from golden.gen_golden import SEARCH_CASES, SINGLE_CASES  # noqa: E402

CASES = {c[0]: c for c in SEARCH_CASES + SINGLE_CASES}


def _inputs(name):
    _, n, nq, C, R, k, mode, arch, seed, thr = CASES[name]
    w = workloads.clustered(n=n, nq=nq, C=C, arch=arch, seed=seed, label_mode=mode)
    h = hashlib.sha256()
    for a in (w["x"], w["q"], w["xn"], w["qn"], w["labels"]):
        h.update(a.tobytes())
    assert h.hexdigest() == str(G[f"search_{name}__sha"]), "input generator drifted"
    return w


def test_fixture_inventory():
    assert len(SEARCH) == len(SEARCH_CASES) + len(SINGLE_CASES)
    assert len(ROUTERS) == 3


@pytest.mark.parametrize("key", ROUTERS)
def test_router_oracle_matches_reference(key):
    x = G[f"{key}__x"]
    layers = []
    i = 0
    while f"{key}__W{i}" in G.files:
        layers.append((G[f"{key}__W{i}"], G[f"{key}__b{i}"]))
        i += 1
    probs, classes = O.predict_proba(x, layers)
    ref_c = G[f"{key}__classes"].astype(np.int64)
    # ranks agree except where two logits tie within fp32 noise
    logits = O.mlp_forward(x, layers)
    bad = 0
    for r in np.nonzero((classes[:, :16] != ref_c).any(axis=1))[0]:
        srt = np.sort(logits[r])[::-1][:17]
        if np.min(np.abs(np.diff(srt))) > 1e-6:
            bad += 1
    assert bad == 0
    np.testing.assert_allclose(probs[:, :16], G[f"{key}__probs"], rtol=1e-5, atol=1e-8)
    assert (O.predict(x, layers) == G[f"{key}__predict"]).mean() > 0.999


def _check(name, dists, anns):
    ref_d, ref_a = G[f"search_{name}__dists"], G[f"search_{name}__anns"]
    assert dists.shape == ref_d.shape
    assert O.compare_lists(ref_d, ref_a, dists, anns) == 0


@pytest.mark.parametrize("name", [c[0] for c in SEARCH_CASES])
def test_search_direct_matches_reference(name):
    """Literal restatement (full distance matrices) == reference."""
    _, n, nq, C, R, k, mode, arch, seed, thr = CASES[name]
    w = _inputs(name)
    classes = G[f"search_{name}__classes"].astype(np.int64)
    ids = np.arange(1, n + 1)
    d, a = O.search_direct(w["labels"], ids, w["x"], w["q"], classes, n_buckets=R, k=k,
                           use_threshold=thr)
    _check(name, d, a)


@pytest.mark.parametrize("name", [c[0] for c in SEARCH_CASES])
def test_lists_plus_replay_match_reference(name):
    """The decomposition the GPU path implements — per-(query, probe) lists +
    replay — reproduces the reference, through both the Python twin and the
    product's C++ lmi_replay (host code, callable without a GPU)."""
    from li.index import replay as lmi_replay
    _, n, nq, C, R, k, mode, arch, seed, thr = CASES[name]
    w = _inputs(name)
    classes = G[f"search_{name}__classes"].astype(np.int64)
    order, off = O.layout(w["labels"], C)
    ids = np.arange(1, n + 1)
    lists_d, lists_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, 10, C)
    kw = dict(k_round=10, k_final=k, bucket_size=np.diff(off), pos_to_id=ids[order],
              use_threshold=thr)
    st = {}
    d, a = O.replay(classes[:, :R], lists_d, lists_p, stats=st, **kw)
    _check(name, d, a)
    d2, a2 = lmi_replay(classes[:, :R], lists_d, lists_p, **kw)
    np.testing.assert_array_equal(d2, d)
    np.testing.assert_array_equal(a2, a)


@pytest.mark.parametrize("name", [c[0] for c in SINGLE_CASES])
def test_search_single_matches_reference(name):
    from li.index import replay as lmi_replay
    _, n, nq, C, R, k, mode, arch, seed, thr = CASES[name]
    w = _inputs(name)
    classes = G[f"search_{name}__classes"].astype(np.int64)
    thr_arr = G[f"search_{name}__thr"] if thr else None
    ids = np.arange(1, n + 1)
    d, a = O.search_single_direct(w["labels"], ids, w["x"], w["q"], classes[:, 0], k=k,
                                  threshold_dist=thr_arr)
    _check(name, d, a)
    order, off = O.layout(w["labels"], C)
    lists_d, lists_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, 1, k, C)
    d2, a2 = lmi_replay(classes[:, :1], lists_d, lists_p, k_round=k, k_final=k,
                        bucket_size=np.diff(off), pos_to_id=ids[order], use_threshold=False,
                        thr_round0=thr_arr)
    _check(name, d2, a2)


def test_fixtures_exercise_every_replay_branch():
    """The fixture set must drive the quirk paths (LearnedIndex.py:174-193),
    empty-threshold skips (:157-159) and fillers (utils.py:35-42)."""
    tot = {}
    for c in SEARCH_CASES:
        name, n, nq, C, R, k, mode, arch, seed, thr = c
        w = _inputs(name)
        classes = G[f"search_{name}__classes"].astype(np.int64)
        order, off = O.layout(w["labels"], C)
        lists_d, lists_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, 10, C)
        O.replay(classes[:, :R], lists_d, lists_p, k_round=10, k_final=k,
                 bucket_size=np.diff(off), pos_to_id=np.arange(1, n + 1)[order],
                 use_threshold=thr, stats=tot)
    assert tot["quirk0"] > 0 and tot["quirk_thr"] > 0
    assert tot["skipped"] > 0 and tot["fillers"] > 0
