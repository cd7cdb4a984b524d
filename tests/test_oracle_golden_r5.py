"""Pin the oracle and the product's host replay to the reference's own outputs
on float32 inputs that are NOT fp16-exact (tests/golden/reference_outputs_r5.npz,
written by tests/golden/gen_golden_r5.py running the reference itself): the
split mode's inputs (lmi_index_desc.corpus32).  float32 queries run the
reference's float32 arithmetic, float16 / float64 queries its float64 one
(utils.py:11, :19).  The fixtures are sharp for the split mode: ranking by the
normalised fp16 rounding the split mode scans disagrees with the reference."""
import hashlib
import os

import numpy as np
import pytest

import lmi_oracle as O
import workloads
from golden.gen_golden_r5 import X_BASELINE, X_SEARCH, X_SINGLE, queries

HERE = os.path.dirname(os.path.abspath(__file__))
G5 = np.load(os.path.join(HERE, "golden", "reference_outputs_r5.npz"))
CASES = {c[0]: c for c in X_SEARCH}
SINGLES = {c[0]: c for c in X_SINGLE}
BASES = {c[0]: c for c in X_BASELINE}
TIE32, TIE64 = 1e-6, 1e-12


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(a.tobytes())
    return h.hexdigest()


def inputs_r5(name):
    """(workload, float32 data_search values, queries, arithmetic) of a case,
    checked against the fixture's input hash."""
    if name in CASES:
        _, n, nq, C, R, k, mode, arch, seed, thr, qdt = CASES[name]
    else:
        (_, n, nq, C, R, k, mode, arch, seed), qdt = SINGLES[name], "f32"
    w = workloads.clustered(n=n, nq=nq, C=C, arch=arch, seed=seed, label_mode=mode)
    x32, q32 = workloads.float32_inputs(w, seed)
    q = queries(w, seed, q32, qdt)
    assert _sha(x32, q, w["xn"], w["qn"], w["labels"]) == str(G5[f"search_{name}__sha"]), \
        "input generator drifted"
    return w, x32, q, ("f32" if qdt == "f32" else "f64")


def check(name, dists, anns, arith):
    ref_d, ref_a = G5[f"search_{name}__dists"], G5[f"search_{name}__anns"]
    assert dists.shape == ref_d.shape
    tol = dict(atol=1e-5, tie=TIE32) if arith == "f32" else dict(atol=1e-12, tie=TIE64)
    assert O.compare_lists(ref_d, ref_a, dists, anns, **tol) == 0


def test_fixture_inventory_r5():
    keys = {k.split("__")[0] for k in G5.files}
    assert len(keys) == len(X_SEARCH) + len(X_SINGLE) + len(X_BASELINE)


@pytest.mark.parametrize("name", list(CASES))
def test_x_search_direct_matches_reference(name):
    _, n, nq, C, R, k, mode, arch, seed, thr, qdt = CASES[name]
    w, x, q, arith = inputs_r5(name)
    classes = G5[f"search_{name}__classes"].astype(np.int64)
    d, a = O.search_direct(w["labels"], np.arange(1, n + 1), x, q, classes, n_buckets=R, k=k,
                           use_threshold=thr)
    check(name, d, a, arith)


@pytest.mark.parametrize("name", list(CASES))
def test_x_lists_plus_replay_match_reference(name):
    from li.index import replay as lmi_replay
    _, n, nq, C, R, k, mode, arch, seed, thr, qdt = CASES[name]
    w, x, q, arith = inputs_r5(name)
    classes = G5[f"search_{name}__classes"].astype(np.int64)
    order, off = O.layout(w["labels"], C)
    lists_d, lists_p = O.bucket_lists(w["labels"], x, q, classes, R, 10, C)
    kw = dict(k_round=10, k_final=k, bucket_size=np.diff(off),
              pos_to_id=np.arange(1, n + 1)[order], use_threshold=thr)
    d, a = O.replay(classes[:, :R], lists_d, lists_p, **kw)
    check(name, d, a, arith)
    d2, a2 = lmi_replay(classes[:, :R], lists_d, lists_p, **kw)
    np.testing.assert_array_equal(d2, d)
    np.testing.assert_array_equal(a2, a)


def test_x_fixtures_are_sharp_for_the_fp16_rounding():
    """The same searches on the normalised fp16 rounding of the inputs (what
    the split mode's first scan sees) disagree with the reference's ids."""
    def r16(v):
        v = v.astype(np.float64)
        n = np.sqrt((v * v).sum(axis=1, keepdims=True))
        return (v / np.where(n == 0, 1, n)).astype(np.float32).astype(np.float16).astype(np.float32)
    flips = 0
    for name, c in CASES.items():
        _, n, nq, C, R, k, mode, arch, seed, thr, qdt = c
        w, x, q, arith = inputs_r5(name)
        classes = G5[f"search_{name}__classes"].astype(np.int64)
        d, a = O.search_direct(w["labels"], np.arange(1, n + 1), r16(x), r16(q), classes, n_buckets=R,
                               k=k, use_threshold=thr)
        flips += O.compare_lists(G5[f"search_{name}__dists"], G5[f"search_{name}__anns"], d, a,
                                 atol=1e-2, tie=TIE32)
    assert flips > 0


@pytest.mark.parametrize("name", list(SINGLES))
def test_x_search_single_matches_reference(name):
    from li.index import replay as lmi_replay
    _, n, nq, C, R, k, mode, arch, seed = SINGLES[name]
    w, x, q, arith = inputs_r5(name)
    classes = G5[f"search_{name}__classes"].astype(np.int64)
    d, a = O.search_single_direct(w["labels"], np.arange(1, n + 1), x, q, classes[:, 0], k=k)
    check(name, d, a, arith)
    order, off = O.layout(w["labels"], C)
    lists_d, lists_p = O.bucket_lists(w["labels"], x, q, classes, 1, k, C)
    d2, a2 = lmi_replay(classes[:, :1], lists_d, lists_p, k_round=k, k_final=k,
                        bucket_size=np.diff(off), pos_to_id=np.arange(1, n + 1)[order],
                        use_threshold=False)
    check(name, d2, a2, arith)


@pytest.mark.parametrize("name", list(BASES))
def test_x_baseline_oracle_matches_reference(name):
    _, n, nq, k, mode, seed = BASES[name]
    w = workloads.clustered(n=n, nq=nq, C=16, seed=seed, label_mode=mode)
    x32, q32 = workloads.float32_inputs(w, seed)
    assert _sha(x32, q32) == str(G5[f"base_{name}__sha"])
    D = O.pairwise_cosine(x32, q32).T  # Baseline.py:17
    nns = np.argsort(D, kind="stable")[:, :k] + 1
    dists = np.sort(D)[:, :k]
    ref_d, ref_n = G5[f"base_{name}__dists"], G5[f"base_{name}__nns"]
    assert ref_d.dtype == np.float32
    assert O.compare_lists(ref_d, ref_n, dists, nns, atol=1e-5, tie=TIE32) == 0
