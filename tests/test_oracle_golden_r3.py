"""Pin the oracle and the product's host replay to the reference's own outputs
on float64 INPUTS (tests/golden/reference_outputs_r3.npz, written by
tests/golden/gen_golden_r3.py running the reference itself): float64 data
and/or queries, where sklearn computes float64 distances on the float64
values (utils.py:11, :19).  The inputs carry a perturbation below half a
float32 ulp (tests/workloads.float64_inputs), so the fixtures are sharp:
computing on the float32-rounded inputs flips ids."""
import hashlib
import os

import numpy as np
import pytest

import lmi_oracle as O
import workloads
from golden.gen_golden_r3 import F64_BASELINE, F64_SEARCH, F64_SINGLE

HERE = os.path.dirname(os.path.abspath(__file__))
G3 = np.load(os.path.join(HERE, "golden", "reference_outputs_r3.npz"))
CASES = {c[0]: c for c in F64_SEARCH}
SINGLES = {c[0]: c for c in F64_SINGLE}
BASES = {c[0]: c for c in F64_BASELINE}
TIE64 = 1e-12


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(a.tobytes())
    return h.hexdigest()


def inputs_r3(name):
    """(workload, data_search values, queries) of a case, checked against the
    fixture's input hash."""
    if name in CASES:
        _, n, nq, C, R, k, mode, arch, seed, thr, fd, fq = CASES[name]
    else:
        (_, n, nq, C, R, k, mode, arch, seed), fd, fq = SINGLES[name], True, True
    w = workloads.clustered(n=n, nq=nq, C=C, arch=arch, seed=seed, label_mode=mode)
    x64, q64 = workloads.float64_inputs(w, seed)
    assert _sha(x64, q64, w["xn"], w["qn"], w["labels"]) == str(G3[f"search_{name}__sha"]), \
        "input generator drifted"
    return w, (x64 if fd else w["x"]), (q64 if fq else w["q"])


def check(name, dists, anns):
    ref_d, ref_a = G3[f"search_{name}__dists"], G3[f"search_{name}__anns"]
    assert dists.shape == ref_d.shape
    assert O.compare_lists(ref_d, ref_a, dists, anns, atol=1e-12, tie=TIE64) == 0


def test_fixture_inventory_r3():
    keys = {k.split("__")[0] for k in G3.files}
    assert len(keys) == len(F64_SEARCH) + len(F64_SINGLE) + len(F64_BASELINE)
    for c in F64_SEARCH:
        assert G3[f"search_{c[0]}__dists"].dtype == np.float64


@pytest.mark.parametrize("name", list(CASES))
def test_f64_search_direct_matches_reference(name):
    _, n, nq, C, R, k, mode, arch, seed, thr, fd, fq = CASES[name]
    w, x, q = inputs_r3(name)
    classes = G3[f"search_{name}__classes"].astype(np.int64)
    d, a = O.search_direct(w["labels"], np.arange(1, n + 1), x, q, classes, n_buckets=R, k=k,
                           use_threshold=thr)
    check(name, d, a)


@pytest.mark.parametrize("name", list(CASES))
def test_f64_lists_plus_replay_match_reference(name):
    from li.index import replay as lmi_replay
    _, n, nq, C, R, k, mode, arch, seed, thr, fd, fq = CASES[name]
    w, x, q = inputs_r3(name)
    classes = G3[f"search_{name}__classes"].astype(np.int64)
    order, off = O.layout(w["labels"], C)
    lists_d, lists_p = O.bucket_lists(w["labels"], x, q, classes, R, 10, C)
    assert lists_d.dtype == np.float64
    kw = dict(k_round=10, k_final=k, bucket_size=np.diff(off),
              pos_to_id=np.arange(1, n + 1)[order], use_threshold=thr)
    d, a = O.replay(classes[:, :R], lists_d, lists_p, **kw)
    check(name, d, a)
    d2, a2 = lmi_replay(classes[:, :R], lists_d, lists_p, **kw)
    np.testing.assert_array_equal(d2, d)
    np.testing.assert_array_equal(a2, a)


def test_f64_fixtures_hold_float32_rounding_flips():
    """Sharp: the same search on the float32-rounded inputs (float32 data and
    queries, whatever the arithmetic) disagrees with the reference's ids."""
    flips = 0
    for name, c in CASES.items():
        _, n, nq, C, R, k, mode, arch, seed, thr, fd, fq = c
        if not (fd and fq):
            continue
        w, x, q = inputs_r3(name)
        classes = G3[f"search_{name}__classes"].astype(np.int64)
        d, a = O.search_direct(w["labels"], np.arange(1, n + 1), x.astype(np.float32).astype(np.float64),
                               q.astype(np.float32).astype(np.float64), classes, n_buckets=R, k=k,
                               use_threshold=thr)
        flips += O.compare_lists(G3[f"search_{name}__dists"], G3[f"search_{name}__anns"], d, a,
                                 atol=1e-5, tie=TIE64)
    assert flips > 0


@pytest.mark.parametrize("name", list(SINGLES))
def test_f64_search_single_matches_reference(name):
    from li.index import replay as lmi_replay
    _, n, nq, C, R, k, mode, arch, seed = SINGLES[name]
    w, x, q = inputs_r3(name)
    classes = G3[f"search_{name}__classes"].astype(np.int64)
    d, a = O.search_single_direct(w["labels"], np.arange(1, n + 1), x, q, classes[:, 0], k=k)
    check(name, d, a)
    order, off = O.layout(w["labels"], C)
    lists_d, lists_p = O.bucket_lists(w["labels"], x, q, classes, 1, k, C)
    d2, a2 = lmi_replay(classes[:, :1], lists_d, lists_p, k_round=k, k_final=k,
                        bucket_size=np.diff(off), pos_to_id=np.arange(1, n + 1)[order],
                        use_threshold=False)
    check(name, d2, a2)


@pytest.mark.parametrize("name", list(BASES))
def test_f64_baseline_oracle_matches_reference(name):
    _, n, nq, k, mode, seed = BASES[name]
    w = workloads.clustered(n=n, nq=nq, C=16, seed=seed, label_mode=mode)
    x64, q64 = workloads.float64_inputs(w, seed)
    assert _sha(x64, q64) == str(G3[f"base_{name}__sha"])
    D = O.pairwise_cosine(x64, q64).T  # Baseline.py:17
    nns = np.argsort(D, kind="stable")[:, :k] + 1
    dists = np.sort(D)[:, :k]
    ref_d, ref_n = G3[f"base_{name}__dists"], G3[f"base_{name}__nns"]
    assert ref_d.dtype == np.float64
    assert O.compare_lists(ref_d, ref_n, dists, nns, atol=1e-12, tie=TIE64) == 0
