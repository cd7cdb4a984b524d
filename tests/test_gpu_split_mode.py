"""The split mode (ABI 9, lmi_index_desc.corpus32): float32 corpora that are
not fp16-exact.  The fp16 scan runs on the normalised fp16 rounding of rows
and queries, every row within d~_k + 2 eps_x is collected, and the
candidates are re-scored exactly (float64, rounded to float32 for the float32
arithmetic).  Checked against the oracle's lists (the reference's float32 /
float64 arithmetic restated, pinned by tests/golden/reference_outputs_r5.npz)
and the reference's own outputs through the drop-in (test_gpu_golden_r5.py's
cases live here too)."""
import numpy as np
import pandas as pd
import pytest
import torch

import lmi_oracle as O
import workloads
from li import _lib
from li.index import (DeviceIndex, DeviceRouter, Searcher, bucket_topk, bucket_topk_f64,
                      split_sample_fallback_count)
from test_oracle_golden_r5 import BASES, CASES, G5, SINGLES, check, inputs_r5

pytestmark = pytest.mark.gpu
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731


def _x(mode, seed, n=6000, nq=200, C=16):
    w = workloads.clustered(n=n, nq=nq, C=C, seed=seed, label_mode=mode)
    x32, q32 = workloads.float32_inputs(w, seed)
    return w, x32, q32


def test_split_eps_bound():
    lib = _lib.load()
    eps = lib.lmi_split_eps(768)
    # 2 asin(2^-11 + 2^-22 + sqrt(768) 2^-25) + the fp16 scan's arithmetic
    assert 9.7e-4 < eps < 1.0e-3


@pytest.mark.parametrize("mode,seed", [("near", 601), ("dup", 602), ("skewed", 603)])
@pytest.mark.parametrize("k", [1, 10, 12, 16])
def test_split_lists_match_oracle(mode, seed, k):
    """k <= 10: the collect bound from the k-th of each bucket's sample (its
    first chunk); 11-15: from the sampled chunk lists' 15th; 16: from a whole
    first scan -- the same exact lists."""
    w, x, q = _x(mode, seed)
    C, R = w["C"], 4
    ix = DeviceIndex(x, w["labels"], C, chunk_rows=512, device="cuda")
    assert ix.storage == "f32x" and ix.corpus32 is not None
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    cls = T(classes.astype(np.int32))
    d, p, st = bucket_topk(ix, T(q), cls, k)
    assert int(st.item()) == 0
    ref_d, ref_p = O.bucket_lists(w["labels"], x, q, classes, R, k, C)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), p.cpu().numpy(), atol=1e-5, tie=1e-6) == 0
    # the float64 arithmetic (float64 queries: the reference computes in float64)
    q64 = q.astype(np.float64)
    d64, p64, st64, nfb = bucket_topk_f64(ix, T(q64), cls, k, fallback_count=True)
    assert int(st64.item()) == 0 and nfb == 0
    ref_d64, ref_p64 = O.bucket_lists(w["labels"], x, q64, classes, R, k, C)
    assert O.compare_lists(ref_d64, ref_p64, d64.cpu().numpy(), p64.cpu().numpy(), atol=1e-12,
                           tie=1e-12) == 0


@pytest.mark.parametrize("dist", ["f32", "f64"])
def test_split_multi_chunk_sample(dist):
    """Buckets of ~4500 rows at 128-row chunks: each bucket's sample (n_c / 16
    rows, rounded up to 32, at least one chunk) spans several chunks of the
    sample descriptor; the lists equal the oracle's."""
    w, x, q = _x("router", 641, n=9000, nq=96, C=2)
    C, R = w["C"], 2
    ix = DeviceIndex(x, w["labels"], C, chunk_rows=128, device="cuda")
    assert int(np.bincount(w["labels"], minlength=C).max()) // 16 > 2 * 128
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    cls = T(classes.astype(np.int32))
    if dist == "f32":
        d, p, st = bucket_topk(ix, T(q), cls, 10)
        ref_d, ref_p = O.bucket_lists(w["labels"], x, q, classes, R, 10, C)
        tol = dict(atol=1e-5, tie=1e-6)
    else:
        q64 = q.astype(np.float64)
        d, p, st, nfb = bucket_topk_f64(ix, T(q64), cls, 10, fallback_count=True)
        assert nfb == 0
        ref_d, ref_p = O.bucket_lists(w["labels"], x, q64, classes, R, 10, C)
        tol = dict(atol=1e-12, tie=1e-12)
    assert int(st.item()) == 0
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), p.cpu().numpy(), **tol) == 0


@pytest.mark.parametrize("in_sample,n_near", [(16, 24), (8, 24), (16, 300)])
def test_split_skipped_sample_rows(in_sample, n_near):
    """Buckets of thousands of rows at 128-row chunks: the collect scan skips
    each bucket's sample (n_c / 16 rows, under a quarter of it) and takes the
    sample scan's own list for it.  16 near-copies of one vector at the front of a
    bucket (all in its sample) and queries next to them: the pairs' band
    reaches the sample's 10th, so they are scored over their sample rows and
    candidates (the count says they were; 300 such pairs: past the 256 sliced
    ones, a workgroup each); 8 in the sample and 8 at the
    bucket's end: the list covers the sample.  Both arithmetics equal the oracle's lists."""
    w, x, q = _x("router", 643, n=9000, nq=max(96, n_near + 20), C=2)
    C = w["C"]
    rng = np.random.default_rng(7)
    b = 0
    rows = np.nonzero(w["labels"] == b)[0]
    assert rows.size >= 4 * 128
    # (the sample: the bucket's first max(128, n_c / 16 rounded up to 32) rows)
    near = np.concatenate([rows[:in_sample], rows[rows.size - (16 - in_sample):]])
    x = x.copy()
    # (a direction of its own, far from every clustered row: past the near
    # copies, a bucket's next rows lie well outside any band)
    v = rng.standard_normal(x.shape[1]) * (np.linalg.norm(x[near[0]]) / np.sqrt(x.shape[1]))
    x[near] = (v * (1 + 1e-3 * rng.standard_normal((near.size, x.shape[1])))).astype(np.float32)
    q = q.copy()
    q[:n_near] = (v * (1 + 1e-3 * rng.standard_normal((n_near, x.shape[1])))).astype(np.float32)
    ix = DeviceIndex(x, w["labels"], C, chunk_rows=128, device="cuda")
    classes = np.tile(np.array([[b, 1 - b]], np.int64), (q.shape[0], 1))
    cls = T(classes.astype(np.int32))
    nq, R = q.shape[0], 2
    d, p, st = bucket_topk(ix, T(q), cls, 10)
    assert int(st.item()) == 0
    ns = split_sample_fallback_count(ix, nq, R, 10)
    assert (ns >= n_near) if in_sample == 16 else (ns < n_near)
    ref_d, ref_p = O.bucket_lists(w["labels"], x, q, classes, R, 10, C)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), p.cpu().numpy(), atol=1e-5, tie=1e-6) == 0
    q64 = q.astype(np.float64)
    d64, p64, st64, nfb = bucket_topk_f64(ix, T(q64), cls, 10, fallback_count=True)
    assert int(st64.item()) == 0 and nfb == 0
    ns64 = split_sample_fallback_count(ix, nq, R, 10, f64=True)
    assert (ns64 >= n_near) if in_sample == 16 else (ns64 < n_near)
    ref_d64, ref_p64 = O.bucket_lists(w["labels"], x, q64, classes, R, 10, C)
    assert O.compare_lists(ref_d64, ref_p64, d64.cpu().numpy(), p64.cpu().numpy(), atol=1e-12,
                           tie=1e-12) == 0


def test_split_overflow_takes_the_whole_shard():
    """A bucket of 3000 copies of one vector (relative noise 1e-4: one fp16
    value after normalising and rounding, distinct exact distances): every
    pair probing it collects more rows than the buffer holds (2048) and is
    scanned whole in float64."""
    w, x, q = _x("skewed", 611, n=8000, nq=64)
    rng = np.random.default_rng(5)
    big = int(np.bincount(w["labels"]).argmax())
    rows = np.nonzero(w["labels"] == big)[0][:3000]
    assert rows.size == 3000
    x = x.copy()
    x[rows] = (x[rows[0]].astype(np.float64) * (1 + 1e-4 * rng.standard_normal((3000, x.shape[1])))
               ).astype(np.float32)
    q = q.copy()
    q[:16] = x[rows[0]] * np.float32(1.0001)
    C = w["C"]
    ix = DeviceIndex(x, w["labels"], C, chunk_rows=512, device="cuda")
    classes = np.full((q.shape[0], 1), big, np.int64)
    cls = T(classes.astype(np.int32))
    d, p, st = bucket_topk(ix, T(q), cls, 10)
    ref_d, ref_p = O.bucket_lists(w["labels"], x, q, classes, 1, 10, C)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), p.cpu().numpy(), atol=1e-5, tie=1e-6) == 0
    # (ABI 11: the whole-shard path computes float32 in the reference's order:
    # one group of 64 queries x the bucket, OpenBLAS's blocked kernel)
    assert O.blas32_kernel(q.shape[0], int(np.sum(w["labels"] == big)), x.shape[1]) == "blocked"
    np.testing.assert_array_equal(d.cpu().numpy(), ref_d)
    d64, p64, st64, nfb = bucket_topk_f64(ix, T(q.astype(np.float64)), cls, 10, fallback_count=True)
    assert nfb > 0  # the whole-shard path ran
    ref_d64, ref_p64 = O.bucket_lists(w["labels"], x, q.astype(np.float64), classes, 1, 10, C)
    assert O.compare_lists(ref_d64, ref_p64, d64.cpu().numpy(), p64.cpu().numpy(), atol=1e-12,
                           tie=1e-12) == 0


def test_split_search_and_striped_shards_match_oracle():
    """Searcher.search end to end (router, lists, device replay) in both
    arithmetics, and the lists of a 3-way striped index merged = one GPU."""
    from li.index import merge_topk
    w, x, q = _x("near", 621)
    C = w["C"]
    ix = DeviceIndex(x, w["labels"], C, chunk_rows=512, device="cuda")
    s = Searcher(ix, DeviceRouter(w["layers"], device="cuda"))
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))
    ids = np.arange(1, x.shape[0] + 1)
    for dist_, qq in (("f32", q), ("f64", q.astype(np.float64))):
        d, a = s.search(T(w["qn"]), T(qq), 4, k=10, dist=dist_)
        ref_d, ref_a = O.search_direct(w["labels"], ids, x, qq, classes, n_buckets=4, k=10,
                                       use_threshold=True)
        tol = dict(atol=1e-5, tie=1e-6) if dist_ == "f32" else dict(atol=1e-12, tie=1e-12)
        assert O.compare_lists(ref_d, ref_a, d, a, **tol) == 0
    cls = T(classes[:, :4].astype(np.int32))
    d1, p1, _ = bucket_topk(ix, T(q), cls, 10)
    parts = [bucket_topk(DeviceIndex(x, w["labels"], C, chunk_rows=256, device="cuda", rank=g, world=3),
                         T(q), cls, 10) for g in range(3)]
    md, mp = merge_topk(torch.stack([p_[0] for p_ in parts]), torch.stack([p_[1] for p_ in parts]), 10)
    assert torch.equal(md, d1) and torch.equal(mp, p1)


def test_split_wide_k_uses_the_general_scan():
    """k > 16 in the split mode scans the float32 rows (the general exact-fp32
    kernel, a second descriptor over corpus32)."""
    w, x, q = _x("dup", 631)
    C = w["C"]
    ix = DeviceIndex(x, w["labels"], C, chunk_rows=512, device="cuda")
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :1]
    d, p, st = bucket_topk(ix, T(q), T(classes.astype(np.int32)), 30)
    ref_d, ref_p = O.bucket_lists(w["labels"], x, q, classes, 1, 30, C)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), p.cpu().numpy(), atol=1e-5, tie=1e-6) == 0


# ---- the drop-in against the reference's own outputs (r5 fixtures) ------------
def _frames(w, x):
    data = pd.DataFrame(w["xn"])
    data.index += 1
    data_search = pd.DataFrame(x)
    data_search.index += 1
    return data, data_search


@pytest.mark.parametrize("name", list(CASES))
def test_split_dropin_search_matches_reference(name):
    from li.LearnedIndex import LearnedIndex, dist_dtype
    from test_gpu_golden_r2 import _nn
    _, n, nq, C, R, k, mode, arch, seed, thr, qdt = CASES[name]
    w, x, q, arith = inputs_r5(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    data, data_search = _frames(w, x)
    assert dist_dtype(data_search, q) == arith
    dists, anns = li.search(data, w["qn"], data_search, q, w["labels"], n_buckets=R, k=k,
                            use_threshold=thr)
    assert li._index.storage == "f32x"
    check(name, dists, anns, arith)


@pytest.mark.parametrize("name", list(SINGLES))
def test_split_dropin_search_single_matches_reference(name):
    from li.LearnedIndex import LearnedIndex
    from test_gpu_golden_r2 import _nn
    _, n, nq, C, R, k, mode, arch, seed = SINGLES[name]
    w, x, q, arith = inputs_r5(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    data, data_search = _frames(w, x)
    data["category"] = w["labels"]
    classes = G5[f"search_{name}__classes"].astype(np.int64)
    dists, anns = li.search_single(data, data_search, q, classes[:, 0], k=k)
    check(name, dists, anns, arith)


@pytest.mark.parametrize("name", list(BASES))
def test_split_dropin_baseline_matches_reference(name):
    from li.Baseline import Baseline
    _, n, nq, k, mode, seed = BASES[name]
    w = workloads.clustered(n=n, nq=nq, C=16, seed=seed, label_mode=mode)
    x32, q32 = workloads.float32_inputs(w, seed)
    dists, nns, _ = Baseline().search(q32, x32, k=k)
    ref_d, ref_n = G5[f"base_{name}__dists"], G5[f"base_{name}__nns"]
    assert O.compare_lists(ref_d, ref_n, dists, nns, atol=1e-5, tie=1e-6) == 0


@pytest.mark.parametrize("k", [10, 30])
def test_split_subcluster_layout_moves_the_float32_rows(k):
    """subcluster=True reorders the rows inside each bucket; the split mode's
    float32 rows (the exact re-score's and the k > 16 scan's input) and their
    norms move with them: the lists equal the oracle's and the
    plain layout's."""
    w, x, q = _x("near", 651, n=6000)
    C, R = w["C"], 2
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    cls = T(classes.astype(np.int32))
    ix = DeviceIndex(x, w["labels"], C, chunk_rows=256, device="cuda", subcluster=True)
    assert ix.storage == "f32x" and ix.chunk_centroid is not None
    d, p, st = bucket_topk(ix, T(q), cls, k)
    assert int(st.item()) == 0
    ref_d, ref_p = O.bucket_lists(w["labels"], x, q, classes, R, k, C)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), p.cpu().numpy(), atol=1e-5, tie=1e-6) == 0
    if k <= 16:
        q64 = q.astype(np.float64)
        d64, p64, st64 = bucket_topk_f64(ix, T(q64), cls, k)
        ref_d64, ref_p64 = O.bucket_lists(w["labels"], x, q64, classes, R, k, C)
        assert O.compare_lists(ref_d64, ref_p64, d64.cpu().numpy(), p64.cpu().numpy(), atol=1e-12,
                               tie=1e-12) == 0



@pytest.mark.parametrize("norm32", ["1", "0"])
@pytest.mark.parametrize("mode,seed", [("near", 661), ("skewed", 662), ("router", 663)])
def test_split_float32_is_the_references_own_arithmetic(mode, seed, norm32, monkeypatch):
    """ABI 10: the split mode's float32 re-score follows the reference's
    float32 operation order (oracle blas32_*: sklearn's einsum norms and
    division, OpenBLAS sgemm's summation order for the (round, bucket)
    group's shape), so wherever that shape's order is restated the lists'
    float32 distances equal the oracle's (= numpy's = the reference's) bit for
    bit and ids differ only inside runs of identical distances.  Both with the
    rows normalised once at build (ABI 11, corpus32n) and per candidate
    (LMI_SPLIT_NORM32=0)."""
    monkeypatch.setenv("LMI_SPLIT_NORM32", norm32)
    w, x, q = _x(mode, seed, n=6000, nq=200)
    C, R, k = w["C"], 4, 10
    ix = DeviceIndex(x, w["labels"], C, chunk_rows=512, device="cuda")
    assert (ix.corpus32n is not None) == (norm32 == "1")
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    d, p, st = bucket_topk(ix, T(q), T(classes.astype(np.int32)), k)
    assert int(st.item()) == 0
    ref_d, ref_p = O.bucket_lists(w["labels"], x, q, classes, R, k, C)
    sizes = np.bincount(w["labels"], minlength=C)
    keep = np.zeros(classes.shape, bool)
    kinds = set()
    for r in range(R):
        grp = np.bincount(classes[:, r], minlength=C)
        for i in range(classes.shape[0]):
            kern = O.blas32_kernel(int(grp[classes[i, r]]), int(sizes[classes[i, r]]), x.shape[1])
            keep[i, r] = kern is not None
            kinds.add(kern)
    # (groups of one query -- OpenBLAS's gemv, whose order follows its thread
    # split -- keep the exact value rounded: many at 200 queries x 16 buckets)
    assert keep.sum() > 100 and kinds & {"small", "blocked"}
    gd, gp = d.cpu().numpy()[keep], p.cpu().numpy()[keep]
    rd, rp = ref_d[keep], ref_p[keep]
    np.testing.assert_array_equal(gd, rd)     # float32 distances: bit for bit
    assert O.compare_lists(rd, rp, gd, gp, atol=0.0, tie=0.0) == 0


def test_split_normalize_is_sklearns_float32_normalize():
    """ABI 11: lmi_split_normalize (corpus32n) = sklearn's normalize(Y) in
    float32 (oracle blas32_normalize: numpy einsum norms, the zero rule, IEEE
    division), bit for bit, padding zeroed; zero rows stay zero."""
    w, x, q = _x("dup", 671, n=3000)
    x = x.copy()
    x[5] = 0.0
    ix = DeviceIndex(x, w["labels"], w["C"], chunk_rows=512, device="cuda")
    assert ix.corpus32n is not None and ix.corpus32n.shape == ix.corpus32.shape
    rows = ix.layout.order[ix.gpos.cpu().numpy().astype(np.int64)]
    got = ix.corpus32n.cpu().numpy()
    np.testing.assert_array_equal(got[:, : x.shape[1]], O.blas32_normalize(x[rows]))
    assert not got[:, x.shape[1]:].any()
    # through the C-ABI directly, rows not a multiple of 4 (a partial workgroup)
    lib = _lib.load()
    src = T(np.ascontiguousarray(x[:7]))
    out = torch.full_like(src, 7.0)
    assert lib.lmi_split_normalize(src.data_ptr(), 7, x.shape[1], x.shape[1], out.data_ptr(),
                                   _lib.stream_handle(src.device)) == 0
    np.testing.assert_array_equal(out.cpu().numpy(), O.blas32_normalize(x[:7]))
    assert lib.lmi_split_normalize(src.data_ptr(), 7, 100, 128, out.data_ptr(), None) != 0
