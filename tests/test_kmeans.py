"""Row f3 (index build k-means) on the CPU: the oracle's Lloyd restatement
(oracle/lmi_oracle.py::kmeans_*) pinned to sklearn's published Lloyd
(KMeans(algorithm="lloyd") with the same explicit init), and the product's
host half (li/kmeans.py::split_empty, faiss split_clusters) equal to the
oracle's.  The GPU kernels are checked against the oracle in
test_gpu_kmeans.py.  faiss itself is absent: its RNG-dependent sample / init
/ split choices are not reproduced ("parity unpinned" against faiss)."""
import numpy as np
import pytest

import lmi_oracle as O


def _blobs(n, d, c, seed, spread=0.15):
    rng = np.random.default_rng(seed)
    centres = rng.standard_normal((c, d)).astype(np.float32)
    lab = rng.integers(0, c, n)
    return (centres[lab] + spread * rng.standard_normal((n, d))).astype(np.float32)


def test_assign_matches_float64_argmin():
    x = _blobs(2000, 40, 12, 0)
    cent = x[np.random.default_rng(1).permutation(2000)[:12]]
    lab, dist = O.kmeans_assign(x, cent)
    d64 = ((x[:, None, :].astype(np.float64) - cent[None].astype(np.float64)) ** 2).sum(-1)
    assert (lab == d64.argmin(1)).all()
    np.testing.assert_allclose(dist, d64.min(1), rtol=1e-5)


def test_assign_ties_lower_index():
    x = np.zeros((3, 4), np.float32)
    cent = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [1, 0, 0, 0]], np.float32)
    lab, dist = O.kmeans_assign(x, cent)
    assert lab.tolist() == [0, 0, 0] and dist.tolist() == [1.0, 1.0, 1.0]


@pytest.mark.parametrize("n,d,k,seed", [(3000, 24, 8, 0), (5000, 96, 20, 1)])
def test_lloyd_matches_sklearn(n, d, k, seed):
    from sklearn.cluster import KMeans
    x = _blobs(n, d, k, seed)
    c0 = x[np.random.RandomState(seed).permutation(n)[:k]].copy()
    niter = 6
    cent = c0.copy()
    for _ in range(niter):
        lab, _ = O.kmeans_assign(x, cent)
        cent, cnt = O.kmeans_update(x, lab, cent)
        assert (cnt > 0).all()
    km = KMeans(n_clusters=k, init=c0, n_init=1, max_iter=niter, tol=0.0,
                algorithm="lloyd").fit(x)
    np.testing.assert_allclose(cent, km.cluster_centers_, rtol=1e-5, atol=1e-6)
    lab, _ = O.kmeans_assign(x, cent)
    assert (lab == km.predict(x)).mean() > 0.999


def test_update_slices_and_empty_rows():
    x = _blobs(5000, 16, 5, 3)
    lab = np.random.default_rng(0).integers(0, 4, 5000).astype(np.int32)  # cluster 4 empty
    cent = np.full((5, 16), 7.0, np.float32)
    out, cnt = O.kmeans_update(x, lab, cent)
    assert O.kmeans_slices(5000) == 40 and cnt[4] == 0 and (out[4] == 7.0).all()
    for c in range(4):
        np.testing.assert_allclose(out[c], x[lab == c].astype(np.float64).mean(0), rtol=1e-6)


def test_split_empty_product_equals_oracle():
    from li.kmeans import split_empty
    rng0 = np.random.default_rng(5)
    cent = rng0.standard_normal((10, 7)).astype(np.float32)
    counts = np.array([0, 30, 0, 5, 1, 0, 40, 2, 9, 13], np.int64)
    a_c, a_n = cent.copy(), counts.copy()
    b_c, b_n = cent.copy(), counts.copy()
    na = split_empty(a_c, a_n, 100, np.random.RandomState(1234))
    nb = O.kmeans_split_empty(b_c, b_n, 100, np.random.RandomState(1234))
    assert na == nb == 3
    assert (a_n == b_n).all() and a_n.sum() == counts.sum() and (a_n > 0).all()
    assert (a_c.view(np.uint32) == b_c.view(np.uint32)).all()


def test_train_sample_and_convergence():
    x = _blobs(6000, 32, 10, 7)
    sel = O.kmeans_train_sample(6000, 10, 2023, max_points_per_centroid=256)
    assert sel.size == 2560 and np.unique(sel).size == 2560
    cent, obj = O.kmeans_train(x, 10, niter=10, seed=2023)
    assert all(b <= a * (1 + 1e-6) for a, b in zip(obj, obj[1:]))  # Lloyd never increases it
