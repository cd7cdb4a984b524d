"""Row f3 on the GPU: the k-means kernels (csrc/lmi_kmeans.hip) against the
oracle's restatement (oracle/lmi_oracle.py::kmeans_*), bit for bit — labels,
distances, centroids and counts — and the faiss.Kmeans stand-in
(li/kmeans.py) end to end, including the training sample, empty-cluster
splits and LearnedIndex.cluster."""
import numpy as np
import pandas as pd
import pytest
import torch

import lmi_oracle as O
from li import kmeans as K
from li.LearnedIndex import LearnedIndex

pytestmark = pytest.mark.gpu


def _blobs(n, d, c, seed, spread=0.15):
    rng = np.random.default_rng(seed)
    centres = rng.standard_normal((c, d)).astype(np.float32)
    lab = rng.integers(0, c, n)
    return (centres[lab] + spread * rng.standard_normal((n, d))).astype(np.float32)


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("n,d,k", [(1, 5, 1), (777, 24, 7), (5000, 96, 122), (3001, 100, 40),
                                   (2000, 128, 300), (4000, 96, 700)])
def test_assign_bitwise(n, d, k):
    x = _blobs(n, d, max(2, k // 3), n + d)
    cent = _blobs(k, d, max(2, k // 3), k)
    lab, dist = K.assign(torch.from_numpy(x).cuda(), torch.from_numpy(cent).cuda())
    ol, od = O.kmeans_assign(x, cent)
    assert (lab.cpu().numpy() == ol).all()
    assert (_bits(dist.cpu().numpy()) == _bits(od)).all()


def test_assign_ties_and_duplicates():
    x = np.zeros((300, 96), np.float32)
    x[::2, 3] = 1.0
    cent = np.zeros((6, 96), np.float32)
    cent[[1, 4], 3] = 1.0  # 0,2,3,5 tie at the origin; 1 and 4 tie at e_3
    lab, _ = K.assign(torch.from_numpy(x).cuda(), torch.from_numpy(cent).cuda())
    assert (lab.cpu().numpy() == np.where(np.arange(300) % 2 == 0, 1, 0)).all()


@pytest.mark.parametrize("n,d,k", [(999, 24, 9), (70000, 96, 122), (300000, 96, 122)])
def test_update_bitwise(n, d, k):
    x = _blobs(n, d, k, 11)
    rng = np.random.default_rng(2)
    lab = rng.integers(0, k, n).astype(np.int32)
    lab[lab == k - 1] = 0  # one empty cluster keeps its row
    cent = rng.standard_normal((k, d)).astype(np.float32)
    c_dev = torch.from_numpy(cent).cuda()
    cnt = K.update(torch.from_numpy(x).cuda(), torch.from_numpy(lab).cuda(), c_dev)
    oc, ocnt = O.kmeans_update(x, lab, cent)
    assert (cnt.cpu().numpy() == ocnt).all()
    assert (_bits(c_dev.cpu().numpy()) == _bits(oc)).all()


def test_update_rejects_bad_label():
    x = torch.zeros((10, 8), device="cuda")
    lab = torch.full((10,), 3, dtype=torch.int32, device="cuda")
    with pytest.raises(RuntimeError):
        K.update(x, lab, torch.zeros((2, 8), device="cuda"))


@pytest.mark.parametrize("n,d,k,mppc,dup", [(3000, 24, 16, 8, False), (4000, 96, 122, 256, False),
                                            (2000, 32, 20, 256, True)])
def test_train_bitwise_with_oracle(n, d, k, mppc, dup):
    x = _blobs(n, d, k, 5)
    if dup:  # many exact duplicates: identical initial centroids, empty clusters, splits
        x[: n // 2] = x[0]
    km = K.Kmeans(d, k, niter=12, seed=2023, max_points_per_centroid=mppc)
    km.train(x)
    oc, oobj = O.kmeans_train(x, k, niter=12, seed=2023, max_points_per_centroid=mppc)
    assert (_bits(km.centroids) == _bits(oc)).all()
    np.testing.assert_allclose(km.obj, oobj, rtol=1e-9)
    D, I = km.index.search(x, 1)
    ol, od = O.kmeans_assign(x, oc)
    assert I.shape == (n, 1) and I.dtype == np.int64 and (I[:, 0] == ol).all()
    assert (_bits(D[:, 0]) == _bits(od)).all()


def test_learned_index_cluster():
    x = _blobs(6000, 96, 30, 9)
    df = pd.DataFrame(x)
    df.index += 1
    km, labels = LearnedIndex().cluster(df, 30)
    oc, _ = O.kmeans_train(x, 30, niter=25, seed=2023)
    assert (labels == O.kmeans_assign(x, oc)[0]).all()
    # reference's small-data rule (LearnedIndex.py:265-268)
    _, small = LearnedIndex().cluster(pd.DataFrame(x[:50]), 100)
    assert small.max() < 10
