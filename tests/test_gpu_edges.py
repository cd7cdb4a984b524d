"""Edge cases of the GPU path against the oracle: zero vectors (sklearn's
zero-norm rule, utils.py:11), a corpus smaller than k, k = 1, one bucket,
queries routed to a single bucket, and an empty query batch."""
import numpy as np
import pytest
import torch

import lmi_oracle as O
import workloads
from li.index import DeviceIndex, DeviceRouter, Searcher, bucket_topk

pytestmark = pytest.mark.gpu


def _searcher(w, chunk_rows=256):
    return Searcher(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=chunk_rows, device="cuda"),
                    DeviceRouter(w["layers"], device="cuda"))


def _check(w, s, R, k, use_threshold=True):
    ids = np.arange(1, w["x"].shape[0] + 1)
    d, a = s.search(torch.from_numpy(w["qn"]).cuda(), torch.from_numpy(w["q"]).cuda(), R, k=k,
                    use_threshold=use_threshold)
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))
    rd, ra = O.search_direct(w["labels"], ids, w["x"], w["q"], classes, n_buckets=R, k=k,
                             use_threshold=use_threshold)
    assert O.compare_lists(rd, ra, d, a) == 0
    return d, a


def test_zero_vectors_follow_sklearn_rule():
    w = workloads.clustered(n=2000, nq=64, C=8, seed=31, label_mode="router")
    w["x"][::97] = 0.0  # zero corpus rows: norm -> 1, distance 1 - 0 = 1
    w["q"][5] = 0.0     # a zero query: every distance is 1
    d, _ = _check(w, _searcher(w), 3, 10)
    assert np.all(d[5] == 1.0)


@pytest.mark.parametrize("k", [1, 10])
def test_corpus_smaller_than_k_and_k1(k):
    w = workloads.clustered(n=40, nq=32, C=8, seed=5, label_mode="skewed")
    _check(w, _searcher(w, chunk_rows=32), 2, k)


def test_single_bucket():
    w = workloads.clustered(n=1500, nq=50, C=16, seed=8, label_mode="router")
    w["labels"] = np.zeros_like(w["labels"])  # every object in bucket 0
    _check(w, _searcher(w), 1, 10, use_threshold=False)


def test_empty_query_batch():
    w = workloads.clustered(n=500, nq=8, C=8, seed=2, label_mode="router")
    s = _searcher(w)
    ix = s.index
    q = torch.zeros((0, w["x"].shape[1]), device="cuda")
    cls = torch.zeros((0, 2), dtype=torch.int32, device="cuda")
    d, pos, st = bucket_topk(ix, q, cls, 10)
    assert d.shape == (0, 2, 10) and pos.shape == (0, 2, 10)
