"""LMI_Q_SEED_ROUND0: with the thresholded reference replay, the scan starts
every (query, probe r >= 1) pair from the bound of pair (query, 0) (the
running threshold of the reference's later rounds never exceeds round 0's
k-th distance: LearnedIndex.py:71-75, utils.py:23).  The seeded lists are
truncated, the answers must not change: bitwise equal to the unseeded search,
in both arithmetics, for every replay branch the workloads reach (tiny
buckets, duplicates, near-duplicates, k below the round width), and equal to
the oracle."""
import numpy as np
import pytest
import torch

import lmi_oracle as O
import workloads
from li import index as I

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode,R,k,dist", [
    ("skewed", 4, 10, "f32"), ("skewed", 7, 10, "f64"), ("dup", 4, 10, "f32"),
    ("near", 4, 10, "f64"), ("near", 2, 5, "f32"), ("router", 8, 10, "f32"),
    ("skewed", 3, 7, "f64")])
def test_seeded_search_equals_unseeded(mode, R, k, dist, monkeypatch):
    w = workloads.clustered(n=6000, nq=300, C=16, seed=71 + R, label_mode=mode)
    ix = I.DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda")
    s = I.Searcher(ix, I.DeviceRouter(w["layers"], device="cuda"))
    qn = torch.from_numpy(w["qn"]).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    monkeypatch.setattr(I, "_SEED_ROUND0", True)
    d1, a1 = s.search(qn, q, R, k=k, dist=dist)
    g = s.graph(w["qn"], w["q"], R, k=k, dist=dist)
    d3, a3 = g.run()
    monkeypatch.setattr(I, "_SEED_ROUND0", False)
    d0, a0 = s.search(qn, q, R, k=k, dist=dist)
    np.testing.assert_array_equal(d1, d0)
    np.testing.assert_array_equal(a1, a0)
    np.testing.assert_array_equal(d3, d0)
    np.testing.assert_array_equal(a3, a0)
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))
    x = w["x"] if dist == "f32" else w["x"].astype(np.float16)
    qq = w["q"] if dist == "f32" else w["q"].astype(np.float16)
    rd, ra = O.search_direct(w["labels"], np.arange(1, w["x"].shape[0] + 1), x, qq, classes,
                             n_buckets=R, k=k, use_threshold=True)
    tie, atol = (1e-6, 1e-5) if dist == "f32" else (1e-12, 1e-12)
    assert O.compare_lists(rd, ra, d1, a1, atol=atol, tie=tie) == 0


@pytest.fixture
def few_scan_workgroups(monkeypatch):
    """Two persistent scan workgroups (LMI_SCAN_WGS): tiles run in turn, so
    later tiles start after round-0 pairs published their bounds (with one
    workgroup per CU every tile of a small test starts at once)."""
    from li import _lib
    monkeypatch.setenv("LMI_SCAN_WGS", "2")
    _lib.load().lmi_config_reload()
    yield
    monkeypatch.delenv("LMI_SCAN_WGS")
    _lib.load().lmi_config_reload()


def test_seeded_lists_hold_every_object_under_the_round0_bound(few_scan_workgroups):
    """The seeded lists of probes r >= 1 equal the unseeded ones on every entry
    below the pair's round-0 k-th distance (what the replay reads)."""
    w = workloads.clustered(n=8000, nq=300, C=16, seed=79, label_mode="skewed")
    # many chunks per bucket: the seed applies from a pair's first tile that
    # starts after its round-0 pair published a bound
    ix = I.DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=64, device="cuda")
    classes = torch.from_numpy(np.ascontiguousarray(
        O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :4], dtype=np.int32)).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    d0, p0, _ = I.bucket_topk(ix, q, classes, 10)
    d1, p1, _ = I.bucket_topk(ix, q, classes, 10, seed_round0=True)
    d0, p0, d1, p1 = (t.cpu().numpy() for t in (d0, p0, d1, p1))
    np.testing.assert_array_equal(d1[:, 0], d0[:, 0])
    np.testing.assert_array_equal(p1[:, 0], p0[:, 0])
    thr0 = d0[:, 0, 9][:, None]
    for r in range(1, 4):
        keep = d0[:, r] < thr0
        assert np.array_equal(np.where(keep, d0[:, r], 0), np.where(keep, d1[:, r], 0))
        assert np.array_equal(np.where(keep, p0[:, r], 0), np.where(keep, p1[:, r], 0))
    assert (p1[:, 1:] < 0).sum() > (p0[:, 1:] < 0).sum()   # the seed did prune
