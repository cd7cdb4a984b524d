"""k > 16 by bound + collect (csrc/lmi_scan.hip, bucket_topk_wide): a chunk-list
scan (every bucket cut into 2 kw / 15 lists, each the top-15 of a sample of its
rows) gives each pair a bound -- the kw-th smallest of its lists' distances --,
a collect scan gathers every row within it, a sort keeps the first kw; buckets
too small for kw list entries are collected whole, pairs whose candidates
overflow take the lower-bound passes.  Every list
entry must equal the passes alone (LMI_WIDE_PASSES=1) bit for bit, in both
arithmetics, with and without the tail split, and the oracle."""
import os

import numpy as np
import pytest
import torch

import lmi_oracle as O
import workloads
from li import _lib
from li import index as I

pytestmark = pytest.mark.gpu


def _lists(ix, q, classes, k, dist="f32", **env):
    keys = ("LMI_WIDE_PASSES", "LMI_WIDE_NO_FIXUP", "LMI_SCAN_SPLIT", "LMI_SCAN_SPLIT_PARTS",
            "LMI_SCAN_WGS")
    for var in keys:
        os.environ.pop(var, None)
    for var, val in env.items():
        os.environ[var] = str(val)
    _lib.load().lmi_config_reload()
    try:
        r = (I.bucket_topk_f64 if dist == "f64" else I.bucket_topk)(ix, q, classes, k)
        assert int(r[2].item()) & _lib.LMI_STATUS_INTERNAL == 0
        return r[0].cpu().numpy(), r[1].cpu().numpy()
    finally:
        for var in keys:
            os.environ.pop(var, None)
        _lib.load().lmi_config_reload()


def _fixed_pairs(ix, q, ct, k, d1, p1, dist="f32"):
    """Pairs the fix-up passes answered: those whose lists change when they
    are skipped (LMI_WIDE_NO_FIXUP, diagnostic)."""
    _, pn = _lists(ix, q, ct, k, dist, LMI_WIDE_NO_FIXUP=1)
    return int((pn != p1).reshape(-1, pn.shape[-1]).any(axis=1).sum())


def _setup(w, R, chunk_rows):
    ix = I.DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=chunk_rows, device="cuda")
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    ct = torch.from_numpy(np.ascontiguousarray(classes, dtype=np.int32)).cuda()
    return ix, classes, ct, torch.from_numpy(w["q"]).cuda()


@pytest.mark.parametrize("label_mode", ["skewed", "dup", "near"])
@pytest.mark.parametrize("k", [17, 40, 100])
@pytest.mark.parametrize("chunk_rows", [128, 512])
def test_wide_equals_passes(label_mode, k, chunk_rows):
    w = workloads.clustered(n=20000, nq=400, C=12, seed=61, label_mode=label_mode)
    R = 3
    ix, classes, ct, q = _setup(w, R, chunk_rows)
    d0, p0 = _lists(ix, q, ct, k, LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q, ct, k)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)
    if label_mode == "skewed" and chunk_rows == 128:
        ref_d, ref_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, k, w["C"])
        assert O.compare_lists(ref_d, ref_p, d1, p1) == 0
    if label_mode != "dup":
        # every bucket gives a bound (2 kw / 15 lists) or is collected whole:
        # the fix-up passes answer few pairs (candidates past the slots)
        assert _fixed_pairs(ix, q, ct, k, d1, p1) <= classes.size // 20


@pytest.mark.parametrize("split,parts", [(-1, None), (256, None), (256, 4), (3, 3)])
def test_wide_with_and_without_tail_split(split, parts):
    """The bound reads every part list of a split chunk (slots parts * X + bit)."""
    w = workloads.clustered(n=24000, nq=500, C=10, seed=67, label_mode="skewed")
    ix, _, ct, q = _setup(w, 2, 256)
    env = {"LMI_SCAN_SPLIT": split}
    if parts:
        env["LMI_SCAN_SPLIT_PARTS"] = parts
    d0, p0 = _lists(ix, q, ct, 33, LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q, ct, 33, **env)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)


def test_wide_overflowing_pairs_take_the_passes():
    """A bucket of one repeated vector: every row ties at the bound, the
    candidates overflow the pair's slots, the fix-up passes answer those pairs
    (ties in position order) while the other pairs keep the collected lists."""
    w = workloads.clustered(n=20000, nq=300, C=8, seed=71, label_mode="router")
    x = w["x"].copy()
    big = np.bincount(w["labels"], minlength=w["C"]).argmax()
    rows = np.nonzero(w["labels"] == big)[0]
    x[rows] = x[rows[0]]
    w = dict(w, x=x)
    R = 2
    ix, classes, ct, q = _setup(w, R, 256)
    assert (classes == big).any()
    d0, p0 = _lists(ix, q, ct, 50, LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q, ct, 50)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)
    big_pairs = int((classes == big).sum())
    nfix = _fixed_pairs(ix, q, ct, 50, d1, p1)
    assert big_pairs <= nfix < classes.size
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, 50, w["C"])
    assert O.compare_lists(ref_d, ref_p, d1, p1) == 0


@pytest.mark.parametrize("k", [11, 26, 60])
def test_wide_float64_refinement_equals_passes(k):
    """The float64 mode refines k + 5 entries: k >= 11 takes the wide lists
    (with their rows) under the float64 recomputation."""
    w = workloads.clustered(n=16000, nq=300, C=10, seed=73, label_mode="near")
    ix, _, ct, q = _setup(w, 3, 256)
    d0, p0 = _lists(ix, q, ct, k, "f64", LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q, ct, k, "f64")
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)


def test_wide_few_workgroups_and_r1():
    """R = 1 and a 7-workgroup scan grid (tiles of one pair run one after
    another): the same lists."""
    w = workloads.clustered(n=12000, nq=200, C=6, seed=79, label_mode="skewed")
    ix, _, ct, q = _setup(w, 1, 256)
    d0, p0 = _lists(ix, q, ct, 64, LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q, ct, 64, LMI_SCAN_WGS=7)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)


@pytest.mark.parametrize("k", [40, 100])
def test_wide_sampled_bound(k):
    """Large buckets: the bound scan reads the first quarter of every list (a
    sample); its kw-th smallest still bounds the pair's kw-th distance, the
    collect scan finds ~4 kw rows within it."""
    w = workloads.clustered(n=60000, nq=300, C=6, seed=83, label_mode="router")
    R = 2
    ix, classes, ct, q = _setup(w, R, 2048)
    d0, p0 = _lists(ix, q, ct, k, LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q, ct, k)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)
    assert _fixed_pairs(ix, q, ct, k, d1, p1) <= classes.size // 20
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, k, w["C"])
    assert O.compare_lists(ref_d, ref_p, d1, p1) == 0


def test_wide_edges_tiny_batch_max_k_and_out_of_range_classes():
    """One query, R = 1, k = 17; k = 1024 on buckets smaller than k (pads past
    the bucket); pairs whose class is out of range (-1, C) keep (+inf, -1) --
    all equal to the passes."""
    w = workloads.clustered(n=6000, nq=64, C=8, seed=89, label_mode="skewed")
    ix, _, ct, q = _setup(w, 2, 256)
    d0, p0 = _lists(ix, q[:1], ct[:1, :1].contiguous(), 17, LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q[:1], ct[:1, :1].contiguous(), 17)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)
    d0, p0 = _lists(ix, q, ct, 1024, LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q, ct, 1024)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)
    assert (p1 == -1).any()  # buckets under 1024 rows: padded
    bad = ct.clone()
    bad[::3, 0] = -1
    bad[1::3, 1] = w["C"]
    d0, p0 = _lists(ix, q, bad, 40, LMI_WIDE_PASSES=1)
    d1, p1 = _lists(ix, q, bad, 40)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(d1, d0)
    assert (p1[::3, 0] == -1).all() and np.isinf(d1[::3, 0]).all()
