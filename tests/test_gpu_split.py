"""Tail split (tail_split_kernel, LMI_SCAN_SPLIT / LMI_SCAN_SPLIT_PARTS): the last
tiles of every scan queue replaced by S row parts must not change a single list entry
-- bitwise equal to the unsplit scan, in both arithmetics, for k <= 10, the
float64 mode's 15-entry lists and the k > 16 lower-bound passes, and equal to
the oracle."""
import numpy as np
import pytest
import torch

import lmi_oracle as O
import workloads
from li import _lib
from li import index as I

pytestmark = pytest.mark.gpu


def _lists(ix, q, classes, k, dist, split, groups=None, parts=None):
    import os
    for var, val in (("LMI_SCAN_SPLIT", split), ("LMI_SCAN_GROUPS", groups),
                     ("LMI_SCAN_SPLIT_PARTS", parts)):
        if val is None:
            os.environ.pop(var, None)
        else:
            os.environ[var] = str(val)
    _lib.load().lmi_config_reload()
    try:
        r = (I.bucket_topk_f64 if dist == "f64" else I.bucket_topk)(ix, q, classes, k)
        d, p, st = r[0], r[1], r[2]
        assert int(st.item()) & _lib.LMI_STATUS_INTERNAL == 0
        return d.cpu().numpy(), p.cpu().numpy()
    finally:
        os.environ.pop("LMI_SCAN_SPLIT", None)
        os.environ.pop("LMI_SCAN_GROUPS", None)
        os.environ.pop("LMI_SCAN_SPLIT_PARTS", None)
        _lib.load().lmi_config_reload()


@pytest.mark.parametrize("k,dist", [(10, "f32"), (10, "f64"), (7, "f32"), (40, "f32")])
@pytest.mark.parametrize("chunk_rows", [256, 2048])
def test_split_lists_equal_unsplit(k, dist, chunk_rows):
    w = workloads.clustered(n=20000, nq=600, C=12, seed=91, label_mode="skewed")
    ix = I.DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=chunk_rows, device="cuda")
    classes = torch.from_numpy(np.ascontiguousarray(
        O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :3], dtype=np.int32)).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    d0, p0 = _lists(ix, q, classes, k, dist, -1)       # off
    # default K (the queue's share of the grid), a few others, and one queue
    # (K = 256: nearly every tile of these small workloads is halved, many
    # chunks of one pair block)
    for split, groups in ((None, None), (1, None), (3, None), (256, None), (None, 1), (7, 2)):
        d1, p1 = _lists(ix, q, classes, k, dist, split, groups)
        np.testing.assert_array_equal(p1, p0)
        np.testing.assert_array_equal(d1, d0)
    # S row parts per split tile (3, 4, 8), default K and every tile split
    for parts in (3, 4, 8):
        for split in (None, 256):
            d1, p1 = _lists(ix, q, classes, k, dist, split, None, parts)
            np.testing.assert_array_equal(p1, p0)
            np.testing.assert_array_equal(d1, d0)


def test_split_search_matches_oracle():
    w = workloads.clustered(n=12000, nq=300, C=10, seed=93, label_mode="router")
    ix = I.DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda")
    s = I.Searcher(ix, I.DeviceRouter(w["layers"], device="cuda"))
    d, a = s.search(torch.from_numpy(w["qn"]).cuda(), torch.from_numpy(w["q"]).cuda(), 4, k=10)
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))
    rd, ra = O.search_direct(w["labels"], np.arange(1, w["x"].shape[0] + 1), w["x"], w["q"], classes,
                             n_buckets=4, k=10, use_threshold=True)
    assert O.compare_lists(rd, ra, d, a, atol=1e-5, tie=1e-6) == 0
