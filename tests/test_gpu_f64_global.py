"""ABI 10, lmi_bucket_topk_f64g: the float64 band of a striped index decided
over every rank's lists.  Each stripe's MERGE phase
writes its pairs' k smallest d32; the G blocks (what the all-gather hands
every rank) give each pair's k-th over all ranks, and each stripe's REFINE
phase refines only its rows of that merged band.  K3 over the stripes'
outputs must equal the one-GPU float64 lists bit for bit (and the round-5
per-rank form's), with and without the round-0 seed, on workloads with tied
and near-tied runs (the fallback), float16 and float64 inputs."""
import numpy as np
import pytest
import torch

import lmi_oracle as O
import workloads
from li import _lib
from li.index import DeviceIndex, bucket_topk_f64, global_band, merge_topk

pytestmark = pytest.mark.gpu
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
PH3 = _lib.LMI_Q_PHASE_PLAN | _lib.LMI_Q_PHASE_SCAN | _lib.LMI_Q_PHASE_MERGE


def _stripes_global(w, x, q, cls, G, k, seed, chunk=256):
    """The G stripes' lists through the global band, merged by K3; and the
    refined entries per stripe (rows of the merged band it refined)."""
    ixs = [DeviceIndex(x, w["labels"], w["C"], chunk_rows=chunk, device="cuda", rank=g, world=G)
           for g in range(G)]
    nq, R = cls.shape
    P = nq * R
    assert all(global_band(ix, nq, R, k, _lib.LMI_Q_F16) for ix in ixs)
    outs, kths = [], []
    for ix in ixs:
        d = torch.empty((nq, R, k), dtype=torch.float64, device="cuda")
        p = torch.empty((nq, R, k), dtype=torch.int32, device="cuda")
        st = torch.zeros((1,), dtype=torch.int32, device="cuda")
        kth = torch.empty((P * k,), dtype=torch.float32, device="cuda")
        bucket_topk_f64(ix, q, cls, k, qmode=_lib.LMI_Q_F16, out=(d, p, st), seed_round0=seed,
                        phases=PH3, band_x=(kth, None, G))
        outs.append((d, p, st))
        kths.append(kth)
    kall = torch.stack(kths)
    for ix, (d, p, st) in zip(ixs, outs):
        bucket_topk_f64(ix, q, cls, k, qmode=_lib.LMI_Q_F16, out=(d, p, st), seed_round0=seed,
                        phases=_lib.LMI_Q_PHASE_REFINE, band_x=(None, kall, G))
        assert int(st.item()) == 0
    md, mp = merge_topk(torch.stack([o[0] for o in outs]), torch.stack([o[1] for o in outs]), k)
    refined = sum(int((o[1] >= 0).sum()) for o in outs)
    return md, mp, refined, outs


@pytest.mark.parametrize("mode,seed_", [("near", 701), ("dup", 702), ("skewed", 703)])
@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("seeded", [False, True])
def test_global_band_stripes_equal_one_gpu(mode, seed_, G, seeded):
    w = workloads.clustered(n=6000, nq=160, C=16, seed=seed_, label_mode=mode)
    R, k = 4, 10
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    cls = T(classes.astype(np.int32))
    q = T(w["q"])
    one = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256, device="cuda")
    d0, p0, st0 = bucket_topk_f64(one, q, cls, k, qmode=_lib.LMI_Q_F16, seed_round0=seeded)
    assert int(st0.item()) == 0
    md, mp, refined, _ = _stripes_global(w, w["x"], q, cls, G, k, seeded)
    assert torch.equal(md, d0) and torch.equal(mp, p0)
    # the round-5 form (each stripe refines the band of its own list) gives
    # the same lists
    parts = [bucket_topk_f64(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256, device="cuda",
                                         rank=g, world=G), q, cls, k, qmode=_lib.LMI_Q_F16,
                             seed_round0=seeded) for g in range(G)]
    ld, lp = merge_topk(torch.stack([x[0] for x in parts]), torch.stack([x[1] for x in parts]), k)
    assert torch.equal(ld, md) and torch.equal(lp, mp)
    if not seeded:
        # the oracle's float64 lists (sklearn's arithmetic) within the comparator
        rd, rp = O.bucket_lists(w["labels"], w["x"].astype(np.float16), w["q"].astype(np.float16),
                                classes, R, k, w["C"])
        assert O.compare_lists(rd, rp, md.cpu().numpy().reshape(rd.shape),
                               mp.cpu().numpy().reshape(rp.shape), atol=1e-12, tie=1e-12) == 0


def test_global_band_refines_fewer_rows_than_the_local_band():
    """The point of the global band: a stripe's refined entries are its rows
    of the MERGED band, about 1/G of the band's rows, where the per-rank form
    refines a band of about k + its width per stripe."""
    w = workloads.clustered(n=20000, nq=200, C=8, seed=711, label_mode="router")
    R, k, G = 2, 10, 8
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    cls = T(classes.astype(np.int32))
    _, _, refined, outs = _stripes_global(w, w["x"], T(w["q"]), cls, G, k, False)
    P = classes.size
    # every pair keeps k entries after the merge; the stripes together hold
    # the merged band's rows, not G bands of >= k rows
    assert refined < 2 * k * P, (refined, P)


def test_one_call_of_every_phase_is_the_plain_float64_scan():
    """No phase flag: PLAN, SCAN, MERGE and REFINE on one rank (kth_all ==
    kth_send, G = 1) = lmi_bucket_topk_f64q."""
    w = workloads.clustered(n=6000, nq=120, C=16, seed=721, label_mode="near")
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :4]
    cls = T(classes.astype(np.int32))
    ix = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256, device="cuda")
    q = T(w["q"])
    d0, p0, _ = bucket_topk_f64(ix, q, cls, 10, qmode=_lib.LMI_Q_F16)
    kth = torch.empty((classes.size * 10,), dtype=torch.float32, device="cuda")
    d1, p1, st = bucket_topk_f64(ix, q, cls, 10, qmode=_lib.LMI_Q_F16, band_x=(kth, kth, 1))
    assert int(st.item()) == 0 and torch.equal(d0, d1) and torch.equal(p0, p1)
    with pytest.raises(_lib.LmiError):   # all phases at G > 1: the exchange is missing
        bucket_topk_f64(ix, q, cls, 10, qmode=_lib.LMI_Q_F16, band_x=(kth, kth, 2))


def test_global_band_with_float64_inputs():
    """float64 rows and queries below half a float32 ulp (corpus64 / q64):
    the striped global band equals one GPU."""
    w = workloads.clustered(n=6000, nq=120, C=16, seed=731, label_mode="skewed")
    x64, q64 = workloads.float64_inputs(w, 731)
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :4]
    cls = T(classes.astype(np.int32))
    one = DeviceIndex(x64, w["labels"], w["C"], chunk_rows=256, device="cuda")
    assert one.corpus64 is not None
    d0, p0, _ = bucket_topk_f64(one, T(q64), cls, 10)
    md, mp, _, _ = _stripes_global(w, x64, T(q64), cls, 3, 10, False)
    assert torch.equal(md, d0) and torch.equal(mp, p0)


def test_global_band_not_offered_without_band_lists():
    w = workloads.clustered(n=3000, nq=40, C=8, seed=741)
    ix = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256, device="cuda")
    assert global_band(ix, 40, 4, 10, _lib.LMI_Q_F16)
    assert not global_band(ix, 40, 4, 12, _lib.LMI_Q_F16)   # k > 10: 15-entry lane lists
    assert not global_band(ix, 40, 4, 10, _lib.LMI_Q_F32)   # the general fp32 scan


@pytest.mark.parametrize("n,G", [(6000, 3), (6, 8)])
def test_kth_blocks_cover_every_pair(n, G):
    """The MERGE phase writes each pair's k smallest d32 beside its band list
    (chunk_merge_band_kernel): every entry of the kth block is written -- +inf
    for pairs whose class is out of range (no grouped position) and for a
    stripe with no rows at all (n = 6 over 8 stripes) -- and the stripes still
    merge to the one-GPU float64 lists."""
    w = workloads.clustered(n=n, nq=40, C=4 if n < 100 else 16, seed=705,
                            label_mode="router" if n < 100 else "near")
    w["x"] = w["x"].astype(np.float16).astype(np.float32)  # (fp16-exact: the band lists' scan)
    R, k = 4, 10
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R].astype(np.int32)
    classes[0, :] = -1
    classes[1, 2] = w["C"]
    cls = T(classes)
    q = T(w["q"])
    nq = classes.shape[0]
    P = nq * R
    one = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256, device="cuda")
    d0, p0, st0 = bucket_topk_f64(one, q, cls, k, qmode=_lib.LMI_Q_F16)
    for g in range(G):
        ix = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256, device="cuda", rank=g, world=G)
        kth = torch.full((P * k,), float("nan"), dtype=torch.float32, device="cuda")
        d = torch.empty((nq, R, k), dtype=torch.float64, device="cuda")
        p = torch.empty((nq, R, k), dtype=torch.int32, device="cuda")
        st = torch.zeros((1,), dtype=torch.int32, device="cuda")
        bucket_topk_f64(ix, q, cls, k, qmode=_lib.LMI_Q_F16, out=(d, p, st), phases=PH3,
                        band_x=(kth, None, G))
        kb = kth.view(nq, R, k).cpu().numpy()
        assert not np.isnan(kb).any()
        assert np.isinf(kb[0]).all() and np.isinf(kb[1, 2]).all()
        assert (np.diff(kb, axis=2)[np.isfinite(kb[..., 1:])] >= 0).all()
    md, mp, _, _ = _stripes_global(w, w["x"], q, cls, G, k, False)
    assert torch.equal(md, d0) and torch.equal(mp, p0)
