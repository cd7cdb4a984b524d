"""GPU drop-in vs the reference's own float64 outputs on float16 inputs
(tests/golden/reference_outputs_r2.npz): the real clip768 'emb' is float16 and
the reference then computes, thresholds and merges float64 distances
(utils.py:11, :19, :23; LearnedIndex.py:86-97).  The drop-in detects that from
the dtypes (li.LearnedIndex.dist_dtype) and runs lmi_bucket_topk_f64 + the
float64 replay.  Ids must match up to float64 ties (1e-12) and distances to
1e-12, on workloads full of near-duplicates 1e-9..1e-6 apart."""
import numpy as np
import pandas as pd
import pytest
import torch

import lmi_oracle as O
import workloads
from test_oracle_golden_r2 import BASES, CASES, G2, SINGLES, TIE64, base_inputs, check, inputs_r2

pytestmark = pytest.mark.gpu


def _nn(layers, arch, C):
    from li.model import NeuralNetwork
    nn = NeuralNetwork(input_dim=96, output_dim=C, lr=0.009, model_type=arch)
    lin = [m for m in nn.model.layers if isinstance(m, torch.nn.Linear)]
    with torch.no_grad():
        for m, (w, b) in zip(lin, layers):
            m.weight.copy_(torch.from_numpy(w))
            m.bias.copy_(torch.from_numpy(b))
    return nn


def _frames(w, f16=True):
    data = pd.DataFrame(w["xn"])
    data.index += 1
    x = w["x"].astype(np.float16) if f16 else w["x"]
    data_search = pd.DataFrame(x)
    data_search.index += 1
    return data, data_search, (w["q"].astype(np.float16) if f16 else w["q"])


@pytest.mark.parametrize("name", list(CASES))
def test_f16_search_matches_reference_float64(name):
    from li.LearnedIndex import LearnedIndex, dist_dtype
    from li.model import data_X_to_torch
    _, n, nq, C, R, k, mode, arch, seed, thr = CASES[name]
    w = inputs_r2(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    _, classes = li.model.predict_proba(data_X_to_torch(w["qn"]))
    assert (classes[:, :R] == G2[f"search_{name}__classes"][:, :R]).all()
    data, data_search, q = _frames(w)
    assert dist_dtype(data_search, q) == "f64"
    dists, anns = li.search(data, w["qn"], data_search, q, w["labels"], n_buckets=R, k=k,
                            use_threshold=thr)
    assert dists.dtype == np.float64 and anns.dtype == np.uint32
    check(name, dists, anns)


@pytest.mark.parametrize("name", list(SINGLES))
def test_search_single_r2_matches_reference(name):
    """search_single on float16 (float64 arithmetic) and float32 inputs, k up to
    100 (the R == 1 CLI path passes k: search.py:134-140)."""
    from li.LearnedIndex import LearnedIndex
    _, n, nq, C, R, k, mode, arch, seed, thr, dt = SINGLES[name]
    w = inputs_r2(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    data, data_search, q = _frames(w, dt == "f16")
    data["category"] = w["labels"]
    classes = G2[f"search_{name}__classes"].astype(np.int64)
    thr_arr = G2[f"search_{name}__thr"] if thr else None
    dists, anns = li.search_single(data, data_search, q, classes[:, 0], k=k, threshold_dist=thr_arr)
    assert dists.shape == (nq, k)
    if dt == "f16":
        check(name, dists, anns)
    else:
        check(name, dists, anns, tie=1e-6, atol=1e-5)


@pytest.mark.parametrize("name", list(BASES))
def test_baseline_r2_matches_reference(name):
    from li.Baseline import Baseline
    _, n, nq, k, mode, seed, dt = BASES[name]
    w = base_inputs(name)
    x = w["x"].astype(np.float16) if dt == "f16" else w["x"]
    q = w["q"].astype(np.float16) if dt == "f16" else w["q"]
    dists, nns, _ = Baseline().search(q, x, k=k)
    ref_d, ref_n = G2[f"base_{name}__dists"], G2[f"base_{name}__nns"]
    assert dists.dtype == ref_d.dtype and dists.shape == ref_d.shape
    tie, atol = (TIE64, 1e-12) if dt == "f16" else (1e-6, 1e-5)
    assert O.compare_lists(ref_d, ref_n, dists, nns, atol=atol, tie=tie) == 0


def _index_and_classes(w, C, R, world=1, rank=0):
    from li.index import DeviceIndex
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    ix = DeviceIndex(w["x"].astype(np.float16), w["labels"], C, device="cuda", chunk_rows=256,
                     rank=rank, world=world)
    return ix, torch.from_numpy(np.ascontiguousarray(classes, dtype=np.int32)).cuda(), classes


@pytest.mark.parametrize("seed,mode,R", [(401, "near", 4), (402, "dup", 3), (403, "skewed", 7)])
def test_f64_lists_match_oracle(seed, mode, R):
    """K2 in float64 equals the oracle's float64 per-(query, probe) lists."""
    from li.index import bucket_topk_f64
    w = workloads.clustered(n=4000, nq=160, C=16, seed=seed, label_mode=mode)
    ix, cls, classes = _index_and_classes(w, 16, R)
    q = torch.from_numpy(w["q"]).cuda()
    d, pos, st, nfb = bucket_topk_f64(ix, q, cls, 10, fallback_count=True)
    assert int(st.item()) == 0 and d.dtype == torch.float64
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"].astype(np.float16), w["q"].astype(np.float16),
                                  classes, R, 10, 16)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), pos.cpu().numpy(), atol=1e-12,
                           tie=TIE64) == 0
    assert nfb <= 2  # the whole-bucket path is for long runs of ties only


@pytest.mark.parametrize("nq", [96, 256])
def test_f64_fallback_path_is_exact(nq):
    """eps so large that every (query, probe) band overflows its list: every
    pair takes the whole-bucket float64 path, with the same results.  (The
    band lists hold 15 entries and a bound of the rows they drop: a pair falls
    back when its bucket has more than 15 rows, the 16th being in the band.)
    The first 512 failed pairs run in row slices over many workgroups, the
    rest (nq = 256: ~750 pairs) one workgroup each."""
    from li.index import bucket_topk_f64
    w = workloads.clustered(n=3000, nq=nq, C=8, seed=404, label_mode="near")
    ix, cls, classes = _index_and_classes(w, 8, 3)
    q = torch.from_numpy(w["q"]).cuda()
    d0, p0, _ = bucket_topk_f64(ix, q, cls, 10)
    d1, p1, st, nfb = bucket_topk_f64(ix, q, cls, 10, eps=0.75, fallback_count=True)
    assert int(st.item()) == 0
    assert nfb == int((ix.bucket_size[classes] >= 16).sum())
    assert torch.equal(p0, p1) and torch.equal(d0, d1)


@pytest.mark.parametrize("copies", [12, 40])
def test_f64_band_bound_sends_tied_runs_to_the_fallback(copies):
    """A run of `copies` identical rows (consecutive in their bucket) next to
    the queries: with 40 copies each scan lane fills its 10-entry list with
    them, so the bound of the rows the band lists drop lies in the float64
    band and those pairs take the whole-bucket path; with 12 the list holds
    the run.  Either way the lists equal the oracle's."""
    from li.index import bucket_topk_f64
    w = workloads.clustered(n=3000, nq=64, C=8, seed=407, label_mode="skewed")
    x = w["x"].astype(np.float16).copy()
    lab = w["labels"]
    big = int(np.bincount(lab, minlength=8).argmax())
    rows = np.nonzero(lab == big)[0]
    assert rows.size > copies + 50
    x[rows[20:20 + copies]] = x[rows[20]]
    q = w["q"].astype(np.float16).copy()
    q[:32] = x[rows[20]] + np.float16(0.01)
    w = dict(w, x=x.astype(np.float32), q=q.astype(np.float32))
    ix, _, _ = _index_and_classes(w, 8, 1)
    classes = np.full((q.shape[0], 1), big, np.int64)
    cls = torch.from_numpy(classes.astype(np.int32)).cuda()
    d, p, st, nfb = bucket_topk_f64(ix, torch.from_numpy(w["q"]).cuda(), cls, 10, fallback_count=True)
    assert int(st.item()) == 0
    ref_d, ref_p = O.bucket_lists(lab, x, q, classes, 1, 10, 8)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), p.cpu().numpy(), atol=1e-12, tie=TIE64) == 0
    if copies == 40:
        assert nfb >= 32


def test_f64_shard_merge_equals_single_gpu():
    """Per-shard float64 lists (G = 3 stripes) merged by K3 (lmi_merge_topk_f64)
    are bitwise the single-shard lists."""
    from li.index import bucket_topk_f64, merge_topk
    w = workloads.clustered(n=3000, nq=100, C=16, seed=405, label_mode="near")
    ix, cls, _ = _index_and_classes(w, 16, 4)
    q = torch.from_numpy(w["q"]).cuda()
    d, p, _ = bucket_topk_f64(ix, q, cls, 10)
    parts = []
    for g in range(3):
        ixg, _, _ = _index_and_classes(w, 16, 4, world=3, rank=g)
        parts.append(bucket_topk_f64(ixg, q, cls, 10)[:2])
    md, mp = merge_topk(torch.stack([a for a, _ in parts]), torch.stack([b for _, b in parts]), 10)
    assert torch.equal(mp, p) and torch.equal(md, d)


def test_f64_device_replay_equals_host_replay():
    from li.index import bucket_topk_f64, replay, replay_device
    w = workloads.clustered(n=3000, nq=200, C=16, seed=406, label_mode="near")
    ix, cls, classes = _index_and_classes(w, 16, 4)
    q = torch.from_numpy(w["q"]).cuda()
    d, p, _ = bucket_topk_f64(ix, q, cls, 10)
    kw = dict(k_round=10, k_final=10, use_threshold=True)
    hd, ha = replay(classes, d.cpu().numpy(), p.cpu().numpy(), bucket_size=ix.bucket_size,
                    pos_to_id=ix.pos_to_id, **kw)
    dd, da, st = replay_device(cls, d, p, bucket_size=torch.from_numpy(ix.bucket_size).cuda(),
                               pos_to_id=torch.from_numpy(ix.pos_to_id).cuda(), **kw)
    assert int(st.item()) == 0
    np.testing.assert_array_equal(dd.cpu().numpy(), hd)
    np.testing.assert_array_equal(da.cpu().numpy().view(np.uint32), ha)


def test_mutated_data_search_is_not_served_stale():
    """the HBM index cache is keyed on the bytes of data_search; a
    frame changed in place between two searches gives the new neighbours."""
    from li.LearnedIndex import LearnedIndex
    name = "f16_near_r4"
    _, n, nq, C, R, k, mode, arch, seed, thr = CASES[name]
    w = inputs_r2(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    data, data_search, q = _frames(w)
    d0, a0 = li.search(data, w["qn"], data_search, q, w["labels"], n_buckets=R, k=k,
                       use_threshold=thr)
    # move query 0's nearest neighbour far away, in place
    row = int(a0[0, 0])
    data_search.loc[row] = -data_search.loc[row]
    d1, a1 = li.search(data, w["qn"], data_search, q, w["labels"], n_buckets=R, k=k,
                       use_threshold=thr)
    assert row not in a1[0]
    x2 = w["x"].copy()
    x2[row - 1] = -x2[row - 1]
    classes = G2[f"search_{name}__classes"].astype(np.int64)
    rd, ra = O.search_direct(w["labels"], np.arange(1, n + 1), x2.astype(np.float16),
                             q, classes, n_buckets=R, k=k, use_threshold=thr)
    assert O.compare_lists(rd, ra, d1, a1, atol=1e-12, tie=TIE64) == 0


@pytest.mark.parametrize("k,mode", [(40, "skewed"), (100, "near"), (250, "dup")])
def test_large_k_lists_match_oracle(k, mode):
    """k > 16: the scan's lower-bound passes give the exact per-(query, probe)
    top-k (float32), and their first entries are bitwise one pass's."""
    from li.index import bucket_topk
    w = workloads.clustered(n=4000, nq=100, C=8, seed=420 + k, label_mode=mode)
    ix, cls, classes = _index_and_classes(w, 8, 2)
    q = torch.from_numpy(w["q"]).cuda()
    d, pos, st = bucket_topk(ix, q, cls, k)
    assert int(st.item()) == 0 and d.shape == (100, 2, k)
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, 2, k, 8)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), pos.cpu().numpy()) == 0
    d10, p10, _ = bucket_topk(ix, q, cls, 10)
    assert torch.equal(d[..., :10], d10) and torch.equal(pos[..., :10], p10)


@pytest.mark.parametrize("k", [20, 100, 240])
def test_large_k_f64_lists_match_oracle(k):
    from li.index import bucket_topk_f64
    w = workloads.clustered(n=4000, nq=80, C=8, seed=430 + k, label_mode="near")
    ix, cls, classes = _index_and_classes(w, 8, 2)
    q = torch.from_numpy(w["q"]).cuda()
    d, pos, st, nfb = bucket_topk_f64(ix, q, cls, k, fallback_count=True)
    assert int(st.item()) == 0 and d.shape == (80, 2, k) and d.dtype == torch.float64
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"].astype(np.float16), w["q"].astype(np.float16),
                                  classes, 2, k, 8)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), pos.cpu().numpy(), atol=1e-12,
                           tie=TIE64) == 0
