"""GPU parity: K1 router, K2 bucket scan, K3 merge and the full search against
the CPU oracle (oracle/lmi_oracle.py), through the C-ABI (liblmi_hip.so)."""
import numpy as np
import pytest
import torch

import lmi_oracle as O
import workloads
from li import _lib
from li.index import DeviceIndex, DeviceRouter, Searcher, bucket_topk, merge_topk

pytestmark = pytest.mark.gpu


def _router_mismatch(classes_gpu, logits, R, gap=1e-5):
    """Rows whose top-R differs from the oracle and is not explained by a
    near-tie of logits at the cut."""
    ref = O.rank_classes(logits)[:, :R]
    bad = 0
    for i in np.nonzero((classes_gpu != ref).any(axis=1))[0]:
        srt = np.sort(logits[i])[::-1]
        if np.min(np.abs(np.diff(srt[: R + 1]))) > gap:
            bad += 1
    return bad


@pytest.mark.parametrize("arch", ["MLP", "MLP-5"])
def test_router_topr_and_argmax(arch):
    w = workloads.clustered(n=4000, nq=700, C=122, arch=arch, seed=11)
    r = DeviceRouter(w["layers"])
    logits = O.mlp_forward(w["qn"], w["layers"])
    for R in (1, 4, 7, 122):
        cls, probs = r.topr(torch.from_numpy(w["qn"]).cuda(), R, with_probs=True)
        cls = cls.cpu().numpy()
        assert _router_mismatch(cls, logits, R) == 0
        ref_p = np.take_along_axis(O.softmax(logits), cls.astype(np.int64), axis=1)
        np.testing.assert_allclose(probs.cpu().numpy(), ref_p, rtol=1e-5, atol=1e-7)
    am = r.argmax(torch.from_numpy(w["xn"]).cuda()).cpu().numpy()
    assert (am != O.predict(w["xn"], w["layers"])).sum() <= 1


@pytest.mark.parametrize("label_mode", ["router", "skewed"])
@pytest.mark.parametrize("storage", ["f16", "f32"])
@pytest.mark.parametrize("k", [10, 3, 16])
def test_bucket_topk_matches_oracle(label_mode, storage, k):
    w = workloads.clustered(n=6000, nq=257, C=16, seed=5, label_mode=label_mode)
    R = 4
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    ix = DeviceIndex(w["x"], w["labels"], w["C"], storage=storage, chunk_rows=512)
    d, pos, st = bucket_topk(ix, torch.from_numpy(w["q"]).cuda(),
                             torch.from_numpy(classes.astype(np.int32)).cuda(), k)
    assert int(st.item()) == 0
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, k, w["C"])
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), pos.cpu().numpy()) == 0


def test_bucket_topk_nonf16_queries_fall_back_exactly():
    w = workloads.clustered(n=3000, nq=64, C=8, seed=9, label_mode="skewed")
    q = w["q"] + np.float32(1e-4)  # no longer fp16-representable
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :2]
    ix = DeviceIndex(w["x"], w["labels"], w["C"], storage="f16", chunk_rows=256)
    qt = torch.from_numpy(q).cuda()
    ct = torch.from_numpy(classes.astype(np.int32)).cuda()
    _, _, st = bucket_topk(ix, qt, ct, 10)
    assert int(st.item()) & _lib.LMI_STATUS_QUERY_NOT_F16
    d, pos, _ = bucket_topk(ix, qt, ct, 10, qmode=_lib.LMI_Q_F32)
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"], q, classes, 2, 10, w["C"])
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), pos.cpu().numpy()) == 0


def test_shard_merge_equals_single_gpu():
    """Striping + K3 merge gives bitwise the single-shard lists (any G)."""
    w = workloads.clustered(n=5000, nq=150, C=16, seed=3, label_mode="skewed")
    R, k = 3, 10
    classes = torch.from_numpy(
        O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R].astype(np.int32)).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    full = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256)
    d1, p1, _ = bucket_topk(full, q, classes, k)
    for G in (2, 3, 8):
        parts = [bucket_topk(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256, rank=g, world=G),
                             q, classes, k)[:2] for g in range(G)]
        dm, pm = merge_topk(torch.stack([p[0] for p in parts]), torch.stack([p[1] for p in parts]), k)
        assert torch.equal(dm, d1) and torch.equal(pm, p1)


@pytest.mark.parametrize("f64,k", [(False, 10), (False, 16), (True, 10), (False, 40),
                                   (True, 30)])
def test_packed_merge_equals_single_gpu(f64, k):
    """The G > 1 product path: every shard's K2 writes its lists and status word
    into its packed send buffer (li.dist.packed_lists), the buffers are
    gathered (here by concatenation, as all_gather_into_tensor lays them out)
    and K3 merges them in place (lmi_merge_topk_packed): bitwise the
    single-shard lists, and the OR of the ranks' status words.  k > 16: the
    lower-bound passes' wide lists and K3's merge by rank."""
    from li import _lib
    from li.dist import packed_lists
    from li.index import bucket_topk_f64, check, ptr
    w = workloads.clustered(n=5000, nq=150, C=16, seed=3, label_mode="skewed")
    R = 3
    classes = torch.from_numpy(
        O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R].astype(np.int32)).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    scan = bucket_topk_f64 if f64 else bucket_topk
    d1, p1, _ = scan(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256), q, classes, k)
    nq = q.shape[0]
    rows = nq * R
    lib = _lib.load()
    for G in (2, 3, 8):
        bufs = []
        for g in range(G):
            buf, dv, pv, sv = packed_lists(rows, k, f64, q.device)
            ix = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=256, rank=g, world=G)
            scan(ix, q, classes, k, out=(dv.view(nq, R, k), pv.view(nq, R, k), sv))
            if g == 1:
                sv.fill_(4)  # a status bit on one rank reaches every rank's result
            bufs.append(buf)
        W = bufs[0].numel()
        gathered = torch.cat(bufs)
        md = torch.empty((rows, k), dtype=torch.float64 if f64 else torch.float32, device=q.device)
        mp = torch.empty((rows, k), dtype=torch.int32, device=q.device)
        st = torch.full((1,), -1, dtype=torch.int32, device=q.device)
        check("lmi_merge_topk_packed", lib.lmi_merge_topk_packed(
            ptr(gathered), G, W, rows, k, int(f64), ptr(md), ptr(mp), ptr(st), _lib.stream_handle(q.device)))
        assert torch.equal(md.view(nq, R, k), d1) and torch.equal(mp.view(nq, R, k), p1)
        assert int(st.item()) == 4


@pytest.mark.parametrize("use_threshold", [True, False])
@pytest.mark.parametrize("R", [1, 4])
def test_full_search_matches_direct_oracle(use_threshold, R):
    w = workloads.clustered(n=6000, nq=300, C=16, seed=21, label_mode="skewed")
    ids = np.arange(1, w["x"].shape[0] + 1)
    router = DeviceRouter(w["layers"])
    ix = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=1024)
    s = Searcher(ix, router)
    dists, anns = s.search(torch.from_numpy(w["qn"]).cuda(), torch.from_numpy(w["q"]).cuda(), R,
                           k=10, use_threshold=use_threshold)
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))
    ref_d, ref_a = O.search_direct(w["labels"], ids, w["x"], w["q"], classes, n_buckets=R, k=10,
                                   use_threshold=use_threshold)
    assert dists.shape == ref_d.shape and anns.dtype == np.uint32
    assert O.compare_lists(ref_d, ref_a, dists, anns) == 0


@pytest.mark.parametrize("label_mode", ["router", "dup"])
def test_scan_tiles_of_many_pairs_match_oracle_and_4wave_ring(label_mode, monkeypatch):
    """Buckets probed by > 256 pairs (several 8-wave tiles per chunk), exact
    duplicate vectors (tied distances): the 8-wave scan equals the oracle and,
    bitwise, the 4-wave ring (same MFMA accumulation order)."""
    w = workloads.clustered(n=20000, nq=1500, C=8, seed=13, label_mode=label_mode)
    R, k = 2, 10
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    ix = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=2048)
    q = torch.from_numpy(w["q"]).cuda()
    ct = torch.from_numpy(classes.astype(np.int32)).cuda()
    d3, p3, st = bucket_topk(ix, q, ct, k)
    assert int(st.item()) == 0
    monkeypatch.setenv("LMI_SCAN_V2", "1")
    d2, p2, _ = bucket_topk(ix, q, ct, k)
    assert torch.equal(d3, d2) and torch.equal(p3, p2)
    ref_d, ref_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, k, w["C"])
    assert O.compare_lists(ref_d, ref_p, d3.cpu().numpy(), p3.cpu().numpy()) == 0


@pytest.mark.parametrize("hidden", [(128,), (256, 128), (100,)])
def test_router_mfma_matches_fma_path(hidden, monkeypatch):
    """K1's MFMA form (widths multiples of 16) and its FMA-chain form
    (LMI_ROUTER_FMA=1, and the automatic fallback for other widths) agree with
    the oracle and with each other up to near-ties of the logits."""
    rng = np.random.default_rng(5)
    dims = (96,) + hidden + (122,)
    layers = [(rng.standard_normal((o, i)).astype(np.float32) / np.sqrt(i),
               rng.standard_normal(o).astype(np.float32) * 0.1) for i, o in zip(dims, dims[1:])]
    x = rng.standard_normal((1000, 96)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    logits = O.mlp_forward(x, layers)
    r = DeviceRouter(layers)
    xt = torch.from_numpy(x).cuda()
    cls_m, p_m = r.topr(xt, 7, with_probs=True)
    monkeypatch.setenv("LMI_ROUTER_FMA", "1")
    cls_f, p_f = r.topr(xt, 7, with_probs=True)
    am_f = r.argmax(xt).cpu().numpy()
    monkeypatch.delenv("LMI_ROUTER_FMA")
    am_m = r.argmax(xt).cpu().numpy()
    for cls in (cls_m.cpu().numpy(), cls_f.cpu().numpy()):
        assert _router_mismatch(cls, logits, 7) == 0
    np.testing.assert_allclose(p_m.cpu().numpy(), p_f.cpu().numpy(), rtol=1e-5, atol=1e-7)
    assert (am_m != am_f).sum() <= 1


@pytest.mark.parametrize("world", [1, 2])
def test_row_source_index_equals_tensor_index(world):
    """configs[4]'s generated corpus (li.index.RowSource, chunks scattered into
    the shard) lays out exactly the index built from the whole tensor."""
    from li import synth
    from li.index import RowSource
    n, d, ch = 5000, 96, 1024
    fn = synth.random_rows_fn(d, 7, "cuda", chunk=ch)
    x = torch.cat([fn(a, min(n, a + ch)) for a in range(0, n, ch)])
    labels = torch.from_numpy(np.random.default_rng(3).integers(0, 9, n).astype(np.int32))
    for rank in range(world):
        a = DeviceIndex(x, labels, 9, chunk_rows=512, rank=rank, world=world, device="cuda")
        b = DeviceIndex(RowSource(n, d, fn, ch), labels, 9, chunk_rows=512, rank=rank, world=world,
                        device="cuda")
        assert a.storage == b.storage == "f16" and a.n_rows == b.n_rows
        assert torch.equal(a.corpus, b.corpus) and torch.equal(a.inv_norm, b.inv_norm)
        assert torch.equal(a.gpos, b.gpos) and torch.equal(a.chunk_first, b.chunk_first)


@pytest.mark.parametrize("label_mode,R,k", [("router", 4, 10), ("skewed", 3, 7), ("dup", 5, 16)])
def test_exact_semantics_matches_oracle(label_mode, R, k):
    """semantics="exact": exact top-k over the union of the R probed buckets."""
    w = workloads.clustered(n=4000, nq=150, C=16, seed=23, label_mode=label_mode)
    ids = np.arange(1, w["x"].shape[0] + 1)
    s = Searcher(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda"),
                 DeviceRouter(w["layers"], device="cuda"))
    d, a = s.search(torch.from_numpy(w["qn"]).cuda(), torch.from_numpy(w["q"]).cuda(), R, k=k,
                    semantics="exact")
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    rd, ra = O.search_exact(w["labels"], ids, w["x"], w["q"], classes, w["C"], R, k)
    assert d.shape == (150, k) and a.dtype == np.uint32
    assert O.compare_lists(rd, ra, d, a) == 0


def test_full_size_10m_properties():
    """BASELINE configs[2] at full size (10M x 768 fp16, 122 buckets, 10k
    queries, R = 4): K2's per-(query, probe) lists on a sample of queries equal
    an independent torch fp32 brute force over the same bucket rows, and the
    whole search output has the reference's shape invariants (ascending rows,
    ids in range, distances = recomputed 1 - cos of the returned ids)."""
    from li import synth
    dev = torch.device("cuda")
    x, q, qn, xn, layers = synth.build_lmi_workload(10_000_000, 10_000, 122, "MLP-5", dev)
    router = DeviceRouter(layers, device=dev)
    labels = router.argmax(xn)
    del xn
    ix = DeviceIndex(x, labels, 122, chunk_rows=8192, device=dev)
    classes, _ = router.topr(qn, 4)
    d, pos, st = bucket_topk(ix, q, classes, 10)
    assert int(st.item()) == 0
    d, pos = d.cpu().numpy(), pos.cpu().numpy()
    assert np.all(np.diff(d, axis=2) >= 0)
    off = ix.bucket_off_local.cpu().numpy()
    cls = classes.cpu().numpy()
    rng = np.random.default_rng(0)
    qs = rng.choice(10_000, 48, replace=False)
    qh = q[qs].float()
    qh = qh / qh.norm(dim=1, keepdim=True)
    for i, qi in enumerate(qs):
        for r in range(4):
            c = cls[qi, r]
            a, b = int(off[c]), int(off[c + 1])
            assert ((pos[qi, r] >= a) & (pos[qi, r] < b)).all()
            y = ix.corpus[a:b, :768].float() * ix.inv_norm[a:b, None]
            dd = (1.0 - y @ qh[i]).double().cpu().numpy()
            o = np.lexsort((np.arange(b - a), dd))[:10]
            np.testing.assert_allclose(d[qi, r], dd[o], atol=2e-6)
            assert O.compare_lists(dd[o][None], o[None] + a, d[qi, r][None], pos[qi, r][None]) == 0
    s = Searcher(ix, router)
    dists, anns = s.search(qn, q, 4, k=10)
    assert dists.shape == (10_000, 10) and anns.dtype == np.uint32
    assert np.all(np.diff(dists, axis=1) >= 0)
    assert anns.max() <= 10_000_000
    ids = torch.from_numpy(anns[qs].astype(np.int64) - 1).to(dev)
    y = x[ids.clamp(min=0)].float()
    y = y / y.norm(dim=2, keepdim=True)
    dd = (1.0 - (y * qh[:, None, :]).sum(2)).double().cpu().numpy()
    live = anns[qs] > 0
    np.testing.assert_allclose(dists[qs][live], dd[live], atol=1e-5)


@pytest.mark.parametrize("dist,k", [("f32", 30), ("f64", 24)])
def test_exact_semantics_wide_k_matches_oracle(dist, k):
    """semantics='exact' with k > 16: the R wide lists of a query merged by
    K3's rank merge = the exact top-k of the union of its probed buckets."""
    w = workloads.clustered(n=6000, nq=200, C=16, seed=83, label_mode="skewed")
    R = 4
    s = Searcher(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512), DeviceRouter(w["layers"]))
    d, a = s.search(torch.from_numpy(w["qn"]).cuda(), torch.from_numpy(w["q"]).cuda(), R, k=k,
                    k_round=10, semantics="exact", dist=dist)
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    x = w["x"] if dist == "f32" else w["x"].astype(np.float16)
    q = w["q"] if dist == "f32" else w["q"].astype(np.float16)
    order, off = O.layout(w["labels"], w["C"])
    ids = np.arange(1, w["x"].shape[0] + 1)
    ref_d = np.full((200, k), 10000.0)
    ref_a = np.zeros((200, k), np.int64)
    for i in range(200):
        pos = np.concatenate([np.arange(off[c], off[c + 1]) for c in classes[i]])
        D = O.pairwise_cosine(q[i:i + 1], x[order[pos]])[0]
        o = np.lexsort((pos, D))[:k]
        ref_d[i, :o.size] = D[o]
        ref_a[i, :o.size] = ids[order[pos[o]]]
    tie, atol = (1e-6, 1e-5) if dist == "f32" else (1e-12, 1e-12)
    assert O.compare_lists(ref_d, ref_a, d, a, atol=atol, tie=tie) == 0
