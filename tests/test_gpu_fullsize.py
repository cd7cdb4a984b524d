"""BASELINE configs[1] and configs[2] at full size, against the pinned checkers.

configs[1]: 300K clip768-like rows, 122 buckets, 10k queries, R = 7 (one GPU):
    the whole search equals the oracle's per-(query, probe) lists + its replay
    (oracle.bucket_lists + oracle.replay, pinned to the reference by
    test_oracle_golden*.py) — float32 inputs (the reference's float32 branch,
    float32 tie window) and float16 inputs (float64 branch, 1e-12).
configs[2]: 10M rows, R = 4: the device replay equals the host replay
    (lmi_replay, pinned by test_oracle_golden.py) bit for bit on the full
    10k x 4 lists, in both arithmetics; K2's lists for 512 sampled queries equal
    oracle.bucket_lists over the same bucket rows (float32 and float64)."""
import numpy as np
import pytest
import torch

import lmi_oracle as O
from li import synth
from li.index import DeviceIndex, DeviceRouter, Searcher, bucket_topk, bucket_topk_f64

pytestmark = pytest.mark.gpu
TIE32, TIE64 = 1e-6, 1e-12


def _workload(n, nq=10_000):
    dev = torch.device("cuda")
    x, q, qn, xn, layers = synth.build_lmi_workload(n, nq, 122, "MLP-5", dev)
    router = DeviceRouter(layers, device=dev)
    labels = router.argmax(xn)
    del xn
    ix = DeviceIndex(x, labels, 122, chunk_rows=8192, device=dev)
    return dict(x=x, q=q, qn=qn, router=router, labels=labels, ix=ix, s=Searcher(ix, router))


@pytest.fixture(scope="module")
def w300k():
    return _workload(300_000)


@pytest.fixture(scope="module")
def w10m():
    w = _workload(10_000_000)
    yield w
    w.clear()
    torch.cuda.empty_cache()


def _oracle_search(w, R, dt):
    """oracle.bucket_lists + oracle.replay on the host copy of the workload."""
    ix = w["ix"]
    x = w["x"].cpu().numpy()                       # fp16 rows in input order
    q = w["q"].cpu().numpy()                       # fp16-exact float32
    if dt == "f32":
        x, q = x.astype(np.float32), q.astype(np.float32)
    else:
        q = q.astype(np.float16)
    labels = w["labels"].cpu().numpy().astype(np.int64)
    classes = w["router"].topr(w["qn"], R)[0].cpu().numpy().astype(np.int64)
    d, p = O.bucket_lists(labels, x, q, classes, R, 10, 122)
    order, off = O.layout(labels, 122)
    return O.replay(classes, d, p, k_round=10, k_final=10, bucket_size=np.diff(off),
                    pos_to_id=np.arange(1, x.shape[0] + 1)[order], use_threshold=True)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("dist", ["f32", "f64"])
def test_configs1_300k_r7_search_equals_oracle(w300k, dist):
    w = w300k
    dists, anns = w["s"].search(w["qn"], w["q"], 7, k=10, dist=dist)
    rd, ra = _oracle_search(w, 7, dist)
    assert dists.shape == (10_000, 10)
    tie, atol = (TIE32, 1e-5) if dist == "f32" else (TIE64, 1e-12)
    assert O.compare_lists(rd, ra, dists, anns, atol=atol, tie=tie) == 0


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dist", ["f32", "f64"])
def test_configs2_10m_device_replay_equals_host_replay(w10m, dist):
    w = w10m
    dd, da = w["s"].search(w["qn"], w["q"], 4, k=10, dist=dist, replay_on="device")
    hd, ha = w["s"].search(w["qn"], w["q"], 4, k=10, dist=dist, replay_on="host")
    np.testing.assert_array_equal(dd, hd)
    np.testing.assert_array_equal(da, ha)
    assert np.all(np.diff(dd, axis=1) >= 0) and da.max() <= 10_000_000


@pytest.mark.timeout(600)
@pytest.mark.parametrize("dist", ["f32", "f64"])
def test_configs2_10m_lists_match_oracle(w10m, dist):
    """512 sampled queries: every probed bucket's rows (this index's layout)
    through oracle.bucket_lists, in the reference's arithmetic for the dtype."""
    w = w10m
    ix = w["ix"]
    R, k = 4, 10
    classes = w["router"].topr(w["qn"], R)[0]
    if dist == "f32":
        d, pos, st = bucket_topk(ix, w["q"], classes, k)
    else:
        d, pos, st = bucket_topk_f64(ix, w["q"], classes, k)
    assert int(st.item()) == 0
    d, pos, cls = d.cpu().numpy(), pos.cpu().numpy(), classes.cpu().numpy()
    qs = np.sort(np.random.default_rng(5).choice(10_000, 512, replace=False))
    qh = w["q"].cpu().numpy()[qs]
    qh = qh.astype(np.float32) if dist == "f32" else qh.astype(np.float16)
    off = ix.bucket_off_local.cpu().numpy()
    ref_d = np.full((qs.size, R, k), np.inf)
    ref_p = np.full((qs.size, R, k), -1, np.int64)
    for c in np.unique(cls[qs]):
        a, b = int(off[c]), int(off[c + 1])
        rows = ix.corpus[a:b, : ix.d].cpu().numpy()   # bucket c in global-position order
        rows = rows.astype(np.float32) if dist == "f32" else rows
        sel = np.nonzero((cls[qs] == c).any(axis=1))[0]
        sub_cls = np.where(cls[qs][sel] == c, 0, -1)
        sd, sp = O.bucket_lists(np.zeros(b - a, np.int64), rows, qh[sel], sub_cls, R, k, 1)
        hit = sub_cls == 0
        ref_d[sel[:, None].repeat(R, 1)[hit], np.nonzero(hit)[1]] = sd[hit]
        ref_p[sel[:, None].repeat(R, 1)[hit], np.nonzero(hit)[1]] = sp[hit] + a
    tie, atol = (TIE32, 1e-5) if dist == "f32" else (TIE64, 1e-12)
    assert O.compare_lists(ref_d, ref_p, d[qs], pos[qs], atol=atol, tie=tie) == 0


def _packed_shards(x, labels, q, classes, k, f64, G, chunk_rows, C=122):
    """The G > 1 product path run one shard at a time on this GPU: rank g's
    DeviceIndex (slice g of every bucket), K2 into its packed send buffer
    (li.dist.packed_lists), the buffers concatenated as all_gather_into_tensor
    leaves them, K3 in place (lmi_merge_topk_packed) -> merged lists + status."""
    from li import _lib
    from li.dist import packed_lists
    from li.index import check, ptr
    nq, R = classes.shape
    rows = nq * R
    scan = bucket_topk_f64 if f64 else bucket_topk
    bufs = []
    for g in range(G):
        ix = DeviceIndex(x, labels, C, chunk_rows=chunk_rows, rank=g, world=G)
        buf, dv, pv, sv = packed_lists(rows, k, f64, q.device)
        scan(ix, q, classes, k, out=(dv.view(nq, R, k), pv.view(nq, R, k), sv))
        torch.cuda.synchronize()
        bufs.append(buf)
        del ix
        torch.cuda.empty_cache()
    gathered = torch.cat(bufs)
    del bufs
    md = torch.empty((rows, k), dtype=torch.float64 if f64 else torch.float32, device=q.device)
    mp = torch.empty((rows, k), dtype=torch.int32, device=q.device)
    st = torch.full((1,), -1, dtype=torch.int32, device=q.device)
    check("lmi_merge_topk_packed", _lib.load().lmi_merge_topk_packed(
        ptr(gathered), G, gathered.numel() // G, rows, k, int(f64), ptr(md), ptr(mp), ptr(st),
        _lib.stream_handle(q.device)))
    return md.view(nq, R, k), mp.view(nq, R, k), int(st.item())


@pytest.mark.timeout(600)
@pytest.mark.parametrize("dist", ["f32", "f64"])
def test_configs3_eight_shards_equal_one_gpu(w10m, dist):
    """BASELINE configs[3] (10M, 8 GPUs) exercised on one GPU: the eight
    stripes built one at a time with the 8-GPU chunk size (2048 rows), each
    scanned into its packed all-gather buffer, merged by K3 -> bitwise the
    single-GPU lists; the device replay over them -> bitwise the single-GPU
    answer."""
    from li.index import replay_device
    w = w10m
    ix, s = w["ix"], w["s"]
    R, k = 4, 10
    classes = w["router"].topr(w["qn"], R)[0]
    f64 = dist == "f64"
    scan = bucket_topk_f64 if f64 else bucket_topk
    d1, p1, st1 = scan(ix, w["q"], classes, k)
    assert int(st1.item()) == 0
    md, mp, st = _packed_shards(w["x"], w["labels"], w["q"], classes, k, f64, 8, 2048)
    assert st == 0
    assert torch.equal(md, d1) and torch.equal(mp, p1)
    bsz, p2id = s._device_tables()
    a1 = replay_device(classes, d1, p1, k_round=10, k_final=k, bucket_size=bsz, pos_to_id=p2id,
                       use_threshold=True)
    a8 = replay_device(classes, md, mp, k_round=10, k_final=k, bucket_size=bsz, pos_to_id=p2id,
                       use_threshold=True)
    assert int(a1[2].item()) == 0 and int(a8[2].item()) == 0
    assert torch.equal(a1[0], a8[0]) and torch.equal(a1[1], a8[1])
