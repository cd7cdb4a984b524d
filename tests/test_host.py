"""CPU tests of the host side: the C-ABI library loads and exports every symbol
include/lmi_hip.h declares, argument validation, host helpers, bucket striping."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from li import _lib
from li.index import BucketLayout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "lmi_hip.h")).read()
    declared = set(re.findall(r"^\w[\w\s\*]*?\b(lmi_\w+)\(", hdr, flags=re.M))
    assert declared == set(_lib.EXPORTS)
    for name in declared:
        assert getattr(lib, name) is not None
    assert lib.lmi_abi_version() == _lib.ABI_VERSION == 13


def test_invalid_arguments_fail_loudly_without_a_device():
    lib = _lib.load()
    rc = lib.lmi_merge_topk(None, None, 0, 10, 10, None, None, None)
    assert rc == _lib.LMI_E_INVALID
    assert b"bad G" in lib.lmi_last_error()
    rc = lib.lmi_merge_topk(None, None, 2, 10, _lib.LMI_MAX_K_PASSES + 1, None, None, None)
    assert rc == _lib.LMI_E_INVALID and b"k=1025" in lib.lmi_last_error()
    rc = lib.lmi_merge_topk(None, None, 2, 10, 17, None, None, None)   # wide merge: k > 16 is valid
    assert rc == _lib.LMI_E_INVALID and b"null pointer" in lib.lmi_last_error()
    d = _lib.IndexDesc()
    rc = lib.lmi_bucket_topk(C.byref(d), None, 4, 768, None, 2, 10, 0, None, None, None, None, 0, None)
    assert rc == _lib.LMI_E_INVALID
    rc = lib.lmi_bucket_topk_f64(C.byref(d), None, 4, 768, None, 2, 241, 0, _lib.LMI_REFINE_EPS, None,
                                 None, None, None, 0, None)
    assert rc == _lib.LMI_E_INVALID and b"k=241" in lib.lmi_last_error()
    rc = lib.lmi_bucket_topk(C.byref(d), None, 4, 768, None, 2, 1025, 0, None, None, None, None, 0, None)
    assert rc == _lib.LMI_E_INVALID and b"k=1025" in lib.lmi_last_error()
    d.d = 2048
    rc = lib.lmi_bucket_topk_f64(C.byref(d), None, 4, 768, None, 2, 10, 0, _lib.LMI_REFINE_EPS, None,
                                 None, None, None, 0, None)
    assert rc == _lib.LMI_E_INVALID and b"d=2048" in lib.lmi_last_error()
    rc = lib.lmi_merge_topk_f64(None, None, 2, 10, 0, None, None, None)
    assert rc == _lib.LMI_E_INVALID and b"k=0" in lib.lmi_last_error()
    # packed K3: rank stride of 10 rows x k 10 = 201 words (f32) -> 202; 301 -> 302 (f64)
    assert lib.lmi_packed_rank_words(10, 10, 0) == 202
    assert lib.lmi_packed_rank_words(10, 10, 1) == 302
    rc = lib.lmi_merge_topk_packed(None, 2, 200, 10, 10, 0, None, None, None, None)
    assert rc == _lib.LMI_E_INVALID and b"rank_words" in lib.lmi_last_error()
    rc = lib.lmi_merge_topk_packed(None, 2, 203, 10, 10, 0, None, None, None, None)
    assert rc == _lib.LMI_E_INVALID and b"odd" in lib.lmi_last_error()
    rc = lib.lmi_merge_topk_packed(None, 2, 302, 10, 10, 1, None, None, None, None)
    assert rc == _lib.LMI_E_INVALID and b"null pointer" in lib.lmi_last_error()


def test_plan_chunks():
    lib = _lib.load()
    off = np.array([0, 0, 5, 70, 70, 200], np.int64)
    cf = np.zeros(6, np.int32)
    mx = lib.lmi_plan_chunks(off.ctypes.data, 5, 32, cf.ctypes.data)
    assert mx == 5  # bucket 4 has 130 rows -> 5 chunks of 32
    assert cf.tolist() == [0, 0, 1, 4, 4, 9]
    assert lib.lmi_plan_chunks(off.ctypes.data, 5, 33, cf.ctypes.data) < 0


def test_workspace_size_is_monotone():
    lib = _lib.load()
    d = _lib.IndexDesc()
    d.dtype, d.d, d.d_pad, d.n_rows, d.n_buckets = _lib.LMI_F16, 768, 768, 10**6, 122
    d.chunk_rows, d.n_chunks, d.max_chunks = 8192, 200, 5
    a = lib.lmi_scan_workspace_bytes(C.byref(d), 1000, 4, 10, _lib.LMI_Q_F16)
    b = lib.lmi_scan_workspace_bytes(C.byref(d), 10000, 4, 10, _lib.LMI_Q_F16)
    assert 0 < a < b


def test_wide_k_workspace_follows_the_switch(monkeypatch):
    """k > 16 on the fp16 scan sizes the bound + collect path (candidate slots,
    both scans' plans, the fix-up passes); LMI_WIDE_PASSES=1 the passes alone."""
    lib = _lib.load()
    d = _lib.IndexDesc()
    d.dtype, d.d, d.d_pad, d.n_rows, d.n_buckets = _lib.LMI_F16, 768, 768, 10**6, 122
    d.chunk_rows, d.n_chunks, d.max_chunks = 8192, 200, 5
    size = lambda k: lib.lmi_scan_workspace_bytes(C.byref(d), 10000, 4, k, _lib.LMI_Q_F16)
    try:
        monkeypatch.delenv("LMI_WIDE_PASSES", raising=False)
        lib.lmi_config_reload()
        wide100, wide30 = size(100), size(30)
        monkeypatch.setenv("LMI_WIDE_PASSES", "1")
        lib.lmi_config_reload()
        passes100, passes30 = size(100), size(30)
    finally:
        monkeypatch.delenv("LMI_WIDE_PASSES", raising=False)
        lib.lmi_config_reload()
    assert wide30 > passes30 > 0
    # the wide workspace holds the passes' own (its fix-up) and 40000 pairs x
    # 1024 candidate slots of 8 bytes
    assert wide100 > passes100 + 40000 * 1024 * 8
    assert size(100) == wide100


def test_replay_rejects_the_reference_assert_case():
    """k larger than the merged width: the reference asserts (LearnedIndex.py:99)."""
    from li.index import replay
    nq, R = 3, 2
    cls = np.zeros((nq, R), np.int32)
    d = np.zeros((nq, R, 10), np.float32)
    p = np.zeros((nq, R, 10), np.int32)
    with pytest.raises(_lib.LmiError):
        replay(cls, d, p, k_round=10, k_final=25, bucket_size=np.array([20]),
               pos_to_id=np.arange(1, 21), use_threshold=True)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_bucket_stripes_partition_every_bucket(world):
    rng = np.random.default_rng(0)
    lab = rng.integers(0, 7, 1000)
    lab[lab == 3] = 4  # an empty bucket
    L = BucketLayout.from_labels(lab, 7)
    seen = []
    for r in range(world):
        gpos, loc = L.shard(r, world)
        assert loc[-1] == gpos.size and np.all(np.diff(loc) >= 0)
        for c in range(7):
            part = gpos[loc[c]:loc[c + 1]]
            assert np.all((part >= L.bucket_off[c]) & (part < L.bucket_off[c + 1]))
            assert np.all(np.diff(part) == 1)  # contiguous slice, ascending
        seen.append(gpos)
    allp = np.sort(np.concatenate(seen))
    assert np.array_equal(allp, np.arange(1000))
    # stable in row order inside every bucket (groupby order, LearnedIndex.py:143-145)
    for c in range(7):
        rows = L.order[L.bucket_off[c]:L.bucket_off[c + 1]]
        assert np.all(np.diff(rows) > 0) and np.all(lab[rows] == c)


def test_subcluster_layout_keeps_rows_and_chunk_order():
    """Host-side index layout (no GPU compute): every bucket is re-ordered by
    sub-cluster, each chunk stays in ascending global position, every row keeps
    its vector / 1/||y|| / global position, and the chunk centroids are unit."""
    import numpy as np
    import torch
    import workloads
    from li.index import DeviceIndex
    w = workloads.clustered(n=3000, nq=8, C=8, seed=2, label_mode="skewed")
    ix = DeviceIndex(w["x"], w["labels"], w["C"], device="cpu", chunk_rows=64, subcluster=True)
    base = DeviceIndex(w["x"], w["labels"], w["C"], device="cpu", chunk_rows=64, subcluster=False)
    off = ix.bucket_off_local.numpy()
    cf = ix.chunk_first.numpy()
    gp, gp0 = ix.gpos.numpy(), base.gpos.numpy()
    moved = 0
    for c in range(w["C"]):
        a, b = off[c], off[c + 1]
        assert sorted(gp[a:b]) == list(gp0[a:b])           # same rows per bucket
        moved += int((gp[a:b] != gp0[a:b]).sum())
        for j in range(cf[c + 1] - cf[c]):
            seg = gp[a + 64 * j: min(b, a + 64 * (j + 1))]
            assert np.all(np.diff(seg) > 0)                  # ascending inside a chunk
    assert moved > 0                                          # the layout did change
    row_of = {int(g): i for i, g in enumerate(gp0)}
    idx = torch.tensor([row_of[int(g)] for g in gp])
    assert torch.equal(ix.corpus, base.corpus[idx])
    assert torch.equal(ix.inv_norm, base.inv_norm[idx])
    nrm = ix.chunk_centroid[:, : ix.d].norm(dim=1)
    assert torch.allclose(nrm, torch.ones_like(nrm), atol=1e-5)


def test_dist_dtype_follows_sklearn_rule():
    """float32 DataFrame + float32 queries: the reference's float32 branch;
    float16 (the real clip768 'emb') or float64 on either side: float64
    (utils.py:11 -> check_pairwise_arrays)."""
    import pandas as pd
    from li.LearnedIndex import dist_dtype
    x = np.zeros((4, 3), np.float32)
    assert dist_dtype(pd.DataFrame(x), x) == "f32"
    assert dist_dtype(pd.DataFrame(x.astype(np.float16)), x) == "f64"
    assert dist_dtype(pd.DataFrame(x), x.astype(np.float16)) == "f64"
    assert dist_dtype(pd.DataFrame(x).assign(category=1), x) == "f32"
    assert dist_dtype(x.astype(np.float64), x) == "f64"


def test_content_key_sees_in_place_changes():
    import pandas as pd
    from li.LearnedIndex import content_key
    df = pd.DataFrame(np.random.default_rng(0).standard_normal((50, 8)).astype(np.float16))
    k0 = content_key(df)
    assert content_key(df) == k0  # (a copy in another memory order may miss: safe)
    df.iloc[37, 5] = df.iloc[37, 5] + np.float16(1)
    assert content_key(df) != k0


def test_host_hash64_threads_and_sensitivity():
    """lmi_host_hash64 (the drop-in's index-cache key): independent of the
    thread count, sensitive to one changed byte anywhere, to the length, and
    equal for equal bytes in different buffers."""
    import numpy as np
    from li import _lib
    lib = _lib.load()
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (9 << 20) + 13, dtype=np.uint8)   # 2 full 4-MiB blocks + a tail
    h = [lib.lmi_host_hash64(a.ctypes.data, a.nbytes, t) for t in (1, 2, 3, 8, 0)]
    assert len(set(h)) == 1
    b = a.copy()
    assert lib.lmi_host_hash64(b.ctypes.data, b.nbytes, 4) == h[0]
    for pos in (0, 5 << 20, a.nbytes - 1):
        b[pos] ^= 1
        assert lib.lmi_host_hash64(b.ctypes.data, b.nbytes, 4) != h[0]
        b[pos] ^= 1
    assert lib.lmi_host_hash64(a.ctypes.data, a.nbytes - 1, 4) != h[0]
    assert lib.lmi_host_hash64(None, 0, 1) == lib.lmi_host_hash64(None, 0, 4)


def test_search_path_initialises_workspace_with_kernels():
    """The search step is captured as HIP graphs (li.index.GraphedSearch); round 3
    measured captured hipMemsetAsync nodes answering wrong lists once eager copies
    ran between replays of two graphs, so the search path's sources initialise
    device memory with fill kernels (lmi::fill_u32), never hipMemsetAsync/hipMemset."""
    csrc = os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd", "csrc")
    for name in ("lmi_scan.hip", "lmi_scan_v12.hip", "lmi_refine.hip", "lmi_merge.hip",
                 "lmi_replay_gpu.hip", "lmi_router.hip", "lmi_abi.cpp"):
        src = open(os.path.join(csrc, name)).read()
        assert not re.search(r"\bhipMemset\w*\s*\(", src), name


@pytest.mark.parametrize("scalar", [False, True])
def test_host_stage_f16_matches_numpy(scalar, monkeypatch):
    """lmi_host_stage_f16 (the batch stream's staging of a float32 host batch):
    numpy's float16 rounding bit for bit, and its exactness flag equals numpy's
    array_equal(q.astype(f16).astype(f32), q) -- on normals, subnormals, the
    rounding ties, overflow to inf, signed zeros and NaN, with the F16C path
    and the scalar one (LMI_HOST_SCALAR=1)."""
    import numpy as np
    from li import _lib
    if scalar:
        monkeypatch.setenv("LMI_HOST_SCALAR", "1")
    lib = _lib.load()
    rng = np.random.default_rng(11)
    h = rng.integers(0, 1 << 16, 300_001, dtype=np.uint16).view(np.float16)
    exact = h.astype(np.float32)
    exact = exact[~np.isnan(exact)]
    # every half value, ties between neighbours, values between, and extremes
    a = np.concatenate([exact, exact * np.float32(1 + 2 ** -11), exact * np.float32(1 + 2 ** -12),
                        exact * np.float32(1 + 3 * 2 ** -13),
                        rng.standard_normal(100_000).astype(np.float32) * np.float32(2.0) **
                        rng.integers(-30, 20, 100_000).astype(np.float32),
                        np.array([65504, 65519.99, 65520, -65520, 1e30, -0.0, 0.0, 2 ** -25,
                                  2 ** -25 * 1.0001, 2 ** -24, 3 * 2 ** -25, np.inf, -np.inf],
                                 np.float32)])
    with np.errstate(over="ignore"):
        ref = a.astype(np.float16)
    out = np.empty(a.size, np.uint16)
    for t in (1, 3, 0):
        out[:] = 0
        assert lib.lmi_host_stage_f16(a.ctypes.data, a.size, out.ctypes.data, t) == 0
        np.testing.assert_array_equal(out, ref.view(np.uint16))
    ok = exact.astype(np.float32)
    out = np.empty(ok.size, np.uint16)
    assert lib.lmi_host_stage_f16(ok.ctypes.data, ok.size, out.ctypes.data, 0) == 1
    np.testing.assert_array_equal(out, ok.astype(np.float16).view(np.uint16))
    nan = np.array([1.0, np.nan], np.float32)
    o2 = np.empty(2, np.uint16)
    assert lib.lmi_host_stage_f16(nan.ctypes.data, 2, o2.ctypes.data, 1) == 0
    assert np.isnan(o2.view(np.float16)[1])
    assert lib.lmi_host_stage_f16(None, 4, o2.ctypes.data, 1) == -_lib.LMI_E_INVALID
    assert lib.lmi_host_stage_f16(None, 0, None, 1) == 1


def test_host_copy():
    import numpy as np
    from li import _lib
    lib = _lib.load()
    a = np.random.default_rng(2).integers(0, 256, (5 << 20) + 77, dtype=np.uint8)
    b = np.zeros_like(a)
    assert lib.lmi_host_copy(b.ctypes.data, a.ctypes.data, a.nbytes, 0) == 0
    np.testing.assert_array_equal(a, b)
    assert lib.lmi_host_copy(None, a.ctypes.data, 5, 1) == _lib.LMI_E_INVALID


def test_default_chunk_rows_by_world_and_size():
    """8192 / 4096 / 2048 rows by world, halved (to 1024 at least) while a
    rank's shard would hold fewer than 64 chunks."""
    from li.index import default_chunk_rows
    assert [default_chunk_rows(w) for w in (1, 2, 4, 8)] == [8192, 4096, 4096, 2048]
    assert default_chunk_rows(1, 10_000_000) == 8192
    assert default_chunk_rows(8, 10_000_000) == 2048
    assert default_chunk_rows(1, 100_000_000) == 8192
    assert default_chunk_rows(1, 1_000_000) == 8192
    assert default_chunk_rows(1, 300_000) == 4096
    assert default_chunk_rows(1, 100_000) == 1024
    assert default_chunk_rows(4, 1_000) == 1024


def test_scan_workgroups_setting_is_per_thread():
    """lmi_scan_set_workgroups (ABI 12) returns the previous setting, clamps
    negatives to 0 (every CU) and is the calling thread's own."""
    import threading
    lib = _lib.load()
    assert lib.lmi_scan_set_workgroups(200) == 0
    seen = []
    t = threading.Thread(target=lambda: seen.append(lib.lmi_scan_set_workgroups(5)))
    t.start()
    t.join()
    assert seen == [0]
    assert lib.lmi_scan_set_workgroups(-3) == 200
    assert lib.lmi_scan_set_workgroups(0) == 0
