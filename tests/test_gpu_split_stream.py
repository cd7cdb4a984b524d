"""The split mode's phases (ABI 11: lmi_bucket_topk / _f64 with PLAN, SCAN and
MERGE on a corpus32 index, k <= 10) compose to the one-call result, and the
batch stream over a split index (StreamedSearch with float32 batches)
answers every batch exactly as Searcher.search does."""
import numpy as np
import pytest
import torch

import workloads
from li import _lib
from li.index import DeviceIndex, DeviceRouter, Searcher, bucket_topk, bucket_topk_f64

pytestmark = pytest.mark.gpu
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731


@pytest.fixture(scope="module")
def setup():
    w = workloads.clustered(n=6000, nq=300, C=16, seed=71, label_mode="near")
    x32, q32 = workloads.float32_inputs(w, 71)
    ix = DeviceIndex(x32, w["labels"], w["C"], chunk_rows=512, device="cuda")
    assert ix.storage == "f32x"
    return w, q32, Searcher(ix, DeviceRouter(w["layers"], device="cuda"))


def _batches(w, q32, n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        p = rng.permutation(q32.shape[0])
        out.append((w["qn"][p], q32[p]))
    return out


@pytest.mark.parametrize("dist", ["f32", "f64"])
@pytest.mark.parametrize("k", [10, 7, 1])
def test_split_phases_compose_to_one_call(setup, dist, k):
    w, q32, s = setup
    ix = s.index
    q = T(q32)
    cls = s.router.topr(T(w["qn"]), 4)[0]
    fn = bucket_topk_f64 if dist == "f64" else bucket_topk
    d0, p0, st0 = fn(ix, q, cls, k)
    ws = torch.empty_like(ix._ws["f64"] if dist == "f64" else ix._ws["buf"])
    outd, outp = torch.empty_like(d0), torch.empty_like(p0)
    st = torch.zeros((1,), dtype=torch.int32, device="cuda")
    for ph in (_lib.LMI_Q_PHASE_PLAN, _lib.LMI_Q_PHASE_SCAN, _lib.LMI_Q_PHASE_MERGE):
        fn(ix, q, cls, k, out=(outd, outp, st), ws=ws, phases=ph)
    assert torch.equal(outd, d0) and torch.equal(outp, p0) and int(st.item()) == int(st0.item())


def test_split_phases_need_k_at_most_10(setup):
    w, q32, s = setup
    cls = s.router.topr(T(w["qn"]), 4)[0]
    with pytest.raises(_lib.LmiError, match="k <= 10"):
        bucket_topk(s.index, T(q32), cls, 12, phases=_lib.LMI_Q_PHASE_PLAN)


@pytest.mark.parametrize("dist,R", [("f32", 4), ("f64", 4), ("f32", 1)])
def test_split_stream_of_batches_equals_search(setup, dist, R):
    w, q32, s = setup
    bs = _batches(w, q32, 6, seed=R)
    ref = [s.search(T(a), T(b), R, k=10, dist=dist) for a, b in bs]
    st = s.streamed(w["qn"], q32, R, k=10, dist=dist)
    assert st.split
    got = list(st.stream(bs))
    st.close()
    assert len(got) == len(bs)
    for (d, a), (d0, a0) in zip(got, ref):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)


@pytest.mark.parametrize("n", [1, 2])
def test_split_short_streams(setup, n):
    w, q32, s = setup
    bs = _batches(w, q32, n, seed=20 + n)
    ref = [s.search(T(a), T(b), 4, k=10) for a, b in bs]
    with s.streamed(w["qn"], q32, 4, k=10) as st:
        got = list(st.stream(bs))
    assert len(got) == n
    for (d, a), (d0, a0) in zip(got, ref):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)


def test_split_stream_needs_k_round_at_most_10(setup):
    w, q32, s = setup
    with pytest.raises(ValueError, match="k_round <= 10"):
        s.streamed(w["qn"], q32, 4, k=10, k_round=12)
