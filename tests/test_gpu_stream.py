"""StreamedSearch (li.stream: the step as a four-stage pipeline of captured graphs
over a stream of batches -- route and plan of batch t, scan of t-2,
merge/replay/D2H of t-3 in one launch) answers every batch exactly as
Searcher.search does; the phase flags of lmi_bucket_topk (ABI 7) compose to
the one-call result."""
import numpy as np
import pytest
import torch

import workloads
from li import _lib
from li.index import DeviceIndex, DeviceRouter, Searcher, bucket_topk, bucket_topk_f64

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    w = workloads.clustered(n=6000, nq=300, C=16, seed=61, label_mode="near")
    s = Searcher(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda"),
                 DeviceRouter(w["layers"], device="cuda"))
    return w, s


def _batches(w, n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        p = rng.permutation(w["q"].shape[0])
        out.append((w["qn"][p], w["q"][p]))
    return out


T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("dist", ["f32", "f64"])
@pytest.mark.parametrize("k", [10, 7])
def test_phases_compose_to_one_call(setup, dist, k):
    w, s = setup
    ix = s.index
    q = T(w["q"])
    cls = s.router.topr(T(w["qn"]), 4)[0]
    fn = bucket_topk_f64 if dist == "f64" else bucket_topk
    d0, p0, st0 = fn(ix, q, cls, k, qmode=_lib.LMI_Q_F16)
    ws = torch.empty_like(ix._ws["f64"] if dist == "f64" else ix._ws["buf"])
    outd = torch.empty_like(d0)
    outp = torch.empty_like(p0)
    st = torch.zeros((1,), dtype=torch.int32, device="cuda")
    for ph in (_lib.LMI_Q_PHASE_PLAN, _lib.LMI_Q_PHASE_SCAN, _lib.LMI_Q_PHASE_MERGE):
        fn(ix, q, cls, k, qmode=_lib.LMI_Q_F16, out=(outd, outp, st), ws=ws, phases=ph)
    assert torch.equal(outd, d0) and torch.equal(outp, p0) and int(st.item()) == int(st0.item())


@pytest.mark.parametrize("dist,R", [("f32", 4), ("f64", 4), ("f32", 1), ("f32", 7)])
def test_stream_of_batches_equals_search(setup, dist, R):
    w, s = setup
    bs = _batches(w, 6, seed=R)
    ref = [s.search(T(a), T(b), R, k=10, dist=dist) for a, b in bs]
    st = s.streamed(w["qn"], w["q"], R, k=10, dist=dist)
    got = list(st.stream(bs))
    assert len(got) == len(bs)
    for (d, a), (d0, a0) in zip(got, ref):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)


@pytest.mark.parametrize("n", [1, 2, 3, 4])
def test_short_streams(setup, n):
    w, s = setup
    bs = _batches(w, n, seed=10 + n)
    ref = [s.search(T(a), T(b), 4, k=10) for a, b in bs]
    got = list(s.streamed(w["qn"], w["q"], 4, k=10).stream(bs))
    assert len(got) == n
    for (d, a), (d0, a0) in zip(got, ref):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)


def test_steps_on_one_staged_batch(setup):
    """The bench's use: one batch staged in every slot, step() after step(),
    with eager work between launches."""
    w, s = setup
    d0, a0 = s.search(T(w["qn"]), T(w["q"]), 4, k=10)
    st = s.streamed(w["qn"], w["q"], 4, k=10)
    for i in range(7):
        d, a = st.step()
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)
        if i == 3:
            junk = [t.clone() for t in vars(s.index).values() if isinstance(t, torch.Tensor) and t.is_cuda]
            s.search(T(w["qn"][::-1].copy()), T(w["q"][::-1].copy()), 4, k=10)
            del junk


def test_stream_rejects_inexact_batches(setup):
    w, s = setup
    st = s.streamed(w["qn"], w["q"], 4, k=10)
    assert not st.stage(w["qn"], w["q"] + np.float32(1e-5))
    with pytest.raises(ValueError):
        s.streamed(w["qn"], w["q"] + np.float32(1e-5), 4, k=10)


@pytest.mark.parametrize("lookahead", [False, True])
def test_stream_with_and_without_lookahead(setup, lookahead):
    """The next launch's scan enqueued ahead (the default) or not: the same
    answers, batch by batch, and over repeated steps."""
    w, s = setup
    bs = _batches(w, 5, seed=40)
    ref = [s.search(T(a), T(b), 4, k=10) for a, b in bs]
    st = s.streamed(w["qn"], w["q"], 4, k=10, lookahead=lookahead)
    got = list(st.stream(bs))
    for (d, a), (d0, a0) in zip(got, ref):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)
    d0, a0 = s.search(T(w["qn"]), T(w["q"]), 4, k=10)
    st = s.streamed(w["qn"], w["q"], 4, k=10, lookahead=lookahead)
    for _ in range(4):
        d, a = st.step()
        np.testing.assert_array_equal(a, a0)


@pytest.mark.parametrize("dist,reserve", [("f32", 0), ("f32", 8), ("f32", 255), ("f64", 16)])
def test_stream_with_cus_left_to_the_finish(setup, dist, reserve):
    """reserve_cus (ABI 12 lmi_scan_set_workgroups): the scan's grid leaves
    CUs to the finish chain and the lookahead scan stops waiting for it --
    the same answers, batch by batch; the setting is the stream's own (the
    thread's grid is back to every CU after each scan)."""
    w, s = setup
    lib = _lib.load()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    reserve = min(reserve, ncu - 1)
    bs = _batches(w, 6, seed=70 + reserve)
    ref = [s.search(T(a), T(b), 4, k=10, dist=dist) for a, b in bs]
    st = s.streamed(w["qn"], w["q"], 4, k=10, dist=dist, reserve_cus=reserve)
    assert st.overlap == (reserve > 0) and st.scan_wgs == (ncu - reserve if reserve else 0)
    got = list(st.stream(bs))
    for (d, a), (d0, a0) in zip(got, ref):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)
    assert lib.lmi_scan_set_workgroups(0) == 0
    with pytest.raises(ValueError):
        s.streamed(w["qn"], w["q"], 4, k=10, reserve_cus=ncu)


@pytest.mark.parametrize("where", [0, 2, 5])
def test_inexact_batch_in_a_stream_is_answered_eagerly(setup, where):
    """A batch whose clip768 values fp16 cannot hold, in the middle of a stream
    (or in the pipeline fill): staged with its flag, the launch that finishes it
    raises QueryNotF16, and stream() answers it by Searcher.search (exact fp32
    MFMA); every other batch still comes from the stream, all equal to search."""
    w, s = setup
    bs = _batches(w, 7, seed=90 + where)
    bs[where] = (bs[where][0], bs[where][1] + np.float32(1e-5))
    ref = [s.search(T(a), T(b), 4, k=10) for a, b in bs]
    got = list(s.streamed(w["qn"], w["q"], 4, k=10).stream(bs))
    assert len(got) == len(bs)
    for (d, a), (d0, a0) in zip(got, ref):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)


def test_step_raises_on_an_inexact_staged_batch(setup):
    from li.stream import QueryNotF16
    w, s = setup
    st = s.streamed(w["qn"], w["q"], 4, k=10)
    d0, a0 = s.search(T(w["qn"]), T(w["q"]), 4, k=10)
    st.step()
    assert not st.stage(w["qn"], w["q"] + np.float32(1e-5))   # the slot of launch 1
    for _ in range(3):                                         # launches 1-3 finish slots 2, 3, 0
        d, a = st.step()
        np.testing.assert_array_equal(a, a0)
    with pytest.raises(QueryNotF16):
        st.step()                                              # launch 4 finishes it
    d, a = st.step()                                           # the stream goes on
    np.testing.assert_array_equal(a, a0)


def test_stream_of_float16_host_batches(setup):
    """Batches held as float16 host arrays (the real clip768 'emb' dtype) are
    staged by a copy; answers equal search on the same values."""
    w, s = setup
    bs = [(a, b.astype(np.float16)) for a, b in _batches(w, 6, seed=123)]
    ref = [s.search(T(a), T(b.astype(np.float32)), 4, k=10) for a, b in bs]
    got = list(s.streamed(w["qn"], w["q"], 4, k=10).stream(bs))
    for (d, a), (d0, a0) in zip(got, ref):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)


def test_queue_streams_run_beside_each_other():
    """li.stream.queue_streams: the streams the batch stream runs its finish,
    plan and route on take work while the current stream, and each other,
    are busy (each on its own hardware queue: GPU_MAX_HW_QUEUES is 4 on the
    box, so the scan's stream and these three fill them)."""
    from li.stream import _runs_beside, _spin_cycles, queue_streams
    ss = queue_streams("cuda", 3)
    assert len({s.cuda_stream for s in ss}) == 3
    main = torch.cuda.current_stream()
    spin = _spin_cycles(main, 10.0)
    for i, s in enumerate(ss):
        assert _runs_beside(main, s, spin, 5e-3)
        for o in ss[:i]:
            assert _runs_beside(o, s, spin, 5e-3)


def test_stream_objects_dropped_with_work_in_flight(setup):
    """a StreamedSearch dropped right after step() (its
    lookahead scan still queued) and a new one on the very same streams: the
    old object's __del__ -> close() waits for its work before its graphs and
    their pools are released, so the new object's answers are bitwise those
    of Searcher.search.  Twice, back to back."""
    import gc
    w, s = setup
    bs = _batches(w, 5, seed=77)
    ref = [s.search(T(a), T(b), 4, k=10) for a, b in bs]
    saved = None
    for rep in range(2):
        st = s.streamed(w["qn"], w["q"], 4, k=10, lookahead=True)
        if saved is not None:
            st._fs, st._ps, st._rs = saved   # the streams deliberately shared
            st._cs = st._rs
        got = list(st.stream(bs))
        for (d, a), (d0, a0) in zip(got, ref):
            np.testing.assert_array_equal(d, d0)
            np.testing.assert_array_equal(a, a0)
        assert st.launches == len(bs) - 3
        st.stage(*bs[0])
        st.step()                            # leaves its lookahead scan in flight
        saved = (st._fs, st._ps, st._rs)
        del st
        gc.collect()                         # (the stage closures hold a cycle)


def test_close_is_idempotent_and_final(setup):
    w, s = setup
    st = s.streamed(w["qn"], w["q"], 4, k=10)
    st.step()
    st.close()
    st.close()
    assert st.graphs is None
    with pytest.raises(RuntimeError):
        st.step()
    with s.streamed(w["qn"], w["q"], 4, k=10) as st2:
        st2.step()
    assert st2.graphs is None


def test_object_finalised_inside_another_capture_is_parked(setup):
    """The round-5 abort's cause, reproduced on purpose: a StreamedSearch
    becomes cyclic garbage and the collector finalises it while another graph
    is being captured.  Destroying its graphs (or synchronising its events)
    there would abort the process; close() parks them instead (li._host
    "graph lifetime"), the capture completes and replays, and the parked
    graphs are released at the next safe point."""
    import gc
    from li import _host
    w, s = setup
    st = s.streamed(w["qn"], w["q"], 4, k=10)
    st.step()
    holder = [st]
    del st
    x = torch.zeros(4, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        holder.clear()          # the last reference: the object is now cyclic garbage
        gc.collect()            # its finaliser runs mid-capture
        x += 1
    assert len(_host._PARKED) == 1
    g.replay()
    torch.cuda.synchronize()
    assert int(x.sum()) == 4
    _host.flush_released()
    assert not _host._PARKED
    d0, a0 = s.search(T(w["qn"]), T(w["q"]), 4, k=10)
    d, a = s.streamed(w["qn"], w["q"], 4, k=10).step()
    np.testing.assert_array_equal(d, d0)
    np.testing.assert_array_equal(a, a0)
