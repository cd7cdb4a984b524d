"""The step captured as a HIP graph (Searcher.graph / GraphedSearch), from the
batch in host memory (staged in pinned buffers, uploaded inside the step) to
the answer in host memory, answers exactly as the eager Searcher.search,
replay after replay, for new batches staged between replays; a batch that is
not fp16-exact under an fp16 capture is answered by the eager path; and the
graph keeps working after eager calls that grow the index's own workspace."""
import numpy as np
import pytest
import torch

import workloads
from li.index import DeviceIndex, DeviceRouter, Searcher

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    w = workloads.clustered(n=6000, nq=300, C=16, seed=51, label_mode="near")
    s = Searcher(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda"),
                 DeviceRouter(w["layers"], device="cuda"))
    return w, s


@pytest.mark.parametrize("dist,R", [("f32", 4), ("f64", 4), ("f32", 1), ("f64", 7)])
def test_graph_equals_eager(setup, dist, R):
    w, s = setup
    qn = torch.from_numpy(w["qn"]).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    d0, a0 = s.search(qn, q, R, k=10, dist=dist)
    g = s.graph(w["qn"], w["q"], R, k=10, dist=dist)   # host batch, staged
    assert g.f16_up
    for _ in range(3):
        d1, a1 = g.run()
        np.testing.assert_array_equal(d1, d0)
        np.testing.assert_array_equal(a1, a0)


def test_graph_new_batch_and_inexact_queries(setup):
    w, s = setup
    g = s.graph(w["qn"], w["q"], 4, k=10)
    perm = np.random.default_rng(0).permutation(w["q"].shape[0])
    qn2, q2 = w["qn"][perm], w["q"][perm]
    d1, a1 = g.run(qn2, q2)
    d0, a0 = s.search(torch.from_numpy(qn2).cuda(), torch.from_numpy(q2).cuda(), 4, k=10)
    np.testing.assert_array_equal(d1, d0)
    np.testing.assert_array_equal(a1, a0)
    # float16 input stages as it is
    d1, a1 = g.run(qn2, q2.astype(np.float16))
    np.testing.assert_array_equal(d1, d0)
    np.testing.assert_array_equal(a1, a0)
    # not fp16-exact: the fp16 capture cannot stage it, the eager fp32 path answers
    q3 = q2 + np.float32(1e-5)
    d2, a2 = g.run(qn2, q3)
    d3, a3 = s.search(torch.from_numpy(qn2).cuda(), torch.from_numpy(q3).cuda(), 4, k=10)
    np.testing.assert_array_equal(d2, d3)
    np.testing.assert_array_equal(a2, a3)
    # and the graph still answers fp16-exact batches afterwards
    d4, a4 = g.run(w["qn"], w["q"])
    d5, a5 = s.search(torch.from_numpy(w["qn"]).cuda(), torch.from_numpy(w["q"]).cuda(), 4, k=10)
    np.testing.assert_array_equal(d4, d5)
    np.testing.assert_array_equal(a4, a5)


def test_graph_f32_staging(setup):
    """A batch that is not fp16-exact at capture stages as float32 rows."""
    w, s = setup
    q = w["q"] + np.float32(1e-5)
    g = s.graph(w["qn"], q, 4, k=10)
    assert not g.f16_up
    d0, a0 = s.search(torch.from_numpy(w["qn"]).cuda(), torch.from_numpy(q).cuda(), 4, k=10)
    d1, a1 = g.run()
    np.testing.assert_array_equal(d1, d0)
    np.testing.assert_array_equal(a1, a0)


@pytest.mark.parametrize("dist", ["f32", "f64"])
def test_graph_survives_workspace_growth(setup, dist):
    """an eager call with a bigger batch replaces the index's cached
    scan workspace; the graph owns its own, so its replays stay correct."""
    w, s = setup
    g = s.graph(w["qn"], w["q"], 4, k=10, dist=dist)
    d0, a0 = g.run()
    d0, a0 = d0.copy(), a0.copy()
    big = 4
    qn_big = torch.from_numpy(np.tile(w["qn"], (big, 1))).cuda()
    q_big = torch.from_numpy(np.tile(w["q"], (big, 1))).cuda()
    s.search(qn_big, q_big, 7, k=10, dist=dist)      # more pairs: a bigger workspace
    torch.cuda.empty_cache()
    junk = torch.full((64 << 20,), 7, dtype=torch.int32, device="cuda")  # reuse freed memory
    d1, a1 = g.run()
    del junk
    np.testing.assert_array_equal(d1, d0)
    np.testing.assert_array_equal(a1, a0)


@pytest.mark.parametrize("dist", ["f32", "f64"])
def test_pipelined_graph_stream_of_batches(setup, dist):
    """pipeline=True: two device copies of the staged batch, each with its own
    graph; every run uploads the staged batch into the other copy while its
    graph runs.  Any sequence of runs and newly staged batches answers like
    the eager search of that batch."""
    w, s = setup
    g = s.graph(w["qn"], w["q"], 4, k=10, dist=dist, pipeline=True)
    assert g.pipeline and len(g.graphs) == 2
    d0, a0 = s.search(torch.from_numpy(w["qn"]).cuda(), torch.from_numpy(w["q"]).cuda(), 4, k=10,
                      dist=dist)
    for _ in range(5):                         # both slots, several times each
        d1, a1 = g.run()
        np.testing.assert_array_equal(d1, d0)
        np.testing.assert_array_equal(a1, a0)
    perm = np.random.default_rng(1).permutation(w["q"].shape[0])
    qn2, q2 = w["qn"][perm], w["q"][perm]
    e0, b0 = s.search(torch.from_numpy(qn2).cuda(), torch.from_numpy(q2).cuda(), 4, k=10, dist=dist)
    d2, a2 = g.run(qn2, q2)                    # a new batch: staged, then answered
    np.testing.assert_array_equal(d2, e0)
    np.testing.assert_array_equal(a2, b0)
    for _ in range(3):                         # and streamed again from then on
        d3, a3 = g.run()
        np.testing.assert_array_equal(d3, e0)
        np.testing.assert_array_equal(a3, b0)
    d4, a4 = g.run(w["qn"], w["q"])            # back to the first batch
    np.testing.assert_array_equal(d4, d0)
    np.testing.assert_array_equal(a4, a0)


@pytest.mark.parametrize("pipeline", [False, True])
def test_graph_replays_survive_eager_work_between(setup, pipeline):
    """Eager work between replays (a search of another batch, clones of the index's
    tables) leaves the captured graphs' answers unchanged.  Round 3: with the
    workspace initialised by hipMemsetAsync (memset nodes in the captured
    graphs), the pipelined pair of graphs answered wrong lists after exactly
    this sequence; the library initialises its workspace with kernels now."""
    w, s = setup
    T = lambda a: torch.from_numpy(a).cuda()
    perm = np.random.default_rng(3).permutation(w["q"].shape[0])
    qn2, q2 = w["qn"][perm], w["q"][perm]
    d0, a0 = s.search(T(w["qn"]), T(w["q"]), 4, k=10)
    e0, b0 = s.search(T(qn2), T(q2), 4, k=10)
    g = s.graph(w["qn"], w["q"], 4, k=10, pipeline=pipeline)
    g.run()
    junk = [t.clone() for t in vars(s.index).values() if isinstance(t, torch.Tensor) and t.is_cuda]
    s.search(T(qn2), T(q2), 4, k=10)
    for _ in range(3):
        d1, a1 = g.run()
        np.testing.assert_array_equal(d1, d0)
        np.testing.assert_array_equal(a1, a0)
    del junk
    d2, a2 = g.run(qn2, q2)
    np.testing.assert_array_equal(d2, e0)
    np.testing.assert_array_equal(a2, b0)


def test_launch_one_ahead_answers_each_batch(setup):
    """GraphedSearch(pipeline=True).launch / result: a step launched before the
    previous one's answer is read; every answer equals the eager search of the
    batch staged for it, across a restaged batch."""
    w, s = setup
    T = lambda a: torch.from_numpy(a).cuda()
    perm = np.random.default_rng(7).permutation(w["q"].shape[0])
    qn2, q2 = w["qn"][perm], w["q"][perm]
    d0, a0 = s.search(T(w["qn"]), T(w["q"]), 4, k=10)
    e0, b0 = s.search(T(qn2), T(q2), 4, k=10)
    g = s.graph(w["qn"], w["q"], 4, k=10, pipeline=True)
    t = g.launch()
    for _ in range(5):
        t2 = g.launch()
        d, a = g.result(t)
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)
        t = t2
    d, a = g.result(t)
    np.testing.assert_array_equal(a, a0)
    assert g.stage(qn2, q2)
    t = g.launch()
    t2 = g.launch()
    for tk in (t, t2):
        d, a = g.result(tk)
        np.testing.assert_array_equal(d, e0)
        np.testing.assert_array_equal(a, b0)


@pytest.mark.parametrize("pipeline,dist", [(True, "f32"), (True, "f64"), (False, "f32")])
def test_graph_stream_answers_each_batch(setup, pipeline, dist):
    """GraphedSearch.stream: with pipeline=True batch i + 1 is staged into the
    other slot's pinned buffer and uploaded while batch i's step runs; every
    answer equals the eager search of its own batch, in order, across a batch
    the fp16 capture cannot stage (answered eagerly, in its place), and run()
    without arguments afterwards replays the last staged batch."""
    w, s = setup
    T = lambda a: torch.from_numpy(a).cuda()
    rng = np.random.default_rng(11)
    batches = []
    for i in range(7):
        perm = rng.permutation(w["q"].shape[0])
        qn, q = w["qn"][perm], w["q"][perm]
        if i == 4:
            q = q + np.float32(1e-5)   # not fp16-exact
        batches.append((qn, q))
    want = [s.search(T(qn), T(q), 4, k=10, dist=dist) for qn, q in batches]
    g = s.graph(w["qn"], w["q"], 4, k=10, dist=dist, pipeline=pipeline)
    got = list(g.stream(iter(batches)))
    assert len(got) == len(batches)
    for (d, a), (d0, a0) in zip(got, want):
        np.testing.assert_array_equal(d, d0)
        np.testing.assert_array_equal(a, a0)
    for _ in range(3):
        d, a = g.run()
        np.testing.assert_array_equal(d, want[-1][0])
        np.testing.assert_array_equal(a, want[-1][1])
