"""The step captured as a HIP graph (Searcher.graph / GraphedSearch) answers
exactly as the eager Searcher.search, replay after replay, for new batches
copied into its query buffers, and falls back to the eager path for a batch
that is not fp16-exact under an fp16 capture."""
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
    g = s.graph(qn, q, R, k=10, dist=dist)
    for _ in range(3):
        d1, a1 = g.run()
        np.testing.assert_array_equal(d1, d0)
        np.testing.assert_array_equal(a1, a0)


def test_graph_new_batch_and_inexact_queries(setup):
    w, s = setup
    qn = torch.from_numpy(w["qn"]).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    g = s.graph(qn.clone(), q.clone(), 4, k=10)
    perm = torch.randperm(q.shape[0], generator=torch.Generator().manual_seed(0))
    g.q_nav.copy_(qn[perm.cuda()])
    g.q_search.copy_(q[perm.cuda()])
    d1, a1 = g.run()
    d0, a0 = s.search(qn[perm.cuda()], q[perm.cuda()], 4, k=10)
    np.testing.assert_array_equal(d1, d0)
    np.testing.assert_array_equal(a1, a0)
    # not fp16-exact: the capture's fp16 path flags it, the eager fp32 path answers
    g.q_search.add_(1e-5)
    d2, a2 = g.run()
    d3, a3 = s.search(g.q_nav, g.q_search, 4, k=10)
    np.testing.assert_array_equal(d2, d3)
    np.testing.assert_array_equal(a2, a3)


@pytest.mark.parametrize("dist,depth", [("f32", 2), ("f64", 2), ("f32", 3)])
def test_pipeline_batches_in_flight(setup, dist, depth):
    """PipelinedSearch: several batches in flight (different queries per
    batch, written into the capture's query buffers on the compute stream
    between submits); every ticket's answer equals the eager search of its
    own batch."""
    w, s = setup
    qn = torch.from_numpy(w["qn"]).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    p = s.pipeline(qn.clone(), q.clone(), 4, k=10, dist=dist, depth=depth)
    g = torch.Generator().manual_seed(3)
    perms = [torch.randperm(q.shape[0], generator=g).cuda() for _ in range(7)]
    want = [s.search(qn[pm], q[pm], 4, k=10, dist=dist) for pm in perms]
    got, tickets = [], []
    for i, pm in enumerate(perms):
        if i >= depth:
            t = tickets.pop(0)
            d, a = p.result(t)
            got.append((d.copy(), a.copy()))
        p.q_nav.copy_(qn[pm])
        p.q_search.copy_(q[pm])
        tickets.append(p.submit())
    for t in tickets:
        d, a = p.result(t)
        got.append((d.copy(), a.copy()))
    assert len(got) == len(want)
    for (d1, a1), (d0, a0) in zip(got, want):
        np.testing.assert_array_equal(d1, d0)
        np.testing.assert_array_equal(a1, a0)


def test_pipeline_order_and_capacity(setup):
    w, s = setup
    qn = torch.from_numpy(w["qn"]).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    p = s.pipeline(qn, q, 4, k=10, depth=2)
    t0, t1 = p.submit(), p.submit()
    with pytest.raises(RuntimeError):
        p.submit()  # both slots hold uncollected answers
    with pytest.raises(ValueError):
        p.result(t1)  # out of order
    d0, a0 = p.result(t0)
    d1, a1 = p.result(t1)
    np.testing.assert_array_equal(d0, d1)
    np.testing.assert_array_equal(a0, a1)
