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
