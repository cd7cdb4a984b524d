"""GPU drop-in vs the reference's own outputs (tests/golden/reference_outputs.npz):
li.LearnedIndex.search / search_single and li.model.NeuralNetwork on MI355X,
called exactly as search/search.py calls the reference."""
import os

import numpy as np
import pandas as pd
import pytest
import torch

import lmi_oracle as O
from golden.gen_golden import SEARCH_CASES, SINGLE_CASES
from test_oracle_golden import G, _inputs

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


@pytest.mark.parametrize("case", SEARCH_CASES, ids=[c[0] for c in SEARCH_CASES])
def test_learned_index_search_matches_reference(case):
    from li.LearnedIndex import LearnedIndex
    from li.model import data_X_to_torch
    name, n, nq, C, R, k, mode, arch, seed, thr = case
    w = _inputs(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    _, classes = li.model.predict_proba(data_X_to_torch(w["qn"]))
    ref_cls = G[f"search_{name}__classes"].astype(np.int64)
    assert (classes[:, :R] == ref_cls[:, :R]).all(), "router top-R differs from the reference"
    data = pd.DataFrame(w["xn"])
    data.index += 1
    data_search = pd.DataFrame(w["x"])
    data_search.index += 1
    dists, anns = li.search(data, w["qn"], data_search, w["q"], w["labels"], n_buckets=R, k=k,
                            use_threshold=thr)
    assert "category" in data.columns  # LearnedIndex.py:67 side effect
    ref_d, ref_a = G[f"search_{name}__dists"], G[f"search_{name}__anns"]
    assert dists.dtype == np.float64 and anns.dtype == np.uint32 and dists.shape == ref_d.shape
    assert O.compare_lists(ref_d, ref_a, dists, anns) == 0


@pytest.mark.parametrize("case", SINGLE_CASES, ids=[c[0] for c in SINGLE_CASES])
def test_learned_index_search_single_matches_reference(case):
    from li.LearnedIndex import LearnedIndex
    name, n, nq, C, R, k, mode, arch, seed, thr = case
    w = _inputs(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    data = pd.DataFrame(w["xn"])
    data.index += 1
    data["category"] = w["labels"]
    data_search = pd.DataFrame(w["x"])
    data_search.index += 1
    classes = G[f"search_{name}__classes"].astype(np.int64)
    thr_arr = G[f"search_{name}__thr"] if thr else None
    dists, anns = li.search_single(data, data_search, w["q"], classes[:, 0], k=k,
                                   threshold_dist=thr_arr)
    ref_d, ref_a = G[f"search_{name}__dists"], G[f"search_{name}__anns"]
    assert O.compare_lists(ref_d, ref_a, dists, anns) == 0


@pytest.mark.parametrize("key", ["router_MLP_122", "router_MLP-5_122", "router_MLP_16"])
def test_neural_network_predict_matches_reference(key):
    layers, i = [], 0
    while f"{key}__W{i}" in G.files:
        layers.append((G[f"{key}__W{i}"], G[f"{key}__b{i}"]))
        i += 1
    arch = key.split("_")[1]
    C = int(key.split("_")[2])
    nn = _nn(layers, arch, C)
    x = torch.from_numpy(G[f"{key}__x"])
    probs, classes = nn.predict_proba(x)
    assert probs.shape == (x.shape[0], C) and classes.dtype == np.int64
    ref = G[f"{key}__classes"].astype(np.int64)
    assert (classes[:, :16] != ref).any(axis=1).sum() == 0
    np.testing.assert_allclose(probs[:, :16], G[f"{key}__probs"], rtol=2e-5, atol=1e-7)
    assert (nn.predict(x) == G[f"{key}__predict"]).all()


def test_baseline_matches_exact_oracle():
    from li.Baseline import Baseline
    w = _inputs("skew_r4")
    dists, nns, _ = Baseline().search(w["q"], w["x"], k=10)
    D = O.pairwise_cosine(w["x"], w["q"]).T
    ref_n = np.argsort(D, kind="stable")[:, :10] + 1
    ref_d = np.sort(D)[:, :10]
    assert O.compare_lists(ref_d, ref_n, dists, nns) == 0
