"""Row f1: the reference's pickled LearnedIndex loads into the
drop-in classes.  Fixture: tests/golden/ref_index_mlp16.pkl, written BY THE
REFERENCE (utils.py:46-60 save_as_pickle) with tests/golden/gen_pickle.py, and
the reference's own predict / search outputs on it."""
import os
import pickle

import numpy as np
import pandas as pd
import pytest
import torch

import lmi_oracle as O
import workloads
from golden.gen_pickle import CASE
from li import index_io

HERE = os.path.dirname(os.path.abspath(__file__))
PKL = os.path.join(HERE, "golden", "ref_index_mlp16.pkl")
OUT = np.load(os.path.join(HERE, "golden", "ref_index_mlp16_outputs.npz"))


def _w():
    return workloads.clustered(n=CASE["n"], nq=CASE["nq"], C=CASE["C"], arch=CASE["arch"],
                               seed=CASE["seed"], label_mode="router")


def test_reference_pickle_loads_into_dropin_classes():
    from li.LearnedIndex import LearnedIndex
    from li.model import NeuralNetwork
    ix = index_io.load_index(PKL)
    assert type(ix) is LearnedIndex and type(ix.model) is NeuralNetwork
    w = _w()
    layers = index_io.router_layers(ix)
    assert len(layers) == len(w["layers"])
    for (W, b), (W0, b0) in zip(layers, w["layers"]):
        assert np.array_equal(W, W0) and np.array_equal(b, b0)
    # the object labels the build would compute (LearnedIndex.py:240), on the oracle
    assert (O.predict(w["xn"], layers) == OUT["pred_categories"]).all()


def test_unpickler_refuses_other_globals(tmp_path):
    p = tmp_path / "evil.pkl"
    with open(p, "wb") as f:
        pickle.dump(os.system, f)
    with pytest.raises(pickle.UnpicklingError):
        index_io.load_index(str(p))


@pytest.mark.parametrize("obj", [torch.nn.Conv1d(2, 2, 1), torch.optim.lr_scheduler.partial(print),
                                 torch.nn.modules.linear.Identity()])
def test_unpickler_refuses_torch_names_outside_the_allow_list(tmp_path, obj):
    # any other torch.nn module, and names torch.optim re-exports (functools.partial)
    p = tmp_path / "other.pkl"
    with open(p, "wb") as f:
        pickle.dump(obj, f)
    with pytest.raises(pickle.UnpicklingError):
        index_io.load_index(str(p))


def test_save_roundtrip_keeps_reference_format(tmp_path):
    ix = index_io.load_index(PKL)
    ix._index = object()  # a device cache must not be written
    p = tmp_path / "again.pkl"
    index_io.save_index(str(p), ix)
    assert ix._index is not None
    ix2 = index_io.load_index(str(p))
    assert "_index" not in ix2.__dict__
    for (W, b), (W0, b0) in zip(index_io.router_layers(ix2), index_io.router_layers(ix)):
        assert np.array_equal(W, W0) and np.array_equal(b, b0)


@pytest.mark.gpu
def test_loaded_reference_index_searches_like_the_reference():
    ix = index_io.load_index(PKL)
    w = _w()
    data = pd.DataFrame(w["xn"])
    data.index += 1
    data_search = pd.DataFrame(w["x"])
    data_search.index += 1
    pred = index_io.object_labels(ix, data)
    assert (pred == OUT["pred_categories"]).all()
    dists, anns = ix.search(data, w["qn"], data_search, w["q"], pred, n_buckets=4, k=10,
                            use_threshold=True)
    assert O.compare_lists(OUT["dists"], OUT["anns"], dists, anns) == 0
