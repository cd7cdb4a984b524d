"""Index artefacts: the reference's pickled LearnedIndex -> this build.

The reference persists a built index as a plain pickle of the whole
`LearnedIndex` object (search.py:107-113 -> utils.py:46-60 `save_as_pickle`):
`LearnedIndex.model` is a `NeuralNetwork` (model.py:114-147) holding the torch
`Model` (its `layers` Sequential of Linear/ReLU), the loss and the Adam
optimiser.  It stores no object labels and has no loader: search.py recomputes
nothing from it.  `load_index` reads such a file into this package's drop-in
classes (same module paths `li.LearnedIndex` / `li.model`, same attributes), so
`index.search(...)` runs the MI355X path on the reference-trained router, and
`object_labels` gives the bucket of every corpus row exactly as the build does
(LearnedIndex.py:240: `nn.predict(data_X_to_torch(data))`, K1 ARGMAX).

The unpickler resolves only an allow-list of globals: the reference's `li.*`
classes (mapped onto this package), torch's tensor/parameter rebuild helpers,
the exact torch classes such an index holds (Linear, ReLU, Sequential,
CrossEntropyLoss, Adam) and a few builtins/collections.
Tensor storages embedded by plain pickle are decoded with
`torch.load(..., weights_only=True)`.  Anything else raises
`pickle.UnpicklingError`.
"""
from __future__ import annotations

import collections
import io
import pickle
from typing import Optional

import numpy as np
import torch

_LI_CLASSES = {
    ("li.LearnedIndex", "LearnedIndex"),
    ("li.model", "NeuralNetwork"),
    ("li.model", "Model"),
    ("li.model", "LIDataset"),
    ("li.Logger", "Logger"),
}
_TORCH_FUNCS = {
    ("torch._utils", "_rebuild_tensor_v2"),
    ("torch._utils", "_rebuild_tensor"),
    ("torch._utils", "_rebuild_parameter"),
    ("torch._utils", "_rebuild_parameter_with_state"),
    ("torch", "device"),
    ("torch", "Size"),
    ("torch", "float32"),
    ("torch", "float64"),
    ("torch", "int64"),
}
_BUILTINS = {
    ("collections", "OrderedDict"),
    ("collections", "defaultdict"),
    ("builtins", "set"),
    ("builtins", "frozenset"),
    ("builtins", "dict"),
    ("builtins", "list"),
    ("builtins", "tuple"),
}
# the torch classes a reference index pickles (model.py:18-83 Model layers,
# model.py:114-147 loss and optimiser): nothing else from torch.nn / torch.optim
_TORCH_CLASSES = {
    ("torch.nn.modules.linear", "Linear"),
    ("torch.nn.modules.activation", "ReLU"),
    ("torch.nn.modules.container", "Sequential"),
    ("torch.nn.modules.loss", "CrossEntropyLoss"),
    ("torch.optim.adam", "Adam"),
}


def _load_storage(b: bytes):
    # torch.storage._load_from_bytes, without executing anything from the file
    return torch.load(io.BytesIO(b), weights_only=True, map_location="cpu")


class _IndexUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _LI_CLASSES:
            import importlib
            return getattr(importlib.import_module(module), name)
        if (module, name) == ("torch.storage", "_load_from_bytes"):
            return _load_storage
        if (module, name) in _TORCH_FUNCS or (module, name) in _BUILTINS or \
                (module, name) in _TORCH_CLASSES:
            return super().find_class(module, name)
        if module == "torch" and name.endswith("Storage"):
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"index pickle: global {module}.{name} is not allowed")


def load_index(path: str):
    """A reference-pickled `LearnedIndex` (utils.py:46-60) as this package's
    `li.LearnedIndex.LearnedIndex`, its router weights moved to this host's
    device.  Raises pickle.UnpicklingError on globals outside the allow-list."""
    from .LearnedIndex import LearnedIndex
    from .model import get_device
    with open(path, "rb") as f:
        obj = _IndexUnpickler(f).load()
    if not isinstance(obj, LearnedIndex):
        raise TypeError(f"{path}: expected a pickled LearnedIndex, got {type(obj).__name__}")
    nn = obj.model
    if nn is not None:
        nn.device = get_device()
        nn.model = nn.model.to(nn.device)
    return obj


def router_layers(index) -> list:
    """[(W [out, in] f32, b [out] f32), ...] of the index's router, in order."""
    seq = index.model.model.layers
    return [(m.weight.detach().cpu().numpy().astype(np.float32),
             m.bias.detach().cpu().numpy().astype(np.float32))
            for m in seq if isinstance(m, torch.nn.Linear)]


def object_labels(index, data_navigation) -> np.ndarray:
    """Bucket of every corpus row (LearnedIndex.py:240) on K1: int64 [n]."""
    from .model import data_X_to_torch
    x = data_navigation.drop("category", axis=1, errors="ignore") \
        if hasattr(data_navigation, "columns") else data_navigation
    return index.model.predict(data_X_to_torch(x))


def save_index(path: str, index) -> None:
    """The reference's own format (utils.py:46-60): a plain pickle of the
    LearnedIndex, minus this build's device-side caches."""
    state_i, state_n = index.__dict__.copy(), None
    for k in ("_cache_key", "_index"):
        index.__dict__.pop(k, None)
    if index.model is not None:
        state_n = index.model.__dict__.copy()
        for k in ("_router", "_router_version"):
            index.model.__dict__.pop(k, None)
    try:
        with open(path, "wb") as f:
            pickle.dump(index, f)
    finally:
        index.__dict__.update(state_i)
        if state_n is not None:
            index.model.__dict__.update(state_n)
