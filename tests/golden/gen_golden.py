#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE implementation itself.

Run in the development container (the reference is mounted read-only at
/root/reference; it never travels to the GPU box):

    python tests/golden/gen_golden.py

What is run: the reference's own `li.LearnedIndex.LearnedIndex.search` /
`search_single` and `li.model.NeuralNetwork.predict_proba` / `predict`
(search/li/*.py), on seeded synthetic inputs, with DataFrames built exactly as
search/search.py:71-93 builds them (index += 1).  Environment shims, all
outside the computation:
  * `faiss` and `h5py` are imported at module top by LearnedIndex.py:5 and
    utils.py:6 but unused on the search path; they are absent here, so empty
    placeholder modules satisfy the import (any attribute access would raise).
  * numpy 2 returns a tuple from np.ogrid[...]; LearnedIndex.py:94-95 assigns
    into it (numpy<2 returned a list), so np.ogrid is wrapped to return a list.
  * search/li is a namespace package; it is registered as a plain package
    object over the same directory because torch's lazy imports reject
    namespace modules in sys.modules.
  * NPY_DISABLE_CPU_FEATURES selects numpy's pre-x86-simd-sort quicksort so
    ties sort as in the reference era (py3.8 / numpy<=1.24, ci.yml:29).

Inputs are regenerated from seeds in the tests (numpy PCG64, tests/workloads.py)
and pinned by SHA-256; only small arrays (router weights, outputs) are stored.
"""
import hashlib
import os
import subprocess
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/search"
FEATURES = ("AVX2 FMA3 F16C AVX512F AVX512CD AVX512_KNL AVX512_KNM AVX512_SKX AVX512_CLX "
            "AVX512_CNL AVX512_ICL")

# (name, n, nq, C, R, k, label_mode, arch, seed, use_threshold)
SEARCH_CASES = [
    ("skew_r4", 3000, 200, 16, 4, 10, "skewed", "MLP", 101, True),
    ("skew_r7", 3000, 200, 16, 7, 10, "skewed", "MLP", 102, True),
    ("skew_r1", 3000, 200, 16, 1, 10, "skewed", "MLP", 103, True),
    ("skew_r2_k5", 2500, 150, 16, 2, 5, "skewed", "MLP", 104, True),
    ("skew_r3_k20", 2500, 150, 16, 3, 20, "skewed", "MLP", 105, True),
    ("skew_r4_nothr", 3000, 200, 16, 4, 10, "skewed", "MLP", 106, False),
    ("router_r4", 3000, 200, 16, 4, 10, "router", "MLP", 107, True),
    ("router_r8", 3000, 200, 16, 8, 10, "router", "MLP-5", 108, True),
    ("router_c8_r3", 2000, 300, 8, 3, 10, "router", "MLP", 109, True),
    ("skew_c32_r5", 3000, 250, 32, 5, 10, "skewed", "MLP-5", 110, True),
    ("tiny_r4", 400, 120, 16, 4, 10, "skewed", "MLP", 111, True),
    ("tiny_r6", 300, 100, 32, 6, 10, "skewed", "MLP", 112, True),
    ("dup_r4", 2000, 150, 16, 4, 10, "dup", "MLP", 113, True),
    ("c122_r4", 3000, 200, 122, 4, 10, "skewed", "MLP", 114, True),
    ("c122_r7", 3000, 200, 122, 7, 10, "router", "MLP-5", 115, True),
]
# search_single called directly (search.py:129-140 path and an explicit threshold)
SINGLE_CASES = [
    ("single_k10", 3000, 200, 16, 1, 10, "skewed", "MLP", 121, False),
    ("single_k7", 3000, 200, 16, 1, 7, "skewed", "MLP", 122, False),
    ("single_thr", 3000, 200, 16, 1, 10, "skewed", "MLP", 123, True),
]
ROUTER_CASES = [("MLP", 122, 201), ("MLP-5", 122, 202), ("MLP", 16, 203)]


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(a.tobytes())
    return h.hexdigest()


def _import_reference():
    import numpy as np
    import torch
    import torch.utils.data  # noqa: F401
    # the reference `li` is a namespace package; torch's lazy imports walk
    # sys.modules with inspect and choke on it, so finish them first
    try:
        import torch.distributed.tensor  # noqa: F401
    except Exception:
        pass
    sys.modules.setdefault("faiss", types.ModuleType("faiss"))
    sys.modules.setdefault("h5py", types.ModuleType("h5py"))

    class _OGrid:
        def __init__(self, g):
            self._g = g

        def __getitem__(self, key):
            return list(self._g[key])

    np.ogrid = _OGrid(np.ogrid)
    # this repo's package is also called `li`: keep the objects already bound
    # (tests/workloads.py holds li.synth) but resolve `li` to the reference now
    for m in [m for m in sys.modules if m == "li" or m.startswith("li.")]:
        del sys.modules[m]
    sys.path[:] = [p for p in sys.path if not p.endswith("sisap23-laion-challenge-learned-index_amd")]
    sys.path.insert(0, REF)
    # search/li has no __init__.py (a namespace package); torch's lazy imports
    # call inspect.getfile on every module and reject namespace modules, so
    # register `li` as a plain package object over the same directory
    pkg = types.ModuleType("li")
    pkg.__path__ = [os.path.join(REF, "li")]
    pkg.__file__ = os.path.join(REF, "li", "__init__.py")
    sys.modules["li"] = pkg
    from li.LearnedIndex import LearnedIndex  # noqa: E402
    from li.model import NeuralNetwork, data_X_to_torch  # noqa: E402
    return LearnedIndex, NeuralNetwork, data_X_to_torch


def _nn_with(NeuralNetwork, layers, arch, C):
    import torch
    nn = NeuralNetwork(input_dim=96, output_dim=C, lr=0.009, model_type=arch)
    lin = [m for m in nn.model.layers if isinstance(m, torch.nn.Linear)]
    assert len(lin) == len(layers)
    with torch.no_grad():
        for m, (w, b) in zip(lin, layers):
            m.weight.copy_(torch.from_numpy(w))
            m.bias.copy_(torch.from_numpy(b))
    return nn


def generate():
    import numpy as np
    import pandas as pd
    sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd")]
    import workloads
    from li import synth

    LearnedIndex, NeuralNetwork, data_X_to_torch = _import_reference()
    out = {}
    # ---- router (model.py:201-229) -------------------------------------
    for arch, C, seed in ROUTER_CASES:
        layers = synth.np_router_layers(synth.ARCHS[arch], C, seed)
        x, _ = synth.np_mixture(512, 768, 40, seed)
        xn = synth.np_nav(x, synth.np_projection(768, 96, seed + 1))
        nn = _nn_with(NeuralNetwork, layers, arch, C)
        probs, classes = nn.predict_proba(data_X_to_torch(xn))
        labels = nn.predict(data_X_to_torch(xn))
        key = f"router_{arch}_{C}"
        out[f"{key}__x"] = xn
        for i, (w, b) in enumerate(layers):
            out[f"{key}__W{i}"] = w
            out[f"{key}__b{i}"] = b
        out[f"{key}__probs"] = probs[:, :16].astype(np.float32)
        out[f"{key}__classes"] = classes[:, :16].astype(np.int16)
        out[f"{key}__predict"] = labels.astype(np.int16)
    # ---- search (LearnedIndex.py:22-195) -------------------------------
    for case in SEARCH_CASES + SINGLE_CASES:
        name, n, nq, C, R, k, mode, arch, seed, thr = case
        w = workloads.clustered(n=n, nq=nq, C=C, arch=arch, seed=seed, label_mode=mode)
        li = LearnedIndex()
        li.model = _nn_with(NeuralNetwork, w["layers"], arch, C)
        data = pd.DataFrame(w["xn"])
        data.index += 1                        # search.py:71-72
        data_search = pd.DataFrame(w["x"])
        data_search.index += 1                 # search.py:83-84
        _, classes = li.model.predict_proba(data_X_to_torch(w["qn"]))
        if case in SINGLE_CASES:
            data["category"] = w["labels"]     # search.py:133
            thr_arr = None
            if thr:
                rng = np.random.Generator(np.random.PCG64(seed + 9))
                thr_arr = rng.uniform(0.3, 0.9, nq)
                out[f"search_{name}__thr"] = thr_arr
            dists, anns = li.search_single(data, data_search, w["q"], classes[:, 0], k=k,
                                           threshold_dist=thr_arr)
        else:
            dists, anns = li.search(data, w["qn"], data_search, w["q"], w["labels"],
                                    n_buckets=R, k=k, use_threshold=thr)
        key = f"search_{name}"
        out[f"{key}__meta"] = np.array([n, nq, C, R, k, seed, int(thr)], np.int64)
        out[f"{key}__sha"] = np.array(sha(w["x"], w["q"], w["xn"], w["qn"], w["labels"]))
        out[f"{key}__classes"] = classes[:, : max(R, 1)].astype(np.int16)
        out[f"{key}__dists"] = np.asarray(dists, np.float64)
        out[f"{key}__anns"] = np.asarray(anns, np.uint32)
        print(f"{name}: dists {dists.shape} anns {anns.dtype}", file=sys.stderr)
    path = os.path.join(HERE, "reference_outputs.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)", file=sys.stderr)


if __name__ == "__main__":
    if os.environ.get("_LMI_GOLDEN_CHILD") != "1":
        env = dict(os.environ, _LMI_GOLDEN_CHILD="1", PYTHONDONTWRITEBYTECODE="1",
                   NPY_DISABLE_CPU_FEATURES=FEATURES, CUDA_VISIBLE_DEVICES="",
                   HIP_VISIBLE_DEVICES="")
        sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)], env=env))
    generate()
