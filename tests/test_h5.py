"""Row f2: the HDF5 files around the hot path, on the native
libhdf5 shim liblmi_h5.so (include/lmi_h5.h; h5py is absent from this image).
The result layout is the one the reference's store_results writes
(utils.py:85-97) and eval/ reads; checked with the image's h5dump where present."""
import os
import re
import shutil
import subprocess

import numpy as np
import pandas as pd
import pytest

from li import h5
from li.utils import store_results

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H5DUMP = shutil.which("h5dump") or ("/opt/conda/bin/h5dump" if os.path.exists("/opt/conda/bin/h5dump") else None)


def test_library_exports_every_header_symbol():
    lib = h5.load()
    hdr = open(os.path.join(ROOT, "include", "lmi_h5.h")).read()
    declared = set(re.findall(r"^\w[\w\s\*]*?\b(lmi_h5_\w+)\(", hdr, flags=re.M))
    assert declared == set(h5.EXPORTS)
    for name in declared:
        assert getattr(lib, name) is not None


def test_store_results_layout(tmp_path):
    rng = np.random.default_rng(3)
    anns = rng.integers(1, 10**7, (50, 10)).astype(np.uint32)
    dists = np.sort(rng.random((50, 10)), axis=1)
    dst = tmp_path / "result" / "pca96v2" / "10M" / "learned-index-x.h5"
    store_results(str(dst), "Learned-index", "pca96v2", dists, anns, 12.5, 0.75, "learned-index-x", "10M")
    assert h5.dataset_info(str(dst), "knns") == ((50, 10), h5.U32)
    assert h5.dataset_info(str(dst), "dists") == ((50, 10), h5.F64)
    np.testing.assert_array_equal(h5.read_dataset(str(dst), "dists"), dists)
    if H5DUMP:
        out = subprocess.run([H5DUMP, "-A", str(dst)], capture_output=True, text=True, check=True).stdout
        for key, val in (("algo", "Learned-index"), ("data", "pca96v2"), ("size", "10M"),
                         ("params", "learned-index-x")):
            blk = out[out.index(f'ATTRIBUTE "{key}"'):]
            assert "H5T_VARIABLE" in blk[:300] and "H5T_CSET_UTF8" in blk[:300]
            assert f'"{val}"' in blk[:400]
        for key, val in (("buildtime", "12.5"), ("querytime", "0.75")):
            blk = out[out.index(f'ATTRIBUTE "{key}"'):]
            assert "H5T_IEEE_F64LE" in blk[:200] and f"(0): {val}" in blk[:200]
        full = subprocess.run([H5DUMP, "-d", "knns", str(dst)], capture_output=True, text=True,
                              check=True).stdout
        assert "H5T_STD_U32LE" in full and str(int(anns[0, 0])) in full


def test_dataset_roundtrip_fp16_and_f32(tmp_path):
    rng = np.random.default_rng(4)
    emb = rng.standard_normal((300, 768)).astype(np.float16).astype(np.float32)
    pca = rng.standard_normal((300, 96)).astype(np.float32)
    p = str(tmp_path / "dataset.h5")
    h5.write_dataset(p, "emb", emb, fp16=True)
    h5.write_dataset(p, "pca96", pca, fp16=False, append=True)
    assert h5.dataset_info(p, "emb") == ((300, 768), h5.F16)
    assert h5.dataset_info(p, "pca96") == ((300, 96), h5.F32)
    got = h5.read_dataset(p, "emb")                  # stored type, as np.array(h5py...)
    assert got.dtype == np.float16
    np.testing.assert_array_equal(got, emb.astype(np.float16))
    got = h5.read_dataset(p, "emb", dtype=np.float32)  # fp16 -> f32 through HDF5, exact
    assert got.dtype == np.float32
    np.testing.assert_array_equal(got, emb)
    np.testing.assert_array_equal(h5.read_dataset(p, "emb", 10, 5), emb[10:15].astype(np.float16))
    np.testing.assert_array_equal(h5.read_dataset(p, "pca96", 100, 50), pca[100:150])
    assert h5.read_dataset(p, "pca96").dtype == np.float32
    # a float16 array is stored as it is (no conversion), same file layout
    p2 = str(tmp_path / "stored.h5")
    h5.write_dataset(p2, "emb", emb.astype(np.float16), fp16=True)
    assert h5.dataset_info(p2, "emb") == ((300, 768), h5.F16)
    np.testing.assert_array_equal(h5.read_dataset(p2, "emb"), emb.astype(np.float16))
    np.testing.assert_array_equal(h5.read_dataset(p2, "emb", dtype=np.float32), emb)
    with pytest.raises(OSError, match="no dataset"):
        h5.read_dataset(p, "missing")
    with pytest.raises(OSError, match="past"):
        h5.read_dataset(p, "emb", 290, 20)


@pytest.mark.gpu
def test_cli_reads_h5_and_writes_eval_results(tmp_path, monkeypatch):
    """search.py's flow on reference-layout data/ files: pca96 navigation
    (dataset/query 'pca96') + clip768v2 'emb' (fp16) search data."""
    import sys
    import workloads
    sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
    import search as cli
    w = workloads.clustered(n=3000, nq=100, C=16, seed=41, label_mode="router")
    monkeypatch.chdir(tmp_path)
    for kind, key, data, q, fp16 in (("pca96v2", "pca96", w["xn"], w["qn"], False),
                                     ("clip768v2", "emb", w["x"], w["q"], True)):
        os.makedirs(f"data/{kind}/100K")
        h5.write_dataset(f"data/{kind}/100K/dataset.h5", key, data, fp16=fp16)
        h5.write_dataset(f"data/{kind}/100K/query.h5", key, q, fp16=fp16)
    cli.run("pca96v2", "pca96", "100K", 10, "learned-index", [25], 16, 5, "MLP", 0.01,
            preprocess=True)
    res = tmp_path / "result" / "pca96v2" / "100K"
    files = list(res.glob("learned-index-pca96v2-100K-*-buck=4.h5"))
    assert len(files) == 1
    assert h5.dataset_info(str(files[0]), "knns") == ((100, 10), h5.U32)
    assert h5.dataset_info(str(files[0]), "dists") == ((100, 10), h5.F64)
    d = h5.read_dataset(str(files[0]), "dists")
    assert np.all(np.diff(d, axis=1) >= 0)


@pytest.mark.gpu
@pytest.mark.parametrize("semantics", ["reference", "exact"])
def test_cli_synthetic_build_and_search(tmp_path, monkeypatch, semantics):
    """search.py --synthetic flow end to end on the GPU: K5 k-means build
    (LearnedIndex.cluster), router training, K1 labels, search at two bucket
    percentages (R = 1 via search_single, R > 1 via search), eval-layout H5."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
    import search as cli
    monkeypatch.chdir(tmp_path)
    # -bp 7 25 with 16 categories: R = int(1.12) = 1 and int(4.0) = 4 (search.py:37-38)
    cli.run("pca96v2", "pca96", "100K", 10, "learned-index", [7, 25], 16, 3, "MLP", 0.01,
            preprocess=True, synthetic=3000, semantics=semantics)
    res = tmp_path / "result" / "pca96v2" / "100K"
    files = sorted(p.name for p in res.glob("*.h5"))
    assert len(files) == 2 and any("buck=4" in f for f in files) and any("buck=1" in f for f in files)
    for f in files:
        assert h5.dataset_info(str(res / f), "knns") == ((10_000, 10), h5.U32)
        d = h5.read_dataset(str(res / f), "dists")
        if "buck=4" in f:  # merged rounds are a stable sort; a search_single row need not be
            assert np.all(np.diff(d, axis=1) >= 0)  # (its <k quirk writes 10000 mid-row)


def test_result_knns_read_back_in_their_stored_type(tmp_path):
    anns = np.arange(60, dtype=np.uint32).reshape(6, 10) * 7
    dists = np.sort(np.random.default_rng(1).random((6, 10)), axis=1)
    dst = tmp_path / "r.h5"
    store_results(str(dst), "Learned-index", "pca96v2", dists, anns, 1.0, 0.5, "x", "10M")
    got = h5.read_dataset(str(dst), "knns")
    assert got.dtype == np.uint32
    np.testing.assert_array_equal(got, anns)
