"""GPU drop-in vs the reference's own outputs on float64 INPUTS
(tests/golden/reference_outputs_r3.npz): float64 data_search and/or queries,
where sklearn computes on the float64 values (utils.py:11, :19).  The drop-in
keeps the float64 rows (DeviceIndex.corpus64) and queries for the float64
recomputation (lmi_bucket_topk_f64q); the inputs differ from their float32
rounding by less than half a float32 ulp, so a path that computes on the
rounded values flips ids (test_oracle_golden_r3.py shows the fixtures are
sharp).  Ids must match up to float64 ties (1e-12), distances to 1e-12."""
import numpy as np
import pandas as pd
import pytest
import torch

import lmi_oracle as O
import workloads
from test_gpu_golden_r2 import _nn
from test_oracle_golden_r3 import BASES, CASES, G3, SINGLES, TIE64, check, inputs_r3

pytestmark = pytest.mark.gpu


def _frames(w, x):
    data = pd.DataFrame(w["xn"])
    data.index += 1
    data_search = pd.DataFrame(x)
    data_search.index += 1
    return data, data_search


@pytest.mark.parametrize("name", list(CASES))
def test_f64_input_search_matches_reference(name):
    from li.LearnedIndex import LearnedIndex, dist_dtype
    _, n, nq, C, R, k, mode, arch, seed, thr, fd, fq = CASES[name]
    w, x, q = inputs_r3(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    data, data_search = _frames(w, x)
    assert dist_dtype(data_search, q) == "f64"
    dists, anns = li.search(data, w["qn"], data_search, q, w["labels"], n_buckets=R, k=k,
                            use_threshold=thr)
    assert dists.dtype == np.float64 and anns.dtype == np.uint32
    assert (li._index.corpus64 is not None) == fd
    check(name, dists, anns)


@pytest.mark.parametrize("name", list(SINGLES))
def test_f64_input_search_single_matches_reference(name):
    from li.LearnedIndex import LearnedIndex
    _, n, nq, C, R, k, mode, arch, seed = SINGLES[name]
    w, x, q = inputs_r3(name)
    li = LearnedIndex()
    li.model = _nn(w["layers"], arch, C)
    data, data_search = _frames(w, x)
    data["category"] = w["labels"]
    classes = G3[f"search_{name}__classes"].astype(np.int64)
    dists, anns = li.search_single(data, data_search, q, classes[:, 0], k=k)
    assert dists.shape == (nq, k)
    check(name, dists, anns)


@pytest.mark.parametrize("name", list(BASES))
def test_f64_input_baseline_matches_reference(name):
    from li.Baseline import Baseline
    _, n, nq, k, mode, seed = BASES[name]
    w = workloads.clustered(n=n, nq=nq, C=16, seed=seed, label_mode=mode)
    x64, q64 = workloads.float64_inputs(w, seed)
    dists, nns, _ = Baseline().search(q64, x64, k=k)
    ref_d, ref_n = G3[f"base_{name}__dists"], G3[f"base_{name}__nns"]
    assert dists.dtype == ref_d.dtype and dists.shape == ref_d.shape
    assert O.compare_lists(ref_d, ref_n, dists, nns, atol=1e-12, tie=TIE64) == 0


def test_f64_input_lists_match_oracle_and_rounded_path_differs():
    """K2's float64 lists on float64 rows + queries equal the oracle's
    float64 lists; the same call on the float32-rounded inputs does not."""
    from li.index import DeviceIndex, bucket_topk_f64
    w = workloads.clustered(n=4000, nq=160, C=16, seed=451, label_mode="dup")
    x64, q64 = workloads.float64_inputs(w, 451)
    R = 4
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    cls = torch.from_numpy(np.ascontiguousarray(classes, dtype=np.int32)).cuda()
    ix = DeviceIndex(x64, w["labels"], 16, device="cuda", chunk_rows=256)
    assert ix.corpus64 is not None    # (the rounded rows are fp16-exact here: an fp16 scan)
    d, pos, st = bucket_topk_f64(ix, torch.from_numpy(q64).cuda(), cls, 10)
    assert int(st.item()) == 0
    ref_d, ref_p = O.bucket_lists(w["labels"], x64, q64, classes, R, 10, 16)
    assert O.compare_lists(ref_d, ref_p, d.cpu().numpy(), pos.cpu().numpy(), atol=1e-12,
                           tie=TIE64) == 0
    ix32 = DeviceIndex(w["x"], w["labels"], 16, device="cuda", chunk_rows=256)
    d2, pos2, _ = bucket_topk_f64(ix32, torch.from_numpy(w["q"]).cuda(), cls, 10)
    assert O.compare_lists(ref_d, ref_p, d2.cpu().numpy(), pos2.cpu().numpy(), atol=1e-12,
                           tie=TIE64) > 0
