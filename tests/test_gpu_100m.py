"""BASELINE configs[4] (100M random clip768-shaped rows, 8 GPUs) exercised on
one MI355X: the one-GPU index (154 GB of fp16 in HBM, generated chunk by chunk
straight into its bucket-sorted slots, li.index.RowSource) gives the reference
lists; then the eight stripes of the 8-GPU layout are built one at a time
(19 GB each, beside it), each scanned into its packed all-gather buffer, and
K3 merges the concatenated buffers as the all-gather leaves them: bitwise the
one-GPU lists, in both arithmetics, and the device replay over them bitwise
the one-GPU answer.  The lists of sampled queries are also checked against a
float64 brute force over the same bucket rows."""
import numpy as np
import pytest
import torch

from li import synth
from li.index import DeviceIndex, DeviceRouter, bucket_topk, bucket_topk_f64, replay_device
from test_gpu_fullsize import _packed_shards

pytestmark = pytest.mark.gpu
N = 100_000_000


@pytest.fixture(scope="module")
def w100m():
    free, total = torch.cuda.mem_get_info()
    if free < 200 * (1 << 30):
        pytest.skip(f"needs ~200 GB of free HBM ({free >> 30} GB free)")
    dev = torch.device("cuda")
    src, q, qn, layers, labels = synth.build_random_workload(N, 10_000, 122, "MLP-5", dev)
    router = DeviceRouter(layers, device=dev)
    ix = DeviceIndex(src, labels, 122, chunk_rows=8192, device=dev)
    w = dict(src=src, q=q, qn=qn, labels=labels, router=router, ix=ix)
    yield w
    w.clear()
    torch.cuda.empty_cache()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dist", ["f32", "f64"])
def test_configs4_eight_shards_equal_one_gpu(w100m, dist):
    w = w100m
    ix = w["ix"]
    R, k = 4, 10
    f64 = dist == "f64"
    classes = w["router"].topr(w["qn"], R)[0]
    scan = bucket_topk_f64 if f64 else bucket_topk
    d1, p1, st1 = scan(ix, w["q"], classes, k)
    assert int(st1.item()) == 0
    md, mp, st = _packed_shards(w["src"], w["labels"], w["q"], classes, k, f64, 8, 2048)
    assert st == 0
    assert torch.equal(md, d1) and torch.equal(mp, p1)
    bsz = torch.from_numpy(np.ascontiguousarray(ix.bucket_size, dtype=np.int64)).cuda()
    p2id = torch.from_numpy(np.ascontiguousarray(ix.pos_to_id, dtype=np.int64)).cuda()
    a1 = replay_device(classes, d1, p1, k_round=10, k_final=k, bucket_size=bsz, pos_to_id=p2id,
                       use_threshold=True)
    a8 = replay_device(classes, md, mp, k_round=10, k_final=k, bucket_size=bsz, pos_to_id=p2id,
                       use_threshold=True)
    assert int(a1[2].item()) == 0 and int(a8[2].item()) == 0
    assert torch.equal(a1[0], a8[0]) and torch.equal(a1[1], a8[1])


@pytest.mark.timeout(600)
def test_configs4_lists_match_brute_force(w100m):
    """32 sampled queries' lists (float32 and float64) vs bench.list_parity's
    float64 brute force over the same bucket rows of the one-GPU index."""
    import bench
    w = w100m
    ix = w["ix"]
    classes = w["router"].topr(w["qn"], 4)[0]
    for f64 in (False, True):
        scan = bucket_topk_f64 if f64 else bucket_topk
        d, p, st = scan(ix, w["q"], classes, 10)
        res = bench.list_parity(ix, None, w["q"], classes.cpu().numpy(), d, p, 32, f64)
        assert res["checked_lists"] == 128 and res["mismatches"] == 0, res
