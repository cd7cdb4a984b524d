"""The product multi-GPU path run by two processes on the box's GPU
(torch.distributed over gloo; tests/dist_gpu_worker.py), against one process:
bitwise equal answers (reference semantics R = 1 and 4, exact semantics) and
bitwise equal merged per-(query, probe) lists, in both arithmetics.  This is
the striped index + route_sharded + packed K2 buffers + all-gather +
lmi_merge_topk_packed + device replay, as Searcher.search runs them at G > 1
(the 8-GPU bench uses RCCL for the same collectives)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import dist_gpu_worker
import workloads
from li.index import DeviceIndex, DeviceRouter, Searcher

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_two_process_product_path_equals_one_process(world, tmp_path):
    out = tmp_path / "rank0.npz"
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LMI_DIST_TIMEOUT_S="120")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_gpu_worker.py"),
                                       str(out)], env=env))
    rcs = [p.wait(timeout=240) for p in procs]
    assert rcs == [0] * world, rcs
    got = np.load(out)
    w = workloads.clustered(n=8000, nq=240, C=16, seed=61, label_mode="skewed")
    s = Searcher(DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda"),
                 DeviceRouter(w["layers"], device="cuda"))
    qn = torch.from_numpy(w["qn"]).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    for dist_ in ("f32", "f64"):
        for R in (1, 4):
            d, a = s.search(qn, q, R, k=10, dist=dist_)
            np.testing.assert_array_equal(got[f"{dist_}_R{R}_d"], d)
            np.testing.assert_array_equal(got[f"{dist_}_R{R}_a"], a)
        _, ld, lp, st = s.lists(qn, q, 4, 10, dist=dist_)
        np.testing.assert_array_equal(got[f"{dist_}_lists_d"], ld.cpu().numpy())
        np.testing.assert_array_equal(got[f"{dist_}_lists_p"], lp.cpu().numpy())
        assert int(got[f"{dist_}_lists_st"][0]) == 0 == int(st.item())
    d, a = s.search(qn, q, 4, k=10, semantics="exact")
    np.testing.assert_array_equal(got["exact_d"], d)
    np.testing.assert_array_equal(got["exact_a"], a)
    for dist_ in ("f32", "f64"):
        d, a = s.graph(w["qn"], w["q"], 4, k=10, dist=dist_).run()
        np.testing.assert_array_equal(got[f"graph_{dist_}_d"], d)
        np.testing.assert_array_equal(got[f"graph_{dist_}_a"], a)
    perms = [np.random.default_rng(70 + i).permutation(w["q"].shape[0])
             for i in range(dist_gpu_worker.N_BATCHES)]
    batches = [(w["qn"][p], w["q"][p]) for p in perms]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    for dist_ in ("f32", "f64"):
        ref = [s.search(T(a), T(b), 4, k=10, dist=dist_) for a, b in batches]
        for i in range(3):
            np.testing.assert_array_equal(got[f"graphrun_{dist_}_{i}_d"], ref[i][0])
            np.testing.assert_array_equal(got[f"graphrun_{dist_}_{i}_a"], ref[i][1])
        for i, (d, a) in enumerate(ref):
            np.testing.assert_array_equal(got[f"stream_{dist_}_{i}_d"], d)
            np.testing.assert_array_equal(got[f"stream_{dist_}_{i}_a"], a)
        # step() itself ran: one launch per batch after the three that fill
        assert int(got[f"stream_{dist_}_launches"][0]) == dist_gpu_worker.N_BATCHES - 3
    seq = [batches[i % 4] for i in range(7)]
    seq[5] = (batches[1][0], batches[1][1] + np.float32(1e-5))
    for i, (a_, b_) in enumerate(seq):
        d, a = s.search(T(a_), T(b_), 4, k=10)
        np.testing.assert_array_equal(got[f"stream_odd_{i}_d"], d)
        np.testing.assert_array_equal(got[f"stream_odd_{i}_a"], a)
