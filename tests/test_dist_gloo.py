"""Multi-process (gloo, CPU) test of the multi-GPU protocol of li/dist.py:
corpus striped over the ranks (BucketLayout.shard), per-shard lists keyed by
global position, all_gather_into_tensor, merge by (distance, position) -- both
through gather_merge and through the product's packed exchange
(packed_lists + gather_merge_packed, the layout lmi_merge_topk_packed reads).  The
per-shard lists and the merge are computed by the oracle here (no HIP device);
on the GPU they are lmi_bucket_topk and lmi_merge_topk (tests/test_gpu_parity.py
checks that the GPU merge equals the single-shard result bitwise)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_lists(w, classes, R, k, C, gpos):
    """Oracle per-(q, r) top-k over this shard's rows, keyed by global position."""
    import lmi_oracle as O
    order, off = O.layout(w["labels"], C)
    nq = w["q"].shape[0]
    out_d = np.full((nq, R, k), np.inf, np.float32)
    out_p = np.full((nq, R, k), -1, np.int32)
    mine = np.zeros(off[-1], bool)
    mine[gpos] = True
    for r in range(R):
        for c in np.unique(classes[:, r]):
            pos = np.arange(off[c], off[c + 1])
            pos = pos[mine[pos]]
            if pos.size == 0:
                continue
            G = np.nonzero(classes[:, r] == c)[0]
            D = O.pairwise_cosine(w["q"][G], w["x"][order[pos]])
            for gi, q in enumerate(G):
                o = np.lexsort((pos, D[gi]))[:k]
                out_d[q, r, : o.size] = D[gi][o]
                out_p[q, r, : o.size] = pos[o]
    return out_d, out_p


def _oracle_merge(gd, gp, k):
    G, nq, R, _ = gd.shape
    d = gd.numpy().transpose(1, 2, 0, 3).reshape(nq, R, -1)
    p = gp.numpy().transpose(1, 2, 0, 3).reshape(nq, R, -1)
    key_p = np.where(p < 0, np.iinfo(np.int64).max, p)
    o = np.lexsort((key_p, d), axis=-1)[..., :k]
    return (torch.from_numpy(np.take_along_axis(d, o, -1)),
            torch.from_numpy(np.take_along_axis(p, o, -1)))


def _worker(rank, world, port, result_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "sisap23-laion-challenge-learned-index_amd"),
                    os.path.join(root, "oracle"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import lmi_oracle as O
    import workloads
    from li.dist import (gather_merge, gather_merge_packed, init_from_env, packed_lists,
                         route_sharded)
    from li.index import BucketLayout
    init_from_env(backend="gloo")
    w = workloads.clustered(n=2500, nq=80, C=16, seed=31, label_mode="skewed")
    R, k, C = 3, 10, 16
    nq = w["q"].shape[0]
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :R]
    gpos, _ = BucketLayout.from_labels(w["labels"], C).shard(rank, world)
    d, p = _shard_lists(w, classes, R, k, C, gpos)
    md, mp_ = gather_merge(torch.from_numpy(d), torch.from_numpy(p), k, merge=_oracle_merge)
    # the product's packed exchange (Searcher._scan at G > 1): the lists and the
    # status word written into this rank's send buffer (packed_lists), one
    # all-gather, the gathered buffer unpacked in lmi_merge_topk_packed's layout
    packed_ok = True
    for f64 in (False, True):
        buf, dv, pv, sv = packed_lists(nq * R, k, f64, "cpu")
        dv.copy_(torch.from_numpy(d.astype(np.float64 if f64 else np.float32)).view(-1))
        pv.copy_(torch.from_numpy(p).view(-1))
        sv.fill_(1 << rank)
        st_out = torch.zeros(1, dtype=torch.int32)
        pd_, pp_, pst = gather_merge_packed(buf, nq * R, k, f64, status_out=st_out,
                                            merge=lambda gd, gp, kk: _oracle_merge(
                                                gd.view(-1, nq, R, kk), gp.view(-1, nq, R, kk), kk))
        packed_ok = packed_ok and np.array_equal(pd_.numpy().astype(np.float32).reshape(nq, R, k),
                                                 md.numpy()) and \
            np.array_equal(pp_.numpy().reshape(nq, R, k), mp_.numpy()) and \
            int(st_out[0]) == (1 << world) - 1 and pst is st_out
    # float64 lists (lmi_bucket_topk_f64) through the same collective, with
    # every rank's status word OR-ed into the result on every rank
    md64, mp64, st = gather_merge(torch.from_numpy(d.astype(np.float64)), torch.from_numpy(p), k,
                                  merge=_oracle_merge,
                                  status=torch.tensor([1 << rank], dtype=torch.int32))
    f64_ok = md64.dtype == torch.float64 and \
        np.array_equal(md64.numpy().astype(np.float32), md.numpy()) and \
        np.array_equal(mp64.numpy(), mp_.numpy()) and int(st[0]) == (1 << world) - 1

    class _OracleRouter:  # K1's contract on the CPU: per-query top-R classes
        def topr(self, x, R):
            c = O.rank_classes(O.mlp_forward(x.numpy(), w["layers"]))[:, :R]
            return torch.from_numpy(np.ascontiguousarray(c, dtype=np.int32)), None

    routed = route_sharded(_OracleRouter(), torch.from_numpy(w["qn"]), R).numpy()
    if rank == 0:
        fd, fp = O.bucket_lists(w["labels"], w["x"], w["q"], classes, R, k, C)
        # BLAS results depend on the matrix shape at the ulp level, so the
        # oracle is compared with the tie-aware comparator (the GPU scan is
        # shape-independent and is checked bitwise in test_gpu_parity.py)
        ok = O.compare_lists(fd, fp, md.numpy(), mp_.numpy()) == 0 and \
            np.array_equal(np.isfinite(md.numpy()), np.isfinite(fd)) and \
            np.array_equal(routed, classes) and f64_ok and packed_ok
        with open(result_path, "w") as f:
            f.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_striped_search_equals_single_shard(world, tmp_path):
    res = tmp_path / "result.txt"
    mp.spawn(_worker, args=(world, _free_port(), str(res)), nprocs=world, join=True)
    assert res.read_text() == "ok"
