"""One process of tests/test_gpu_rccl.py: a ONE-RANK RCCL process group
(backend nccl) with LMI_FORCE_EXCHANGE=1, so every step form takes its G > 1
branch -- K2 into the packed send buffer, the all-gather (RCCL, captured in
the graphs), lmi_merge_topk_packed, the sharded router's block exchange --
and each answer is compared bit for bit with a Searcher that does not
exchange.  Exits 0 and prints the checks when every comparison holds."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"),
                os.path.join(ROOT, "oracle"), HERE]


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import workloads
    from li.dist import init_from_env
    from li.index import DeviceIndex, DeviceRouter, Searcher
    os.environ["LMI_FORCE_EXCHANGE"] = "1"
    rank, world, _ = init_from_env()
    assert dist.is_initialized() and dist.get_backend() == "nccl" and world == 1
    w = workloads.clustered(n=8000, nq=240, C=16, seed=61, label_mode="skewed")
    ix = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda:0")
    router = DeviceRouter(w["layers"], device="cuda:0")
    sx = Searcher(ix, router)                    # exchange: forced
    s0 = Searcher(ix, router, exchange=False)    # the plain one-GPU path
    assert sx.exchange and not s0.exchange
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    qn, q = T(w["qn"]), T(w["q"])
    eq = np.testing.assert_array_equal
    checks = []
    for dd in ("f32", "f64"):
        for R in (1, 4):
            eq(sx.search(qn, q, R, k=10, dist=dd), s0.search(qn, q, R, k=10, dist=dd))
        _, ld, lp, st = sx.lists(qn, q, 4, 10, dist=dd)
        _, ld0, lp0, st0 = s0.lists(qn, q, 4, 10, dist=dd)
        assert torch.equal(ld, ld0) and torch.equal(lp, lp0) and int(st.item()) == int(st0.item()) == 0
        checks.append(f"search/lists {dd}")
    eq(sx.search(qn, q, 4, k=10, semantics="exact"), s0.search(qn, q, 4, k=10, semantics="exact"))
    perms = [np.random.default_rng(80 + i).permutation(w["q"].shape[0]) for i in range(7)]
    batches = [(w["qn"][p], w["q"][p]) for p in perms]
    for dd in ("f32", "f64"):
        ref = [s0.search(T(a), T(b), 4, k=10, dist=dd) for a, b in batches]
        # the per-batch step graph: upload, route, the all-gather of the
        # blocks, scan, the all-gather of the packed lists + K3, replay
        g = sx.graph(w["qn"], w["q"], 4, k=10, dist=dd)
        assert g.X and g.G == 1 and g.graph is not None
        for (a, b), r in zip(batches[:3], ref):
            eq(g.run(a, b), r)
        g.close()
        gp = sx.graph(w["qn"], w["q"], 4, k=10, dist=dd, pipeline=True)
        for o, r in zip(gp.stream(batches), ref):
            eq(o, r)
        gp.close()
        # the batch stream: F1 (merge phase + the captured all-gather), F2
        # (lmi_merge_topk_packed + replay + D2H)
        ss = sx.streamed(w["qn"], w["q"], 4, k=10, dist=dd)
        assert ss.X and ss.xall is not None and all((n, 0) in ss.graphs for n in ("F1", "FX", "F2"))
        got = list(ss.stream(batches))
        assert len(got) == len(batches) and ss.launches == len(batches) - 3
        for o, r in zip(got, ref):
            eq(o, r)
        ss.close()
        # step() per launch on one staged batch, the bench's use (a new
        # object: after stream() the slots hold the stream's last batches)
        r0 = s0.search(qn, q, 4, k=10, dist=dd)
        ss = sx.streamed(w["qn"], w["q"], 4, k=10, dist=dd)
        for _ in range(5):
            eq(ss.step(), r0)
        assert ss.launches == 5
        ss.close()
        checks.append(f"graph/pipelined graph/stream {dd}")
    dist.barrier()
    dist.destroy_process_group()
    print("RCCL forced exchange OK: " + "; ".join(checks))


if __name__ == "__main__":
    main()
