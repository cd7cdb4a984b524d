"""One rank of tests/test_gpu_dist.py: the PRODUCT multi-GPU path
(Searcher.search: route_sharded, K2 into the packed send buffer,
gather_merge_packed -> lmi_merge_topk_packed, device replay) with
torch.distributed over gloo, two ranks sharing the box's one GPU (RCCL refuses
two ranks on one device; gloo stages the collectives through host memory).
Rank 0 writes the answers to the .npz named on the command line."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"),
                os.path.join(ROOT, "oracle"), HERE]


N_BATCHES = 7


def main(out_path):
    import numpy as np
    import torch
    import torch.distributed as dist

    import workloads
    from li.dist import init_from_env
    from li.index import DeviceIndex, DeviceRouter, Searcher
    rank, world, _ = init_from_env(backend="gloo")
    torch.cuda.set_device(0)
    w = workloads.clustered(n=8000, nq=240, C=16, seed=61, label_mode="skewed")
    ix = DeviceIndex(w["x"], w["labels"], w["C"], chunk_rows=512, device="cuda:0", rank=rank,
                     world=world)
    s = Searcher(ix, DeviceRouter(w["layers"], device="cuda:0"))
    qn = torch.from_numpy(w["qn"]).cuda()
    q = torch.from_numpy(w["q"]).cuda()
    res = {}
    for dist_ in ("f32", "f64"):
        for R in (1, 4):
            d, a = s.search(qn, q, R, k=10, dist=dist_)
            res[f"{dist_}_R{R}_d"], res[f"{dist_}_R{R}_a"] = d, a
        _, ld, lp, st = s.lists(qn, q, 4, 10, dist=dist_)
        res[f"{dist_}_lists_d"], res[f"{dist_}_lists_p"] = ld.cpu().numpy(), lp.cpu().numpy()
        res[f"{dist_}_lists_st"] = np.array([int(st.item())])
    d, a = s.search(qn, q, 4, k=10, semantics="exact")
    res["exact_d"], res["exact_a"] = d, a
    # the graphed step's G > 1 path (each rank uploads its block, routes it,
    # one all-gather of queries + classes), run eagerly: gloo cannot be
    # captured; RCCL runs the same step as a graph on the 8-GPU node
    for dist_ in ("f32", "f64"):
        g = s.graph(w["qn"], w["q"], 4, k=10, dist=dist_, capture=False)
        d, a = g.run()
        res[f"graph_{dist_}_d"], res[f"graph_{dist_}_a"] = d.copy(), a.copy()
    # repeated graph steps on new staged batches (the sharded upload + one
    # all-gather of queries and classes per step)
    perms = [np.random.default_rng(70 + i).permutation(w["q"].shape[0]) for i in range(N_BATCHES)]
    batches = [(w["qn"][p], w["q"][p]) for p in perms]
    for dist_ in ("f32", "f64"):
        g = s.graph(w["qn"], w["q"], 4, k=10, dist=dist_, capture=False)
        for i, b in enumerate(batches[:3]):
            d, a = g.run(*b)
            res[f"graphrun_{dist_}_{i}_d"], res[f"graphrun_{dist_}_{i}_a"] = d.copy(), a.copy()
    # the batch stream's G > 1 path (each rank stages and uploads its block of
    # the batch and routes it; one all-gather per launch carries the lists of
    # one batch with the blocks of the next), its stages launched eagerly over
    # gloo: N_BATCHES distinct batches, so StreamedSearch.step() itself runs
    # (N_BATCHES - 3 launches after the fill) before the drain
    for dist_ in ("f32", "f64"):
        st = s.streamed(w["qn"], w["q"], 4, k=10, dist=dist_, capture=False)
        for i, (d, a) in enumerate(st.stream(batches)):
            res[f"stream_{dist_}_{i}_d"], res[f"stream_{dist_}_{i}_a"] = d, a
        res[f"stream_{dist_}_launches"] = np.array([st.launches])
    # the bench's use: stage() + step() per launch, a new batch each time,
    # one batch not fp16-exact (answered by Searcher.search on every rank)
    st = s.streamed(w["qn"], w["q"], 4, k=10, capture=False)
    odd = (batches[1][0], batches[1][1] + np.float32(1e-5))
    seq = [batches[i % 4] for i in range(7)]
    seq[5] = odd
    for i, (d, a) in enumerate(st.stream(seq)):
        res[f"stream_odd_{i}_d"], res[f"stream_odd_{i}_a"] = d, a
    if rank == 0:
        np.savez(out_path, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
