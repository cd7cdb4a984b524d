"""Per-rank step time of a W-GPU striped index, timed on ONE GPU: rank 0's shard,
a 1-process RCCL group (the all-gather moves only this rank's lists), full
Searcher.search (router + scan + K3 merge + device replay + D2H).  Estimates the
fixed per-step costs that do not shrink with W."""
import argparse, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import numpy as np, torch, torch.distributed as dist
from li import synth
from li.index import DeviceIndex, DeviceRouter, Searcher

ap = argparse.ArgumentParser()
ap.add_argument("--worlds", default="1,8")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--chunk", type=int, default=0, help="chunk rows (0: the bench default by world)")
ap.add_argument("--scale", default="10M", choices=["10M", "100M"],
                help="100M: configs[4] random vectors, generated per chunk into the shard (li.index.RowSource)")
a = ap.parse_args()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
dev = torch.device("cuda", 0)
if a.scale == "100M":
    x, q, qn, layers, labels = synth.build_random_workload(100_000_000, 10_000, 122, "MLP-5", dev)
    router = DeviceRouter(layers)
else:
    x, q, qn, xn, layers = synth.build_lmi_workload(10_000_000, 10_000, 122, "MLP-5", dev)
    router = DeviceRouter(layers)
    labels = router.argmax(xn); del xn
for W in map(int, a.worlds.split(",")):
    ck = a.chunk or (8192 if W == 1 else 4096 if W <= 4 else 2048)
    ix = DeviceIndex(x, labels, 122, chunk_rows=ck, rank=0, world=W)
    s = Searcher(ix, router)
    for _ in range(3):
        s.search(qn, q, 4, k=10)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(a.steps):
        s.search(qn, q, 4, k=10)
    torch.cuda.synchronize(); el = (time.perf_counter() - t0) / a.steps * 1e3
    tm = {}
    for _ in range(5):
        s.search(qn, q, 4, k=10, timings=tm)
    br = {k: round(v / 5, 3) for k, v in tm.items()}
    g = s.graph(qn, q, 4, k=10)
    for _ in range(3):
        g.run()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(a.steps):
        g.run()
    torch.cuda.synchronize(); elg = (time.perf_counter() - t0) / a.steps * 1e3
    # the graph uploads the whole batch here (a one-process group); on W GPUs
    # each rank uploads 1/W of it and the ranks all-gather it over xGMI
    # (not measurable on one GPU): the projection swaps the whole-batch H2D
    # for the 1/W one, all-gather excluded
    full = g.h_blk[0]
    part = full[: full.numel() // W]
    dst = torch.empty(full.numel(), dtype=torch.int32, device=dev)
    def h2d(src, n=20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dst[: src.numel()].copy_(src, non_blocking=True); e0.record()
        for _ in range(n):
            dst[: src.numel()].copy_(src, non_blocking=True)
        e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1) / n
    h_full, h_part = h2d(full), h2d(part)
    del g
    proj = elg - h_full + h_part
    # the batch stream (StreamedSearch): every rank uploads and routes the
    # whole batch in the plan branch, beside the scan; the list all-gather + K3
    # (rank 0 of W here: a one-process group, so none) runs in the F branch
    st = s.streamed(qn, q, 4, k=10)
    for _ in range(3):
        st.step()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(a.steps):
        st.step()
    torch.cuda.synchronize(); els = (time.perf_counter() - t0) / a.steps * 1e3
    del st
    print(f"world {W} chunk {ck}: step {el:.3f} ms eager (device-resident queries), {elg:.3f} ms graph "
          f"(whole-batch H2D {h_full:.3f} ms); with the 1/{W} upload ({h_part:.3f} ms): {proj:.3f} ms "
          f"-> {10000 / proj * 1e3:.0f} q/s on {W} GPUs (all-gathers over xGMI excluded); "
          f"batch stream {els:.3f} ms/launch (whole-batch H2D, list all-gather excluded) -> "
          f"{10000 / els * 1e3:.0f} q/s; breakdown {br}", flush=True)
    del ix, s; torch.cuda.empty_cache()
dist.destroy_process_group()
