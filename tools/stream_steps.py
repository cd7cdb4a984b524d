"""Rank 0's batch-stream launches (StreamedSearch) of a W-way striped 10M index on
one GPU, for kernel traces (tools/gpu_stream_trace.sh): builds the bench workload,
runs `--steps` launches per world and prints ms per launch.  The process is a
one-rank RCCL group, so a W > 1 stripe takes the exchange branch (its
all-gathers move only this rank's part); in float64 the other stripes' kth
blocks are computed first and held beside the gathered one, so the refinement
sees the W-rank band (StreamedSearch(kth_peers=...))."""
import argparse, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import torch
from li import synth
from li.index import DeviceIndex, DeviceRouter, Searcher

ap = argparse.ArgumentParser()
ap.add_argument("--worlds", default="1,8")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--eager", action="store_true", help="launch the three branches eagerly on three streams")
ap.add_argument("--modes", default="stream", help="comma list of stream (default: lookahead behind the finish), stream-nola (no lookahead), stream-eager, graph-pipe, graph")
ap.add_argument("--dist", default="f32", choices=["f32", "f64"])
ap.add_argument("--chunks", default="", help="comma list of chunk rows to try (default: the bench's by W)")
ap.add_argument("--all-ranks", action="store_true", help="time every rank's stripe of each W (not only rank 0)")
ap.add_argument("--local-band", action="store_true",
                help="float64: every stripe refines the band of its own list (the round-5 form; "
                     "LMI_F64_LOCAL_BAND=1 must be set too) instead of the W-rank band")
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
import torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29534")
dist.init_process_group("nccl", rank=0, world_size=1)   # a one-process group: rank 0 of W
x, q, qn, xn, layers = synth.build_lmi_workload(10_000_000, 10_000, 122, "MLP-5", dev)
router = DeviceRouter(layers)
labels = router.argmax(xn); del xn
from li import _lib
from li.index import bucket_topk_f64, global_band

kth_of = {}


def peer_kth(W, ck):
    """float64 (ABI 10 global band): every stripe's kth block of the batch
    (its pairs' 10 smallest d32 after the chunk merge, what the F1 all-gather
    of a real W-rank run hands every rank), so a one-rank rehearsal of stripe
    rk refines the W-rank band (StreamedSearch(kth_peers=...))."""
    if (W, ck) not in kth_of:
        cls = router.topr(qn, 4)[0]
        out = []
        for g in range(W):
            ixg = DeviceIndex(x, labels, 122, chunk_rows=ck, rank=g, world=W)
            kth = torch.empty((q.shape[0] * 4 * 10,), dtype=torch.float32, device=dev)
            ph = _lib.LMI_Q_PHASE_PLAN | _lib.LMI_Q_PHASE_SCAN | _lib.LMI_Q_PHASE_MERGE
            bucket_topk_f64(ixg, q, cls, 10, qmode=_lib.LMI_Q_F16, seed_round0=True, phases=ph,
                            band_x=(kth, None, W))
            torch.cuda.synchronize()
            out.append(kth)
            del ixg
        kth_of[W, ck] = torch.stack(out)
    return kth_of[W, ck]


for W, ck, rk in [(W, ck, rk) for W in map(int, a.worlds.split(","))
                  for ck in (list(map(int, a.chunks.split(","))) if a.chunks else
                             [8192 if W == 1 else 4096 if W <= 4 else 2048])
                  for rk in (range(W) if a.all_ranks else [0])]:
    ix = DeviceIndex(x, labels, 122, chunk_rows=ck, rank=rk, world=W)
    s = Searcher(ix, router)
    for mode in a.modes.split(","):
        if mode.startswith("stream"):
            kw = {}
            if a.dist == "f64" and W > 1 and not a.local_band and global_band(ix, q.shape[0], 4, 10,
                                                                              _lib.LMI_Q_F16):
                ka = peer_kth(W, ck)
                kw["kth_peers"] = torch.cat([ka[:rk], ka[rk + 1:]])
            st = s.streamed(qn, q, 4, k=10, dist=a.dist, capture=not (a.eager or mode == "stream-eager"),
                            lookahead=mode != "stream-nola", **kw)
            fn = st.step
        else:
            st = s.graph(qn, q, 4, k=10, dist=a.dist, pipeline=mode == "graph-pipe")
            fn = st.run
        for _ in range(3):
            fn()
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        print(f"world {W} rank {rk} chunk {ck} {a.dist}: {mode} {(time.perf_counter() - t0) / a.steps * 1e3:.3f} ms/step "
              f"(scan WGs {os.environ.get('LMI_SCAN_WGS', 'all CUs')})", flush=True)
        del st, fn
    del s, ix; torch.cuda.empty_cache()
