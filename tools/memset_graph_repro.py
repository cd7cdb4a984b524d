"""Minimal repro for the round-3 memset-node finding ("Memset
nodes"): do hipMemsetAsync nodes captured in HIP graphs
keep writing their value after eager device work runs between replays?

Round 3 saw two captured search steps answer wrong lists "for good" once an
eager search or a tensor clone ran between their replays, and cured it by
initialising the workspace with a fill kernel instead of hipMemsetAsync.  This
isolates the mechanism without the library:

  two graphs, each:  memset node(s) on a buffer allocated OUTSIDE capture
                     (as the step's workspace was) -> a kernel that reads it
  replay both, run eager work (allocations, clones, kernels, eager memsets,
  a third graph's capture), scribble the buffers, replay again, check.

Variants: hipMemsetAsync (byte value) and hipMemsetD32Async (word value), on
sizes that are / are not multiples of 4 and above / below 64 KiB; the same
sequence with a torch fill kernel (what the product uses) as the control.
Each check is the buffer's content after the replay (a graph that stopped
applying its memset leaves the scribble), and a reduction kernel inside the
graph that reads it.

    python tools/memset_graph_repro.py [--rounds 20]
"""
import argparse
import ctypes
import json

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=20)
ap.add_argument("--out", default=None)
ap.add_argument("--quick", action="store_true", help="one size per kind, every eager-work mode")
a = ap.parse_args()

hip = ctypes.CDLL("libamdhip64.so.7")  # torch's HIP runtime (same soname: the loaded copy)
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
dev = torch.device("cuda", 0)


def stream():
    return torch.cuda.current_stream(dev).cuda_stream


def memset(kind, buf, nbytes, value):
    if kind == "memset8":
        rc = hip.hipMemsetAsync(buf.data_ptr(), value & 0xFF, nbytes, stream())
    elif kind == "memset32":
        rc = hip.hipMemsetD32Async(buf.data_ptr(), value, nbytes // 4, stream())
    else:  # control: a torch fill kernel
        buf.view(torch.uint8)[:nbytes].fill_(value & 0xFF)
        rc = 0
    assert rc == 0, rc


def expected(kind, nbytes, value):
    if kind == "memset32":
        return bytes((value >> (8 * (i % 4))) & 0xFF for i in range(4)) * (nbytes // 4)
    return bytes([value & 0xFF]) * nbytes


def run(kind, nbytes, rounds, eager="full", n_graphs=2, scribble=True):
    n_words = (nbytes + 3) // 4 + 64
    bufs = [torch.zeros(n_words, dtype=torch.int32, device=dev) for _ in range(2)]
    sums = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(2)]
    vals = [0x5A5A5A5A, 0x3C3C3C3C] if kind != "memset32" else [0x01020304, 0x0A0B0C0D]
    graphs = []
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):  # warm-up (allocator, kernels)
        for i in range(2):
            memset(kind, bufs[i], nbytes, vals[i])
            sums[i].copy_(bufs[i].view(torch.uint8)[:nbytes].sum())
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    for i in range(n_graphs):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            memset(kind, bufs[i], nbytes, vals[i])
            sums[i].copy_(bufs[i].view(torch.uint8)[:nbytes].sum())
        graphs.append(g)
    want = [expected(kind, nbytes, v) for v in vals]
    want_sum = [sum(w) for w in want]
    fails = []
    junk = []
    for r in range(rounds):
        if scribble:
            for i in range(n_graphs):
                bufs[i].fill_(0x77777777)  # scribble: a replay must restore the memset value
        torch.cuda.synchronize()
        for i in range(n_graphs):
            graphs[i].replay()
        torch.cuda.synchronize()
        for i in range(n_graphs):
            got = bytes(bufs[i].view(torch.uint8)[:nbytes].cpu().numpy())
            s = int(sums[i].item())
            if got != want[i] or s != want_sum[i]:
                bad = sum(1 for x, y in zip(got, want[i]) if x != y)
                vals = sorted(set(got))[:4]
                fails.append({"round": r, "graph": i, "bytes_wrong": bad, "byte_values": vals,
                              "sum": s, "want_sum": want_sum[i]})
        if eager == "none":
            continue
        # eager device work between replays, as the bench's checks did
        x = torch.randn(1 << 20, device=dev)
        junk.append(x.clone())
        e = torch.empty(nbytes + 256, dtype=torch.uint8, device=dev)
        memset(kind if kind != "fill" else "fill", e, nbytes, 0x11)
        junk.append((x * 2).sum())
        if r == rounds // 2:
            g3 = torch.cuda.Graph() if hasattr(torch.cuda, "Graph") else torch.cuda.CUDAGraph()
            t3 = torch.zeros(4096, dtype=torch.int32, device=dev)
            with torch.cuda.graph(g3):
                memset(kind, t3, 4096, 0x22)
            g3.replay()
            junk.append((g3, t3))
        if len(junk) > 8:
            junk = junk[-8:]
        torch.cuda.synchronize()
    return fails


res = {}
if a.quick:
    # which ingredient breaks the memset nodes: eager work between replays,
    # the eager scribble of the buffers, a second graph
    for kind in ("memset8", "memset32", "fill"):
        for eager, n_graphs, scribble in (("none", 1, False), ("none", 1, True), ("none", 2, True),
                                          ("full", 1, True), ("full", 2, True), ("full", 2, False)):
            f = run(kind, 1 << 20, a.rounds, eager=eager, n_graphs=n_graphs, scribble=scribble)
            key = f"{kind}_eager-{eager}_graphs-{n_graphs}_scribble-{int(scribble)}"
            res[key] = {"failures": len(f), "first": f[:2]}
            print(f"{key:44s}: {len(f)} failing checks of {n_graphs * a.rounds}"
                  + (f"  first {f[0]}" if f else ""), flush=True)
else:
    for kind in ("memset8", "memset32", "fill"):
        for nbytes in (4096, 4096 + 3, 1 << 20, (1 << 20) + 6, 24 << 20):
            if kind == "memset32" and nbytes % 4:
                continue
            f = run(kind, nbytes, a.rounds)
            res[f"{kind}_{nbytes}"] = {"failures": len(f), "first": f[:3]}
            print(f"{kind:9s} {nbytes:>10d} B: {len(f)} failing checks of {2 * a.rounds}"
                  + (f"  first {f[0]}" if f else ""), flush=True)
if a.out:
    json.dump(res, open(a.out, "w"), indent=1)
