"""Do independent branches of a captured HIP graph run concurrently?  Two spin
kernels (torch.cuda._sleep, one workgroup each) on forked streams inside one
capture: wall time ~1x the spin if the branches overlap, ~2x if the graph runs
them one after the other.  Eager two-stream launch for comparison."""
import time, torch

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
cyc = 20_000_000
main = torch.cuda.current_stream()
side = torch.cuda.Stream()

def one():
    torch.cuda._sleep(cyc)

def two_branches():
    side.wait_stream(torch.cuda.current_stream())
    torch.cuda._sleep(cyc)
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc)
    torch.cuda.current_stream().wait_stream(side)

def timeit(fn, n=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3

print(f"one spin eager: {timeit(one):.2f} ms")
print(f"two spins, two streams eager: {timeit(two_branches):.2f} ms")
g1 = torch.cuda.CUDAGraph()
s = torch.cuda.Stream(); s.wait_stream(main)
with torch.cuda.stream(s):
    one()
torch.cuda.synchronize()
with torch.cuda.graph(g1):
    one()
print(f"one spin graph: {timeit(g1.replay):.2f} ms")
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    two_branches()
print(f"two spins, forked branches in one graph: {timeit(g2.replay):.2f} ms")
