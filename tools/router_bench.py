"""Router (K1) timing: topr / argmax for 10k queries on a few synthetic
architectures, torch events around the launches (diagnostic)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import torch
from li.index import DeviceRouter

dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
for arch, hidden in [("MLP-5", (256, 128)), ("MLP", (128,)), ("MLP-8", (8,))]:
    dims = (96,) + hidden + (122,)
    layers = [((torch.randn(dims[i + 1], dims[i], generator=g) * 0.1).numpy(),
               (torch.randn(dims[i + 1], generator=g) * 0.1).numpy()) for i in range(len(dims) - 1)]
    router = DeviceRouter(layers)
    x = torch.nn.functional.normalize(torch.randn(10000, 96, generator=g), dim=1).to(dev)
    for mode in ("topr", "argmax"):
        fn = (lambda: router.topr(x, 4)) if mode == "topr" else (lambda: router.argmax(x))
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{arch:6s} {mode:6s} {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us", flush=True)
