"""Dump the 10M bench workload's device lists (classes, per-(query, probe)
top-10 d/pos, bucket sizes) to gpurun_out/lists10M.npz, for host-side replay
profiling on the CPU."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import numpy as np, torch
from li import synth
from li.index import DeviceIndex, DeviceRouter, Searcher
dev = torch.device("cuda")
x, q, qn, xn, layers = synth.build_lmi_workload(10_000_000, 10_000, 122, "MLP-5", dev)
router = DeviceRouter(layers)
labels = router.argmax(xn); del xn
ix = DeviceIndex(x, labels, 122)
s = Searcher(ix, router)
classes, d, pos, st = s.lists(qn, q, 4, 10)
torch.cuda.synchronize()
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/lists10M.npz", classes=classes.cpu().numpy(), d=d.cpu().numpy(),
                    pos=pos.cpu().numpy(), bucket_size=ix.bucket_size)
print("ok")
