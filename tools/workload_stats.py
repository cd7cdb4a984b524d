"""Dump the 10M bench workload's bucket sizes and per-bucket pair counts
(gpurun_out/wl_stats.npz) for tile-economics planning on the CPU."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd"))
import numpy as np, torch
from li import synth
from li.index import DeviceRouter
dev = torch.device("cuda")
x, q, qn, xn, layers = synth.build_lmi_workload(10_000_000, 10_000, 122, "MLP-5", dev)
router = DeviceRouter(layers)
labels = router.argmax(xn).cpu().numpy()
classes, _ = router.topr(qn, 7)
classes = classes.cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/wl_stats.npz", labels_count=np.bincount(labels, minlength=122),
                    classes=classes)
print("ok", np.bincount(labels, minlength=122)[:10])
