#!/usr/bin/env python3
"""The eval-facing number: search.py's own `querytime` (the span
search.py:116-141 that store_results writes into the H5 result file, read by
eval/) at BASELINE configs[2], from H5 files in the reference's layout.

    python tools/cli_querytime.py [--n 10000000] [--bp 3 4 5] [--work /tmp/lmi_cli]

Three child processes (this parent never touches the GPU):
  1. gen: the bench's synthetic 10M workload (li.synth.build_lmi_workload) laid
     out as data/pca96v2/10M/{dataset,query}.h5 ['pca96'] (float32) and
     data/clip768v2/10M/{dataset,query}.h5 ['emb'] (float16, the real dtype),
     and its MLP-5 router pickled as a LearnedIndex (save_as_pickle format);
  2. cli: `python search.py --size 10M -bp ... --index <pickle>` in the work
     directory: loads the H5 files, normalises pca96, labels the corpus with
     the router (LearnedIndex.py:240), attaches the index (outside the timer)
     and times li.search per bucket count exactly over search.py:116-141;
  3. cli without attach (LMI_NO_ATTACH=1): every timed call hashes its inputs.
The float16 'emb' makes the reference (and the drop-in) compute float64
distances (utils.py:11).  Writes profiles/r03_cli_10M.json."""
import argparse
import json
import os
import re
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd")


def gen(n, work):
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    from li import h5, synth
    from li.LearnedIndex import LearnedIndex
    from li.index_io import save_index
    from li.model import NeuralNetwork
    t0 = time.time()
    x, q, qn, xn, layers = synth.build_lmi_workload(n, 10_000, 122, "MLP-5", torch.device("cuda"))
    for kind, key, data, qq, fp16 in (("pca96v2", "pca96", xn, qn, False),
                                      ("clip768v2", "emb", x, q, True)):
        d = os.path.join(work, "data", kind, "10M")
        os.makedirs(d, exist_ok=True)
        host = (lambda t: t.half().cpu().numpy()) if fp16 else (lambda t: t.float().cpu().numpy())
        h5.write_dataset(os.path.join(d, "query.h5"), key, host(qq), fp16=fp16)
        h5.write_dataset(os.path.join(d, "dataset.h5"), key, host(data), fp16=fp16)
        print(f"[gen] {kind} written ({time.time() - t0:.1f}s)", flush=True)
    nn = NeuralNetwork(input_dim=96, output_dim=122, lr=0.009, model_type="MLP-5")
    lin = [m for m in nn.model.layers if isinstance(m, torch.nn.Linear)]
    with torch.no_grad():
        for m, (w, b) in zip(lin, layers):
            m.weight.copy_(w)
            m.bias.copy_(b)
    nn.model = nn.model.cpu()      # a host-side pickle, like the reference's (load_index moves it)
    li = LearnedIndex()
    li.model = nn
    os.makedirs(os.path.join(work, "models"), exist_ok=True)
    save_index(os.path.join(work, "models", "lmi.pkl"), li)
    print(f"[gen] done in {time.time() - t0:.1f}s", flush=True)


def _child(cmd, cwd, env, log_path):
    """Run a child with its output streamed into log_path (gpurun_out/: the
    box sees progress) and a heartbeat on stdout every 20 s."""
    t0 = time.time()
    with open(log_path, "w") as f:
        p = subprocess.Popen(cmd, cwd=cwd, env=env, stdout=f, stderr=subprocess.STDOUT)
        while p.poll() is None:
            time.sleep(1)
            if int(time.time() - t0) % 20 == 0:
                print(f"[cli_querytime] {os.path.basename(log_path)}: {time.time() - t0:.0f}s", flush=True)
    with open(log_path) as f:
        return p.returncode, f.read(), time.time() - t0


def run_cli(work, bp, env_extra, label):
    env = dict(os.environ, **env_extra)
    cmd = [sys.executable, "-u", os.path.join(PKG, "search.py"), "--size", "10M", "-bp", *bp,
           "--index", os.path.join(work, "models", "lmi.pkl")]
    rc, log, wall = _child(cmd, work, env, os.path.join(ROOT, "gpurun_out", f"cli_{label}.log"))
    if rc != 0:
        raise SystemExit(f"cli {label} failed ({rc}):\n{log[-3000:]}")
    rs = [int(v) for v in re.findall(r"Searching with (\d+) buckets", log)]
    ts = [float(v) for v in re.findall(r"Search time: ([0-9.eE+-]+)", log)]
    return {"wall_s": round(wall, 1), "querytime_s": {str(R): t for R, t in zip(rs, ts)},
            "qps": {str(R): round(10_000 / t, 1) for R, t in zip(rs, ts)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--bp", nargs="+", default=["3", "4", "5"])
    ap.add_argument("--work", default="/tmp/lmi_cli")
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child == "gen":
        gen(a.n, a.work)
        return
    os.makedirs(a.work, exist_ok=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    t0 = time.time()
    rc, log, _ = _child([sys.executable, "-u", os.path.abspath(__file__), "--child", "gen", "--n",
                         str(a.n), "--work", a.work], ROOT, dict(os.environ),
                        os.path.join(ROOT, "gpurun_out", "cli_gen.log"))
    if rc != 0:
        raise SystemExit(f"gen failed ({rc}):\n{log[-3000:]}")
    gen_s = time.time() - t0
    out = {"what": "search.py (the CLI) querytime = the span search.py:116-141, per bucket count "
                   "(-bp -> R = int(bp/100*122)), from H5 files: pca96 float32, clip768v2 'emb' "
                   "float16 (float64 arithmetic, as the reference on the real data)",
           "n": a.n, "nq": 10_000, "k": 10, "router": "MLP-5 (pickled, --index)", "gen_s": round(gen_s, 1),
           "attached": run_cli(a.work, a.bp, {}, "attached"),
           "not_attached": run_cli(a.work, a.bp, {"LMI_NO_ATTACH": "1"}, "not_attached")}
    print(json.dumps(out))
    with open(os.path.join(ROOT, "profiles", "r03_cli_10M.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
