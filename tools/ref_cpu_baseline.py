#!/usr/bin/env python3
"""Time the REFERENCE itself on the CPU (this container only: the reference
never travels to the GPU box) — BASELINE.md's CPU-baseline plan:

  * imports the reference (/root/reference/search/li) with the environment
    shims of tests/golden/gen_golden.py (empty faiss/h5py modules, a
    list-returning np.ogrid, the namespace package registered as a package);
  * builds the DataFrames exactly as search.py:71-93 does (index += 1);
  * times exactly search.py:116-141 for R > 1:
        s = time.time(); li.search(data, queries, data_search, queries_search,
        pred_categories, n_buckets=R, k=10, use_threshold=True); time.time() - s
    (router predict_proba + every round of search_single + the merges);
  * on the bench's own synthetic workload (li.synth.build_lmi_workload, built
    on the CPU; object labels = the router's argmax, LearnedIndex.py:240),
    at 300K R=7 (configs[1]) and 1M R=4, with 8 threads and 1 thread
    (OMP/OPENBLAS/MKL thread counts and torch.set_num_threads), GPUs hidden.

    python tools/ref_cpu_baseline.py [--sizes 300K:7,1M:4] [--threads 8,1] [--dtype f32]

Writes profiles/ref_cpu_<size>_R<R>_<threads>t_<dtype>.json.  float32
DataFrames take the reference's float32 branch (the bench's arithmetic); with
--dtype f16 the data and queries are float16, as the real clip768 'emb', and
the reference computes in float64 (utils.py:11)."""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SIZES = {"300K": 300_000, "1M": 1_000_000, "10M": 10_000_000}


def child(size: str, R: int, threads: int, dtype: str, nq: int):
    sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests"),
                    os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd")]
    import numpy as np
    import pandas as pd
    import torch
    torch.set_num_threads(threads)
    from li import synth  # this repo's generator (before `li` is re-bound to the reference)
    t0 = time.time()
    x, q, qn, xn, layers = synth.build_lmi_workload(SIZES[size], nq, 122, "MLP-5", "cpu")
    labels = np.empty(xn.shape[0], np.int64)
    with torch.no_grad():
        for a in range(0, xn.shape[0], 1 << 20):   # chunked: 10M x 256 f32 is 10 GB
            h = xn[a:a + (1 << 20)]
            for i, (w, b) in enumerate(layers):
                h = h @ w.T + b
                if i + 1 < len(layers):
                    h = torch.relu(h)
            labels[a:a + h.shape[0]] = h.argmax(dim=1).numpy()
    x = x.numpy()
    q = q.numpy()
    # copy=False: at 10M the fp16 corpus is 15.4 GB, a second copy would not
    # leave room for the reference's per-bucket float64 temporaries in 64 GB
    if dtype == "f32":
        x, q = x.astype(np.float32, copy=False), q.astype(np.float32, copy=False)
    else:
        x, q = x.astype(np.float16, copy=False), q.astype(np.float16, copy=False)
    xn, qn = xn.numpy(), qn.numpy()
    layers = [(w.numpy(), b.numpy()) for w, b in layers]
    t_build = time.time() - t0
    from gen_golden import _import_reference, _nn_with
    LearnedIndex, NeuralNetwork, _ = _import_reference()
    li = LearnedIndex()
    li.model = _nn_with(NeuralNetwork, layers, "MLP-5", 122)
    data = pd.DataFrame(xn)
    data.index += 1                       # search.py:71-72
    data_search = pd.DataFrame(x)
    data_search.index += 1                # search.py:83-84
    s = time.time()                       # search.py:116
    dists, nns = li.search(data_navigation=data, queries_navigation=qn, data_search=data_search,
                           queries_search=q, pred_categories=labels, n_buckets=R, k=10,
                           use_threshold=True)
    search_t = time.time() - s            # search.py:141
    out = {"what": "reference LearnedIndex.search timed as search.py:116-141 (router predict_proba "
                   "+ R rounds of search_single + merges), DataFrames as search.py:71-93",
           "size": size, "n": SIZES[size], "nq": nq, "R": R, "k": 10, "dtype": dtype,
           "arithmetic": "float32" if dtype == "f32" else "float64 (sklearn promotes float16)",
           "threads": threads, "search_s": round(search_t, 3), "qps": round(nq / search_t, 2),
           "workload": "li.synth.build_lmi_workload (bench's synthetic clip768-like mixture, "
                       "MLP-5 router, labels = router argmax)",
           "workload_build_s": round(t_build, 1), "cpu": platform.processor() or platform.machine(),
           "nproc": os.cpu_count(), "dists_dtype": str(dists.dtype), "nns_dtype": str(nns.dtype)}
    print(json.dumps(out))


def main():
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from gen_golden import FEATURES
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="300K:7,1M:4")
    ap.add_argument("--threads", default="8,1")
    ap.add_argument("--dtype", default="f32", choices=["f32", "f16"])
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--child", nargs=4, metavar=("SIZE", "R", "THREADS", "DTYPE"))
    a = ap.parse_args()
    if a.child:
        child(a.child[0], int(a.child[1]), int(a.child[2]), a.child[3], a.nq)
        return
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for sr in a.sizes.split(","):
        size, R = sr.split(":")
        for t in a.threads.split(","):
            env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", NPY_DISABLE_CPU_FEATURES=FEATURES,
                       CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS=t,
                       OPENBLAS_NUM_THREADS=t, MKL_NUM_THREADS=t)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--nq", str(a.nq),
                                "--child", size, R, t, a.dtype], env=env, capture_output=True,
                               text=True)
            if r.returncode != 0:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(r.returncode)
            line = r.stdout.strip().splitlines()[-1]
            path = os.path.join(ROOT, "profiles", f"ref_cpu_{size}_R{R}_{t}t_{a.dtype}.json")
            with open(path, "w") as f:
                f.write(line + "\n")
            print(line, flush=True)


if __name__ == "__main__":
    main()
