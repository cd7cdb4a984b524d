"""faiss.Kmeans stand-in on the GPU k-means kernels.

The reference builds its buckets with

    kmeans = faiss.Kmeans(d=..., k=n_clusters, verbose=True, seed=2023)
    kmeans.train(X)
    labels = kmeans.index.search(X, 1)[1].T[0]        (LearnedIndex.py:275-282)

``Kmeans`` keeps that surface (``d``, ``k``, ``niter``, ``seed``,
``max_points_per_centroid``, ``train``, ``centroids``, ``obj``,
``index.search``).  faiss's Clustering::train is restated: train on a
seeded sample of k·max_points_per_centroid rows, initialise with k random
training rows, then ``niter`` Lloyd iterations — assignment
(``lmi_kmeans_assign``), mean update (``lmi_kmeans_update``), and faiss's
split of empty clusters on the host (k rows, a few microseconds).  The
random streams are numpy's, not faiss's mt19937, so samples and inits differ
from faiss's; the arithmetic is reproduced bit for bit by
oracle/lmi_oracle.py::kmeans_train (tests/test_gpu_kmeans.py).

There is no CPU path: without a HIP device and liblmi_hip.so this raises.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

_EPS = np.float32(1.0 / 1024.0)


def _as_device_f32(X, device) -> torch.Tensor:
    if isinstance(X, torch.Tensor):
        t = X.to(device=device, dtype=torch.float32)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(X), dtype=np.float32)).to(device)
    return t.contiguous()


def assign(x: torch.Tensor, cent: torch.Tensor, want_dist: bool = True):
    """Nearest centroid of every row (squared L2, ties -> lower index)."""
    lib = _lib.load()
    if x.dim() != 2 or cent.dim() != 2 or x.shape[1] != cent.shape[1]:
        raise ValueError(f"shapes {tuple(x.shape)} / {tuple(cent.shape)}")
    if x.device.type != "cuda" or cent.device != x.device:
        raise ValueError("x and centroids must be on the same HIP device")
    x = x.contiguous()
    cent = cent.contiguous()
    n, d = x.shape
    lab = torch.empty(n, dtype=torch.int32, device=x.device)
    dist = torch.empty(n, dtype=torch.float32, device=x.device) if want_dist else None
    _lib.check("lmi_kmeans_assign", lib.lmi_kmeans_assign(
        _lib.ptr(x), n, d, _lib.ptr(cent), cent.shape[0], _lib.ptr(lab), _lib.ptr(dist),
        _lib.stream_handle(x.device)))
    return lab, dist


def update(x: torch.Tensor, labels: torch.Tensor, cent: torch.Tensor):
    """In-place mean update of ``cent``; returns the per-cluster counts (int64)."""
    lib = _lib.load()
    n, d = x.shape
    k = cent.shape[0]
    ws = torch.empty(max(int(lib.lmi_kmeans_workspace_bytes(n, d, k)), 1), dtype=torch.uint8,
                     device=x.device)
    counts = torch.empty(k, dtype=torch.int64, device=x.device)
    status = torch.zeros(1, dtype=torch.int32, device=x.device)
    _lib.check("lmi_kmeans_update", lib.lmi_kmeans_update(
        _lib.ptr(x), n, d, _lib.ptr(labels), k, _lib.ptr(cent), _lib.ptr(counts), _lib.ptr(status),
        _lib.ptr(ws), ws.numel(), _lib.stream_handle(x.device)))
    if int(status.item()):
        raise RuntimeError("lmi_kmeans_update: label outside [0, k)")
    return counts


def split_empty(cent: np.ndarray, counts: np.ndarray, n: int, rng) -> int:
    """faiss split_clusters (Clustering.cpp): an empty centroid ci copies the
    cluster cj met first with r < (|cj| - 1)/(n - k) in a cyclic scan, both
    are nudged by ±1/1024 on alternating dimensions, and cj's count is split."""
    k = cent.shape[0]
    nsplit = 0
    for ci in np.flatnonzero(counts == 0):
        cj = 0
        while True:
            p = np.float32((counts[cj] - 1.0) / float(np.float32(n - k)))
            if np.float32(rng.random_sample()) < p:
                break
            cj = (cj + 1) % k
        cent[ci] = cent[cj]
        cent[ci, 0::2] *= np.float32(1) + _EPS
        cent[cj, 0::2] *= np.float32(1) - _EPS
        cent[ci, 1::2] *= np.float32(1) - _EPS
        cent[cj, 1::2] *= np.float32(1) + _EPS
        counts[ci] = counts[cj] // 2
        counts[cj] -= counts[ci]
        nsplit += 1
    return nsplit


class _FlatL2:
    """faiss.IndexFlatL2 over the centroids, search(X, 1) only (what
    LearnedIndex.py:282 uses): (squared distances [n,1] f32, labels [n,1] i64)."""

    def __init__(self, cent: torch.Tensor):
        self.cent = cent
        self.ntotal = cent.shape[0]

    def search(self, X, k: int = 1):
        if k != 1:
            raise NotImplementedError("only the nearest centroid (k=1) is provided")
        x = _as_device_f32(X, self.cent.device)
        lab, dist = assign(x, self.cent)
        return (dist.cpu().numpy().reshape(-1, 1),
                lab.to(torch.int64).cpu().numpy().reshape(-1, 1))


class Kmeans:
    """faiss.Kmeans(d, k, niter=25, verbose=False, seed=1234, ...) on the GPU."""

    def __init__(self, d: int, k: int, niter: int = 25, verbose: bool = False, seed: int = 1234,
                 max_points_per_centroid: int = 256, device=None, **_unused):
        if d < 1 or d > _lib.LMI_KMEANS_MAX_D:
            raise ValueError(f"d={d} outside [1, {_lib.LMI_KMEANS_MAX_D}]")
        self.d, self.k, self.niter, self.verbose, self.seed = d, k, niter, verbose, seed
        self.max_points_per_centroid = max_points_per_centroid
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.centroids = None
        self.obj = []
        self.index = None

    def train(self, X) -> float:
        x = _as_device_f32(X, self.device)
        n_all, d = x.shape
        if d != self.d:
            raise ValueError(f"data has d={d}, Kmeans was made with d={self.d}")
        k = self.k
        if n_all > k * self.max_points_per_centroid:
            sel = np.random.RandomState(self.seed).permutation(n_all)[: k * self.max_points_per_centroid]
            xt = x[torch.from_numpy(sel).to(self.device)].contiguous()
        else:
            xt = x
        n = xt.shape[0]
        if n < k:
            raise ValueError(f"{n} training points for {k} centroids")
        init = np.random.RandomState(self.seed + 1).permutation(n)[:k]
        cent = xt[torch.from_numpy(init).to(self.device)].contiguous()
        rng = np.random.RandomState(1234)
        self.obj = []
        for it in range(self.niter):
            lab, dist = assign(xt, cent)
            self.obj.append(float(dist.double().sum().item()))
            counts = update(xt, lab, cent)
            cnt = counts.cpu().numpy()
            if (cnt == 0).any():
                c_host = cent.cpu().numpy()
                split_empty(c_host, cnt, n, rng)
                cent.copy_(torch.from_numpy(c_host))
            if self.verbose:
                print(f"  Iteration {it} objective={self.obj[-1]:.6g}", flush=True)
        self.centroids = cent.cpu().numpy()
        self.index = _FlatL2(cent)
        return self.obj[-1] if self.obj else 0.0
