"""Synthetic LAION-like workloads; no dataset is reachable offline.

clip768-like vectors: a Gaussian mixture (centres ~ N(0,1)^d, points =
centre + noise * N(0,1)), L2-normalised and rounded to fp16 (stored as fp32,
so every value is fp16-representable, as the SISAP'23 clip768v2 `emb` is
believed to be).  pca96-like navigation vectors: X @ P with P ~ N(0,1)/sqrt(d)
fixed by the seed, then L2-normalised (search.py:50-52).

Two generators: a numpy PCG64 one for small, bit-reproducible test cases and
fixtures, and a torch one that builds 10M-row corpora directly in HBM for the
benchmark (chunked, counter-free but seeded).  Index building helpers (GPU
k-means, short router training) stand in for the reference's faiss k-means +
MLP training (LearnedIndex.py:197-282), which is outside the hot path.
"""
from __future__ import annotations

import math

import numpy as np
import torch


# ---------------------------------------------------------------------------
# numpy (small, reproducible)
# ---------------------------------------------------------------------------
def np_mixture(n: int, d: int, n_centres: int, seed: int, noise: float = 0.9,
               centres: np.ndarray | None = None):
    rng = np.random.Generator(np.random.PCG64(seed))
    if centres is None:
        centres = rng.standard_normal((n_centres, d)).astype(np.float32)
    lab = rng.integers(0, centres.shape[0], n)
    x = centres[lab] + noise * rng.standard_normal((n, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x.astype(np.float16).astype(np.float32), centres


def np_projection(d: int, d_nav: int, seed: int) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return (rng.standard_normal((d, d_nav)) / math.sqrt(d)).astype(np.float32)


def np_nav(x: np.ndarray, P: np.ndarray) -> np.ndarray:
    v = (x @ P).astype(np.float32)
    n = np.sqrt(np.einsum("ij,ij->i", v, v))
    n[n < 10 * np.finfo(np.float32).eps] = 1.0
    return (v / n[:, None]).astype(np.float32)


def np_router_layers(arch, n_classes: int, seed: int, d_nav: int = 96):
    """torch-nn.Linear-like init (U(-1/sqrt(in), 1/sqrt(in))), seeded numpy."""
    rng = np.random.Generator(np.random.PCG64(seed))
    dims = [d_nav] + list(arch) + [n_classes]
    layers = []
    for a, b in zip(dims, dims[1:]):
        bound = 1.0 / math.sqrt(a)
        layers.append((rng.uniform(-bound, bound, (b, a)).astype(np.float32),
                       rng.uniform(-bound, bound, (b,)).astype(np.float32)))
    return layers


ARCHS = {"MLP": (128,), "MLP-2": (64,), "MLP-3": (256,), "MLP-4": (512,), "MLP-5": (256, 128),
         "MLP-6": (32,), "MLP-7": (16,), "MLP-8": (8,)}


# ---------------------------------------------------------------------------
# torch (large, on device)
# ---------------------------------------------------------------------------
@torch.no_grad()
def torch_mixture(n: int, d: int, n_centres: int, seed: int, device, noise: float = 0.9,
                  centres: torch.Tensor | None = None, out_dtype=torch.float16,
                  chunk: int = 1 << 20):
    """n x d fp16-exact rows on `device` (returned in `out_dtype`)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    if centres is None:
        centres = torch.randn((n_centres, d), generator=g, device=device)
    out = torch.empty((n, d), dtype=out_dtype, device=device)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        lab = torch.randint(0, centres.shape[0], (b - a,), generator=g, device=device)
        x = centres[lab] + noise * torch.randn((b - a, d), generator=g, device=device)
        x /= x.norm(dim=1, keepdim=True)
        out[a:b] = x.half().to(out_dtype)
    return out, centres


@torch.no_grad()
def torch_nav(x: torch.Tensor, P: torch.Tensor, chunk: int = 1 << 20) -> torch.Tensor:
    out = torch.empty((x.shape[0], P.shape[1]), dtype=torch.float32, device=x.device)
    for a in range(0, x.shape[0], chunk):
        v = x[a:a + chunk].float() @ P
        n = v.norm(dim=1, keepdim=True)
        n[n < 10 * 1.1920929e-07] = 1.0
        out[a:a + chunk] = v / n
    return out


@torch.no_grad()
def kmeans(x: torch.Tensor, k: int, iters: int, seed: int) -> torch.Tensor:
    """Lloyd's k-means (squared L2), returns centroids [k, d]."""
    g = torch.Generator(device=x.device)
    g.manual_seed(seed)
    cent = x[torch.randperm(x.shape[0], generator=g, device=x.device)[:k]].clone()
    for _ in range(iters):
        d2 = (x * x).sum(1, keepdim=True) - 2 * x @ cent.T + (cent * cent).sum(1)[None]
        lab = d2.argmin(1)
        s = torch.zeros_like(cent).index_add_(0, lab, x)
        cnt = torch.bincount(lab, minlength=k).float()[:, None]
        cent = torch.where(cnt > 0, s / cnt.clamp(min=1), cent)
    return cent


def train_router(x_nav: torch.Tensor, labels: torch.Tensor, arch, n_classes: int, *,
                 steps: int = 300, batch: int = 4096, lr: float = 0.009, seed: int = 2023):
    """A short Adam/cross-entropy fit of the reference's Model architecture."""
    torch.manual_seed(seed)
    dims = [x_nav.shape[1]] + list(arch) + [n_classes]
    mods = []
    for i, (a, b) in enumerate(zip(dims, dims[1:])):
        mods.append(torch.nn.Linear(a, b))
        if i + 2 < len(dims):
            mods.append(torch.nn.ReLU())
    model = torch.nn.Sequential(*mods).to(x_nav.device)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    lossf = torch.nn.CrossEntropyLoss()
    g = torch.Generator(device=x_nav.device)
    g.manual_seed(seed)
    for _ in range(steps):
        idx = torch.randint(0, x_nav.shape[0], (batch,), generator=g, device=x_nav.device)
        loss = lossf(model(x_nav[idx]), labels[idx])
        opt.zero_grad()
        loss.backward()
        opt.step()
    return model.eval()


def build_lmi_workload(n: int, nq: int, n_buckets: int, arch: str, device, *, d: int = 768,
                       centres: int = 400, train_steps: int = 200, seed: int = 2023):
    """The benchmark workload, deterministic for a given seed.

    Corpus + queries on `device` (torch_mixture), pca96 navigation vectors, a
    router fitted on the CPU (k-means on a 100K subsample + short Adam fit of
    the reference architecture: CPU so the fit is reproducible run to run),
    object labels = router argmax on the GPU (LearnedIndex.py:240).
    Returns (x f16 [n,d], q f32 [nq,d], qn f32 [nq,96], layers, labels int32 [n])."""
    x, cen = torch_mixture(n, d, centres, seed=seed, device=device)
    q, _ = torch_mixture(nq, d, centres, seed=seed + 2219, device=device, centres=cen,
                         out_dtype=torch.float32)
    g = torch.Generator(device="cpu")
    g.manual_seed(96)
    P = (torch.randn((d, 96), generator=g) / math.sqrt(d)).to(device)
    xn = torch_nav(x, P)
    qn = torch_nav(q, P)
    sub_idx = torch.randperm(n, generator=g)[: min(n, 100_000)]
    sub = xn[sub_idx.to(device)].cpu()
    with torch.random.fork_rng(devices=[]):
        cent = kmeans(sub, n_buckets, iters=20, seed=7)
        d2 = (sub * sub).sum(1, keepdim=True) - 2 * sub @ cent.T + (cent * cent).sum(1)[None]
        model = train_router(sub, d2.argmin(1), ARCHS[arch], n_buckets, steps=train_steps,
                             batch=2048, seed=seed)
    layers = [(m.weight.detach().cpu(), m.bias.detach().cpu())
              for m in model if isinstance(m, torch.nn.Linear)]
    return x, q, qn, xn, layers


# ---------------------------------------------------------------------------
# BASELINE configs[4]: 100M random clip768-shaped vectors, k-means buckets
# ---------------------------------------------------------------------------
def random_rows_fn(d: int, seed: int, device, chunk: int = 1 << 20):
    """Counter-based rows: chunk i = normalised N(0,1) rows from a generator
    seeded (seed, i), rounded to fp16, so any rank regenerates any chunk."""
    def fn(a: int, b: int) -> torch.Tensor:
        if a % chunk:
            raise ValueError("rows are generated in whole chunks")
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1_000_003 + a // chunk)
        x = torch.randn((b - a, d), generator=g, device=device)
        x /= x.norm(dim=1, keepdim=True)
        return x.half()
    return fn


def build_random_workload(n: int, nq: int, n_buckets: int, arch: str, device, *, d: int = 768,
                          train_steps: int = 200, seed: int = 2023, chunk: int = 1 << 20):
    """configs[4]: n random unit vectors (fp16-exact), never materialised whole
    (li.index.RowSource).  Buckets: k-means (li.kmeans, the K5 kernels, faiss's
    122·256-row training sample) on the pca96 navigation vectors, a router fitted
    to them on the CPU (reproducible on every rank), object labels = router
    argmax (K1) chunk by chunk.  Returns (source, q f32, qn f32, layers, labels)."""
    from .index import DeviceRouter, RowSource
    from .kmeans import Kmeans
    fn = random_rows_fn(d, seed, device, chunk)
    src = RowSource(n, d, fn, chunk)
    gq = torch.Generator(device=device)
    gq.manual_seed(seed + 2219)
    with torch.no_grad():
        q = torch.randn((nq, d), generator=gq, device=device)
        q = (q / q.norm(dim=1, keepdim=True)).half().float()
    g = torch.Generator(device="cpu")
    g.manual_seed(96)
    P = (torch.randn((d, 96), generator=g) / math.sqrt(d)).to(device)
    qn = torch_nav(q, P)
    n_train = min(n, n_buckets * 256)
    sub = torch_nav(fn(0, min(n, chunk))[:n_train], P)
    km = Kmeans(96, n_buckets, niter=20, seed=seed, device=device)
    km.train(sub)
    _, lab = km.index.search(sub, 1)
    with torch.random.fork_rng(devices=[]):
        model = train_router(sub.cpu(), torch.from_numpy(lab[:, 0]), ARCHS[arch], n_buckets,
                             steps=train_steps, batch=2048, seed=seed)
    layers = [(m.weight.detach().cpu(), m.bias.detach().cpu())
              for m in model if isinstance(m, torch.nn.Linear)]
    router = DeviceRouter(layers, device=device)
    labels = torch.empty(n, dtype=torch.int32, device=device)
    for a, b, blk in src.chunks():
        labels[a:b] = router.argmax(torch_nav(blk, P)).to(torch.int32)
        del blk
    return src, q, qn, layers, labels


# ---------------------------------------------------------------------------
# a stream of distinct query batches for the same workload
# ---------------------------------------------------------------------------
@torch.no_grad()
def query_batches(n_batches: int, nq: int, device, *, kind: str = "mixture", d: int = 768,
                  centres: int = 400, seed: int = 2023):
    """n_batches distinct (q f32 [nq, d] fp16-exact, qn f32 [nq, 96]) batches
    on `device`, from the same distribution as the workload's queries: batch 0
    IS the workload's batch (build_lmi_workload's, or build_random_workload's
    with kind="random"); batch i > 0 draws from its own seed.  The mixture's
    centres and the pca96 projection are regenerated from their seeds (the
    first draws of the same generators), so nothing else of the workload is
    needed."""
    g = torch.Generator(device="cpu")
    g.manual_seed(96)
    P = (torch.randn((d, 96), generator=g) / math.sqrt(d)).to(device)
    out = []
    if kind == "mixture":
        gc = torch.Generator(device=device)
        gc.manual_seed(seed)
        cen = torch.randn((centres, d), generator=gc, device=device)
        for i in range(n_batches):
            q, _ = torch_mixture(nq, d, centres, seed=seed + 2219 + 7919 * i, device=device,
                                 centres=cen, out_dtype=torch.float32)
            out.append((q, torch_nav(q, P)))
    elif kind == "random":
        for i in range(n_batches):
            gq = torch.Generator(device=device)
            gq.manual_seed(seed + 2219 + 7919 * i)
            q = torch.randn((nq, d), generator=gq, device=device)
            q = (q / q.norm(dim=1, keepdim=True)).half().float()
            out.append((q, torch_nav(q, P)))
    else:
        raise ValueError("kind must be 'mixture' or 'random'")
    return out
