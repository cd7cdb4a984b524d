"""Multi-GPU search: one process per GPU, the corpus striped over the ranks.

SURVEY.md §8(e): every bucket's rows are split into G contiguous slices
(li.index.BucketLayout.shard), rank g scans slice g of every probed bucket,
and the per-(query, probe) top-k is recovered exactly by merging the G
per-shard lists: top-k(union of shards) = top-k(union of per-shard top-k).
The one exchange step is an all-gather of the lists (nq*R*k*8 bytes per rank,
~3.2 MB at 10k queries, R=4: latency-bound on xGMI), over RCCL
(torch.distributed backend "nccl"), followed by K3 (lmi_merge_topk) on every
rank.  Every rank ends up with the same classes.  Results are bitwise identical
for any G because every list is ordered by (distance, global position).
The router is sharded by queries (route_sharded): each rank routes nq/G queries
and the classes are all-gathered (nq*R*4 bytes), so its cost shrinks with G;
the per-query results are the same as routing the whole batch on one GPU.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch
import torch.distributed as dist


def init_from_env(backend: Optional[str] = None):
    """torchrun-style init (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); 127.0.0.1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1:
        return rank, world, local
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    if backend is None:
        # LMI_DIST_BACKEND=gloo: control-flow rehearsal of several ranks on one
        # GPU (RCCL refuses two ranks on one device); collectives then stage
        # through host memory (_all_gather).  The product path is RCCL.
        backend = os.environ.get("LMI_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def _all_gather(out: torch.Tensor, part: torch.Tensor, group=None):
    """all_gather_into_tensor; device tensors go through host copies on gloo."""
    if part.is_cuda and dist.get_backend(group) == "gloo":
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, part.cpu(), group=group)
        out.copy_(h)
        return
    dist.all_gather_into_tensor(out, part, group=group)


def all_gather_lists(d: torch.Tensor, pos: torch.Tensor, group=None):
    """[nq, R, k] per rank -> [G, nq, R, k] on every rank, in ONE collective:
    the f32 distances travel bit-for-bit as int32 beside the positions."""
    G = dist.get_world_size(group)
    both = torch.stack((d.contiguous().view(torch.int32), pos.to(torch.int32).contiguous()), dim=-1)
    # concatenated along dim 0 (the form both RCCL and gloo accept), viewed [G, ...]
    out = torch.empty((G * both.shape[0],) + tuple(both.shape[1:]), dtype=both.dtype, device=both.device)
    _all_gather(out, both, group)
    out = out.view((G,) + tuple(both.shape))
    gd = out[..., 0].contiguous().view(torch.float32)
    gp = out[..., 1].contiguous().to(pos.dtype)
    return gd, gp


def gather_merge(d: torch.Tensor, pos: torch.Tensor, k: int, group=None,
                 merge: Optional[Callable] = None):
    """All-gather the shard lists and merge them (K3 on the GPU by default).

    `merge(gd, gp, k) -> (d, pos)` can be swapped for a CPU checker in the
    gloo tests; the product path always uses lmi_merge_topk."""
    gd, gp = all_gather_lists(d, pos, group)
    if merge is None:
        from .index import merge_topk
        return merge_topk(gd, gp, k)
    return merge(gd, gp, k)


def route_sharded(router, q_nav: torch.Tensor, R: int, group=None) -> torch.Tensor:
    """K1 on this rank's contiguous slice of the queries, then an all-gather of
    the classes: [nq, R] int32 on every rank, equal to router.topr(q_nav, R)
    (the router is per-query: a query's classes do not depend on its batch)."""
    G = dist.get_world_size(group)
    g = dist.get_rank(group)
    nq = q_nav.shape[0]
    per = -(-nq // G)
    lo = min(nq, g * per)
    hi = min(nq, lo + per)
    part = torch.zeros((per, R), dtype=torch.int32, device=q_nav.device)
    if hi > lo:
        c, _ = router.topr(q_nav[lo:hi], R)
        part[: hi - lo] = c
    out = torch.empty((G * per, R), dtype=torch.int32, device=q_nav.device)
    _all_gather(out, part, group)
    return out[:nq]
