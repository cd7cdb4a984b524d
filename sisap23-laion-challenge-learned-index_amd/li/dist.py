"""Multi-GPU search: one process per GPU, the corpus striped over the ranks.

SURVEY.md §8(e): every bucket's rows are split into G contiguous slices
(li.index.BucketLayout.shard), rank g scans slice g of every probed bucket,
and the per-(query, probe) top-k is recovered exactly by merging the G
per-shard lists: top-k(union of shards) = top-k(union of per-shard top-k).
The one exchange step is an all-gather of the lists (nq*R*k*8 bytes per rank,
~3.2 MB at 10k queries, R=4: latency-bound on xGMI), over RCCL
(torch.distributed backend "nccl"), followed by K3 on every rank.  The product
path (Searcher) has K2 write each rank's lists and status word straight into
one packed send buffer (packed_lists) and K3 read the gathered buffer in place
(gather_merge_packed: lmi_merge_topk_packed); gather_merge is the general form
(any merge callable, the CPU gloo tests).  Every rank ends up with the same classes.  Results are bitwise identical
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


def force_exchange() -> bool:
    """LMI_FORCE_EXCHANGE=1: every step form takes its G > 1 branch even in a
    one-rank process group -- the striped layout's packed lists, the captured
    all-gather (RCCL over one rank), lmi_merge_topk_packed, the sharded
    router's block exchange -- so the exchange runs on a one-GPU box exactly
    as it does on eight (init_from_env then creates the one-rank group)."""
    return os.environ.get("LMI_FORCE_EXCHANGE") == "1"


def init_from_env(backend: Optional[str] = None):
    """torchrun-style init (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); 127.0.0.1.
    One rank: no process group, unless LMI_FORCE_EXCHANGE=1 (a one-rank
    group, backend nccl = RCCL on a GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and not force_exchange():
        return rank, world, local
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if world == 1 and "MASTER_PORT" not in os.environ:
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        sk.close()
    os.environ.setdefault("MASTER_PORT", "29517")
    if backend is None:
        # LMI_DIST_BACKEND=gloo: control-flow rehearsal of several ranks on one
        # GPU (RCCL refuses two ranks on one device); collectives then stage
        # through host memory (_all_gather).  The product path is RCCL.
        backend = os.environ.get("LMI_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl" or torch.cuda.is_available():
        # the rank's own GPU (gloo ranks too: on a 1-GPU rehearsal LOCAL_RANK
        # is 0 for every rank)
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        # a rank that dies or raises inside a collective must not leave the
        # others waiting forever: past this timeout the process group's
        # watchdog aborts the waiting ranks (non-zero exit, no hang)
        import datetime
        timeout = datetime.timedelta(seconds=float(os.environ.get("LMI_DIST_TIMEOUT_S", "300")))
        dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=timeout)
    return rank, world, local


def rank_world(group=None):
    """(rank, world) of an initialised process group, else (0, 1)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def is_writer(group=None) -> bool:
    """True on the rank that writes files (results, pickles): rank 0 of an
    initialised process group, or the only process."""
    return rank_world(group)[0] == 0


def gpus_arg(argv, flag: str = "--gpus") -> int:
    """The value of `--gpus N` / `--gpus=N` in argv (1 when absent), read
    before argparse so a launcher can start its ranks before any GPU call."""
    for i, a in enumerate(argv):
        if a == flag and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith(flag + "="):
            return int(a.split("=", 1)[1])
    return 1


def launch_ranks(n: int, argv, script: str, relay_stdout: bool = True) -> int:
    """Start n rank processes of `script` (one GPU each) without a launcher:
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in every child's env, LOCAL_RANK
    = rank mod the visible device count (on a 1-GPU box with
    LMI_DIST_BACKEND=gloo the ranks share device 0, a control-flow rehearsal).
    With `relay_stdout` rank 0's stdout is captured and relayed when the ranks
    end (bench.py's single JSON line) and the other ranks' is dropped;
    otherwise every child inherits this process's streams.  Returns the first
    failing rank's exit code (the other ranks are then stopped: they would
    wait at a collective), else 0.  This process never initialises the GPU
    (it only counts devices) and never execs: the ranks are children."""
    import socket
    import subprocess
    import sys
    import time
    ndev = max(1, torch.cuda.device_count())
    if n > ndev and os.environ.get("LMI_DIST_BACKEND") != "gloo":
        print(f"[launch] {n} ranks but {ndev} visible GPU(s): RCCL needs one GPU per rank "
              f"(LMI_DIST_BACKEND=gloo rehearses the ranks on shared devices)", file=sys.stderr)
        return 2
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    # rank 0's stdout goes to an unlinked temporary file, read back when the
    # ranks end: a pipe read only then would block a rank 0 that writes more
    # than the pipe buffer
    import tempfile
    out0 = tempfile.TemporaryFile() if relay_stdout else None
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r % ndev), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = (out0 if r == 0 else subprocess.DEVNULL) if relay_stdout else None
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env, stdout=out))
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c
                for o in live:
                    procs[o].terminate()
        time.sleep(0.05)
    if relay_stdout:
        out0.seek(0)
        sys.stdout.write(out0.read().decode(errors="replace"))
        sys.stdout.flush()
        out0.close()
    return rc


def _all_gather(out: torch.Tensor, part: torch.Tensor, group=None):
    """all_gather_into_tensor; device tensors go through host copies on gloo."""
    if part.is_cuda and dist.get_backend(group) == "gloo":
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, part.cpu(), group=group)
        out.copy_(h)
        return
    dist.all_gather_into_tensor(out, part, group=group)


def all_gather_lists(d: torch.Tensor, pos: torch.Tensor, group=None,
                     status: Optional[torch.Tensor] = None):
    """[nq, R, k] per rank -> [G, nq, R, k] on every rank, in ONE collective:
    the distances (float32 or float64) travel bit for bit as int32 words beside
    the positions, and the rank's device status word (lmi_bucket_topk's
    LMI_STATUS_* bits) rides along, so every rank sees every rank's status
    and all ranks fail together (returned as [G] int32 when given)."""
    G = dist.get_world_size(group)
    parts = [d.contiguous().view(torch.int32).reshape(-1),
             pos.to(torch.int32).contiguous().reshape(-1)]
    if status is not None:
        parts.append(status.to(torch.int32).reshape(-1)[:1])
    flat = torch.cat(parts)
    out = torch.empty((G * flat.numel(),), dtype=torch.int32, device=flat.device)
    _all_gather(out, flat, group)
    out = out.view(G, flat.numel())
    nd, npos = parts[0].numel(), parts[1].numel()
    gd = out[:, :nd].contiguous().view(d.dtype).view((G,) + tuple(d.shape))
    gp = out[:, nd:nd + npos].contiguous().view((G,) + tuple(pos.shape)).to(pos.dtype)
    if status is None:
        return gd, gp
    return gd, gp, out[:, nd + npos]


def gather_merge(d: torch.Tensor, pos: torch.Tensor, k: int, group=None,
                 merge: Optional[Callable] = None, status: Optional[torch.Tensor] = None):
    """All-gather the shard lists and merge them (K3 on the GPU by default).

    `merge(gd, gp, k) -> (d, pos)` can be swapped for a CPU checker in the
    gloo tests; the product path always uses lmi_merge_topk(_f64).  With
    `status`, returns a third value: the OR of every rank's status word."""
    got = all_gather_lists(d, pos, group, status)
    gd, gp = got[0], got[1]
    if merge is None:
        from .index import merge_topk
        md, mp = merge_topk(gd, gp, k)
    else:
        md, mp = merge(gd, gp, k)
    if status is None:
        return md, mp
    st = got[2][0:1].clone()
    for g in range(1, got[2].shape[0]):
        st = torch.bitwise_or(st, got[2][g:g + 1])
    return md, mp, st


def packed_lists(rows: int, k: int, f64: bool, device):
    """This rank's send buffer for gather_merge_packed and views of it:
    (buf int32 [W], d [rows*k] f32/f64, pos [rows*k] int32, status [1] int32,
    zeroed).  K2 writes its lists and status word straight into the views,
    so the all-gather sends the buffer as it is (W = lmi_packed_rank_words)."""
    from . import _lib
    W = int(_lib.load().lmi_packed_rank_words(rows, k, int(bool(f64))))
    buf = torch.empty((W,), dtype=torch.int32, device=device)
    n = rows * k
    nd = n * (2 if f64 else 1)
    d = buf[:nd].view(torch.float64 if f64 else torch.float32)
    pos = buf[nd:nd + n]
    status = buf[nd + n:nd + n + 1]
    status.zero_()
    return buf, d, pos, status


def unpack_gathered(out: torch.Tensor, G: int, rows: int, k: int, f64: bool):
    """Views of a gathered packed buffer [G * W] int32: (d [G, rows, k]
    f32/f64, pos [G, rows, k] int32, status [G] int32) -- the layout
    lmi_merge_topk_packed reads in place."""
    W = out.numel() // G
    o = out.view(G, W)
    n = rows * k
    nd = n * (2 if f64 else 1)
    d = o[:, :nd].contiguous().view(torch.float64 if f64 else torch.float32).view(G, rows, k)
    return d, o[:, nd:nd + n].reshape(G, rows, k), o[:, nd + n]


def gather_merge_packed(buf: torch.Tensor, rows: int, k: int, f64: bool, group=None,
                        status_out: Optional[torch.Tensor] = None, merge: Optional[Callable] = None):
    """All-gather every rank's packed buffer (packed_lists) in one collective,
    then K3 over the gathered buffer in place (lmi_merge_topk_packed): the
    merged lists [rows, k] and the OR of every rank's status word, so all
    ranks fail together.  Two launches at any G (gather_merge's unpacking
    copies and per-rank status ORs are ~10 small kernels at G = 8).
    `merge(gd, gp, k) -> (d, pos)` replaces K3 in the CPU gloo tests (the
    gathered buffer is then unpacked with unpack_gathered)."""
    from . import _lib
    from .index import check, ptr
    G = dist.get_world_size(group)
    W = buf.numel()
    out = torch.empty((G * W,), dtype=torch.int32, device=buf.device)
    _all_gather(out, buf, group)
    if merge is not None:
        gd, gp, gs = unpack_gathered(out, G, rows, k, f64)
        md, mp = merge(gd, gp, k)
        st = gs[0:1].clone()
        for g in range(1, G):
            st = torch.bitwise_or(st, gs[g:g + 1])
        if status_out is not None:
            status_out.copy_(st)
            st = status_out
        return md.reshape(rows, k), mp.reshape(rows, k), st
    md = torch.empty((rows, k), dtype=torch.float64 if f64 else torch.float32, device=buf.device)
    mp = torch.empty((rows, k), dtype=torch.int32, device=buf.device)
    st = status_out if status_out is not None else torch.empty((1,), dtype=torch.int32,
                                                               device=buf.device)
    check("lmi_merge_topk_packed", _lib.load().lmi_merge_topk_packed(
        ptr(out), G, W, rows, k, int(bool(f64)), ptr(md), ptr(mp), ptr(st),
        _lib.stream_handle(buf.device)))
    return md, mp, st


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
