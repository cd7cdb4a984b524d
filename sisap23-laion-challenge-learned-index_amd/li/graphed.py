"""The search step captured once as a HIP graph and replayed per batch
(Searcher.graph -> GraphedSearch): the per-batch step of bench.py --no-stream
and the batch stream's fallback for batches it cannot take."""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._host import capture_underway, host_array, no_gc_capture, np_fp16_exact, release_later, \
    stage_rows_f16, stage_rows_f32, wait_event_with_deadline, wait_with_deadline
from .index import _SEED_ROUND0, _as_torch, answer_buffer, answer_views, replay_device


def _f32_exact(x: np.ndarray) -> bool:
    """False for float64 values that float32 would change."""
    if x.dtype != np.float64:
        return True
    return bool(np.array_equal(x.astype(np.float32).astype(np.float64), x))


class GraphedSearch:
    """One search step captured once as a HIP graph and replayed per batch,
    from queries in HOST memory to the answer in host memory, as the
    reference's timer sees it (search.py:116-141; its queries are host arrays,
    search.py:49, :85-87):

        H2D of the staged batch (pinned host rows)
        -> router (K1) -> scan (K2) [-> all-gather + K3] -> replay (K4)
        -> D2H of the answer and of both status words

    The ~25 launches and the copies go to the GPU as one graph launch, with no
    host work between them.

    Staging (`stage`, outside the step, like the reference's h5 loads before
    its timer): the batch is written into a pinned host buffer laid out per
    rank block as [pca96 f32 (per x 96) | clip768 (per x d) | classes (per x
    R, G > 1 only)].  The clip768 rows are staged as fp16 when the index is
    fp16 and every query value is fp16-representable (checked on the host at
    staging; float16 input is exact by construction): half the bytes over
    PCIe, widened to float32 on the device.  A batch that is not fp16-exact
    under an fp16 capture is answered by the eager path instead.

    G > 1 ranks: rank g uploads only its block (1/G of the batch), routes its
    queries into the block's classes, and ONE all-gather over xGMI hands every
    rank the whole batch and all classes; then the striped scan and the list
    exchange as in Searcher.search.

    The graph owns its scan workspace (index._ws may be replaced by a later
    eager call with a bigger batch).  `run()` returns numpy views
    of the graph's pinned output buffer, valid until the next run."""

    def __init__(self, searcher: "Searcher", q_nav, q_search, R: int,
                 k: int = 10, *, k_round: int = 10, use_threshold: bool = True, dist: str = "f32",
                 capture: bool = True, pipeline: bool = False):
        s = searcher
        ix = s.index
        dev = ix.device
        lib = _lib.load()
        self.searcher, self.R, self.k, self.k_round = s, R, k, k_round
        self.use_threshold, self.dist = use_threshold, dist
        # X: the exchange branch (Searcher.exchange: G > 1 ranks, or a one-rank
        # group under LMI_FORCE_EXCHANGE=1)
        X = s.exchange
        if k_round > _lib.LMI_MAX_K or (capture and X and
                                       torch.distributed.get_backend(s.group) != "nccl"):
            raise ValueError("graph capture needs k_round <= 16 and RCCL collectives "
                             "(capture=False runs the same step eagerly, e.g. over gloo)")
        nav = host_array(q_nav)
        qs = host_array(q_search)
        nq, d, dn = int(qs.shape[0]), ix.d, int(nav.shape[1])
        if qs.shape != (nq, d) or nav.shape[0] != nq:
            raise ValueError("query shapes do not match the index")
        if not _f32_exact(qs):
            # the staged rows are float32 at most; float64 queries that float32
            # changes are answered from their float64 values by Searcher.search
            # (lmi_bucket_topk_f64q), which the graph cannot reproduce
            raise ValueError("float64 queries not exact in float32: use Searcher.search")
        self.nq, self.d, self.dn = nq, d, dn
        # the batch's precision class is decided on the host, once per capture
        self.f16_up = ix.storage == "f16" and d % 2 == 0 and (
            qs.dtype == np.float16 or np_fp16_exact(qs))
        self.qmode = _lib.LMI_Q_F16 if self.f16_up else _lib.LMI_Q_F32
        f64 = dist == "f64"
        # the batch is shared over the ranks of the process group (the index's
        # world is the stripe count; they differ only in a one-process
        # rehearsal of one stripe, tools/shard_step.py)
        G = torch.distributed.get_world_size(s.group) if X else 1
        g = torch.distributed.get_rank(s.group) if X else 0
        self.per = per = -(-nq // G)
        self.wq = wq = d // 2 if self.f16_up else d          # int32 words per staged row
        self.bw = bw = per * dn + per * wq + (per * R if X else 0)
        pin = torch.cuda.is_available()
        self.bw_all = bw
        # pipeline: one pinned staging buffer per slot, so the host stages the
        # next batch while the current one is uploaded and searched (stream())
        self.pipeline = bool(pipeline) and capture
        self.h_blks = [torch.zeros((G, bw), dtype=torch.int32, pin_memory=pin)
                       for _ in range(2 if self.pipeline else 1)]
        self.h_blk = self.h_blks[0]
        self._staged = [None] * len(self.h_blks)
        self._slot = 0
        if not self.stage(nav, qs, slot=0):
            raise ValueError("staging failed")
        if self.pipeline:
            self.h_blks[1].copy_(self.h_blks[0])
            self._staged[1] = self._staged[0]
        need = (lib.lmi_scan_f64_workspace_bytes if f64 else lib.lmi_scan_workspace_bytes)(
            C.byref(ix.desc_for(k_round)), nq, R, k_round, self.qmode)
        self.ws = torch.empty(max(int(need), 256), dtype=torch.uint8, device=dev)
        # pipeline: two device copies of the staged block, each with its own
        # captured graph; the upload of a slot's block runs on a copy stream
        # beside the other slot's step (the upload leaves the graph)
        self.d_blks = [torch.empty((bw,), dtype=torch.int32, device=dev)
                       for _ in range(2 if self.pipeline else 1)]
        self.d_blk = self.d_blks[0]
        self.d_all = torch.empty((G, bw), dtype=torch.int32, device=dev) if X else None
        self.q32 = torch.empty((G * per, d), dtype=torch.float32, device=dev) \
            if (self.f16_up or X) else None
        self.cls = torch.empty((G * per, R), dtype=torch.int32, device=dev) if X else None
        bsz, p2id = s._device_tables()
        self.w = k_round if R == 1 else k
        self.rank_in_group = g
        self.G, self.X = G, X
        # collectives inside a replayed graph are GPU work the process group's
        # watchdog does not track: run() bounds its own wait instead
        self.timeout_s = float(os.environ.get("LMI_DIST_TIMEOUT_S", "300"))
        # (on its own hardware queue: a copy stream on the step's queue would
        # wait for the step it should run beside; li.stream.queue_streams)
        from .stream import queue_streams
        copy_stream = queue_streams(dev, 1)[0]

        def step(slot=0):
            ans = answer_buffer(nq, self.w, dev)
            main = torch.cuda.current_stream(dev)
            d_blk = self.d_blks[slot]
            if not X:
                if not self.pipeline:
                    # pca96 rows first; the clip768 rows come in on a second
                    # stream while the router runs
                    d_blk[:per * dn].copy_(self.h_blk[0, :per * dn], non_blocking=True)
                    copy_stream.wait_stream(main)
                    with torch.cuda.stream(copy_stream):
                        d_blk[per * dn:].copy_(self.h_blk[0, per * dn:], non_blocking=True)
                classes = s.router.topr(d_blk[:per * dn].view(torch.float32).view(per, dn), R)[0]
                if not self.pipeline:
                    main.wait_stream(copy_stream)
                sv = d_blk[per * dn:per * dn + per * wq]
                if self.f16_up:
                    q = self.q32
                    q.copy_(sv.view(torch.float16).view(per, d))
                else:
                    q = sv.view(torch.float32).view(per, d)
            else:
                # this rank's block: upload, route its queries into the block,
                # one all-gather of every block (queries + classes)
                from .dist import _all_gather
                if not self.pipeline:
                    d_blk.copy_(self.h_blk[g], non_blocking=True)
                s.router.topr(d_blk[:per * dn].view(torch.float32).view(per, dn), R,
                              out=d_blk[per * (dn + wq):])
                _all_gather(self.d_all.view(-1), d_blk, s.group)
                sv = self.d_all[:, per * dn:per * (dn + wq)]
                if self.f16_up:
                    self.q32.view(G, per, d).copy_(sv.view(torch.float16).view(G, per, d))
                else:
                    self.q32.view(G, per, d).copy_(sv.view(torch.float32).view(G, per, d))
                self.cls.view(G, per, R).copy_(self.d_all[:, per * (dn + wq):].view(G, per, R))
                q = self.q32[:nq]
                classes = self.cls[:nq]
            d_, pos, _ = s._scan(q, classes, k_round, self.qmode, f64, status_out=ans[3][0:1],
                                 ws=self.ws, seed_round0=use_threshold and k <= k_round and _SEED_ROUND0)
            replay_device(classes, d_, pos, k_round=k_round, k_final=k, bucket_size=bsz,
                          pos_to_id=p2id, use_threshold=use_threshold,
                          out=(ans[1], ans[2], ans[3][1:2]))
            return ans[0]

        # warm up on a side stream (allocations, kernel attributes, RCCL
        # communicators), then capture.  G > 1: the ranks agree that every
        # rank's warm-up succeeded before any rank captures (a rank that
        # raised before entering a collective would otherwise leave the others
        # waiting in the next one; a rank that fails inside a collective is
        # ended by the process group's timeout, li.dist.init_from_env)
        self._step = None
        if not capture:
            # the same step, launched eagerly per run (the multi-process gloo
            # rehearsal of the sharded upload on one GPU: tests/test_gpu_dist.py)
            buf = step()
            torch.cuda.synchronize(dev)
            self.h = torch.empty(tuple(buf.shape), dtype=torch.int32, pin_memory=True)
            self.graph = None
            self._step = step
            return
        self._cs = copy_stream
        if self.pipeline:
            self._up_ev = [torch.cuda.Event() for _ in range(2)]
            self._done_ev = [torch.cuda.Event() for _ in range(2)]
            for slot in range(2):
                self.d_blks[slot].copy_(self.h_blks[slot][g], non_blocking=True)
            torch.cuda.synchronize(dev)
        slots = (0, 1) if self.pipeline else (0, 0)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        err = None
        try:
            with torch.cuda.stream(side):
                for slot in slots:
                    buf = step(slot)
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
        except Exception as e:  # noqa: BLE001 (re-raised below on every rank)
            err = e
        if X:
            ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
            torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN, group=s.group)
            if int(ok.item()) == 0:
                raise RuntimeError(f"graph warm-up failed on some rank: {err!r}")
        elif err is not None:
            raise err
        # one pinned answer buffer per graph: with launch() / result() a graph
        # may run while the host reads the other's answer
        self.hs = [torch.empty(tuple(buf.shape), dtype=torch.int32, pin_memory=True)
                   for _ in range(2 if self.pipeline else 1)]
        self.h = self.hs[0]
        self.graphs, self._keep = [], []
        with no_gc_capture():   # (li._host "graph lifetime")
            for slot in range(2 if self.pipeline else 1):
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                    buf = step(slot)
                    self.hs[slot].copy_(buf, non_blocking=True)
                self.graphs.append(gr)
                self._keep.append(buf)
        self.graph = self.graphs[0]
        self._slot = 0
        self._fresh = [True, True]   # d_blks[slot] holds the staged batch
        # upload the staged batch into the idle slot while a step runs (a batch
        # replayed again, run() without arguments); off once run() stages
        self._prefetch = True
        torch.cuda.synchronize(dev)

    def close(self):
        """Wait for this object's launches and uploads still in flight
        (pipeline=True: launch() returns before its step ends), then release
        the captured graphs and their memory pools (li.stream.StreamedSearch.
        close: a graph destroyed while queued leaves the GPU reading freed
        kernel arguments).  Idempotent."""
        if getattr(self, "graphs", None) is None:
            return
        if capture_underway():
            release_later(self.graphs, self._keep, self.ws)
        else:
            for name in ("_done_ev", "_up_ev"):
                for e in getattr(self, name, ()):
                    e.synchronize()
            self._cs.synchronize()
        self.graphs, self.graph = None, None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown: torch may be gone)
            pass

    def stage(self, q_nav, q_search, slot: Optional[int] = None) -> bool:
        """Write a batch (host or device arrays of the captured shape) into the
        pinned staging buffer of `slot` (default: the slot the next run or
        launch replays).  False if it cannot be staged in the captured
        precision (clip768 values not fp16-representable under an fp16
        capture): run() then answers it on the eager path."""
        nav = host_array(q_nav)
        qs = host_array(q_search)
        nq, d, dn, per, wq = self.nq, self.d, self.dn, self.per, self.wq
        if nav.shape != (nq, dn) or qs.shape != (nq, d):
            raise ValueError("a staged batch must have the captured shape")
        if not _f32_exact(qs):
            return False  # float64 values float32 would change: the eager path
        if slot is None:
            slot = self._slot
        if self.pipeline and getattr(self, "_fresh", None) is not None:
            # an upload may still read the pinned buffer; both device copies
            # are stale from now on (a launch runs the last staged batch)
            for e in self._up_ev:
                e.synchronize()
            self._fresh = [False, False]
        # every rank block, on the host cores (every rank stages the whole
        # batch, so all ranks decide its precision class alike)
        blk = self.h_blks[slot].numpy()
        ok = True
        for g in range(blk.shape[0]):
            lo, hi = min(nq, g * per), min(nq, (g + 1) * per)
            stage_rows_f32(blk[g, :(hi - lo) * dn].view(np.float32).reshape(hi - lo, dn), nav[lo:hi])
            sv = blk[g, per * dn:per * dn + (hi - lo) * wq]
            if self.f16_up:
                ok &= stage_rows_f16(sv.view(np.float16).reshape(hi - lo, d), qs[lo:hi])
            else:
                stage_rows_f32(sv.view(np.float32).reshape(hi - lo, d), qs[lo:hi])
        if not ok:
            # not fp16-exact under an fp16 capture: put the slot's last staged
            # batch back (run() without arguments replays it) and answer eagerly
            last = getattr(self, "_last", slot)
            if self._staged[slot] is not None:
                self.stage(*self._staged[slot], slot=slot)
            self._last = last
            return False
        self._staged[slot] = (nav, qs)
        self._last = slot
        return True

    def upload_bytes(self) -> int:
        """Bytes this rank moves host -> device per step."""
        per, dn, wq = self.per, self.dn, self.wq
        return 4 * per * (dn + wq)

    def run(self, q_nav=None, q_search=None):
        """Replay the step (after staging a new batch, if given) -> (dists f64
        [nq, w], anns uint32 [nq, w])."""
        s = self.searcher
        dev = s.index.device
        if self.graph is None and self._step is None:
            raise RuntimeError("GraphedSearch: run() after close()")
        if q_nav is not None or q_search is not None:
            if q_nav is None or q_search is None:
                raise ValueError("stage both q_nav and q_search")
            # a caller that stages per run replaces the host batch before the
            # next run: uploading this one into the other slot ahead would be
            # wasted PCIe traffic, so the prefetch is off from now on
            self._prefetch = False
            if not self.stage(q_nav, q_search):
                return self._eager(q_nav, q_search)
        if self.pipeline:
            return self.result(self.launch())
        elif self.graph is not None:
            self.graph.replay()
        else:
            self.h.copy_(self._step(), non_blocking=True)
        if self.X and self.graph is not None:
            wait_with_deadline(dev, self.timeout_s)
        else:
            torch.cuda.current_stream(dev).synchronize()
        return self._answer(self.h)

    def stream(self, batches):
        """Answer an iterable of (q_nav, q_search) batches in order, yielding
        (dists, anns) copies per batch.  pipeline=True: batch i + 1 is staged
        on the host cores and uploaded on the copy stream while batch i's step
        runs, and its step is enqueued behind it before batch i's answer is
        read (two steps in flight); otherwise one run() per batch.  A batch
        that cannot be staged is answered by Searcher.search, in order."""
        if not self.pipeline:
            for b in batches:
                yield tuple(a.copy() for a in self.run(*b))
            return
        self._prefetch = False
        pending = None
        for b in batches:
            if not self.stage(*b):
                if pending is not None:
                    yield tuple(a.copy() for a in self.result(pending))
                    pending = None
                yield self._eager(*b)
                continue
            t = self.launch()
            if pending is not None:
                yield tuple(a.copy() for a in self.result(pending))
            pending = t
        if pending is not None:
            yield tuple(a.copy() for a in self.result(pending))

    def _answer(self, h):
        hd, ha, st, rst = answer_views(h, self.nq, self.w)
        if st & _lib.LMI_STATUS_INTERNAL or rst:
            raise RuntimeError(f"search: internal status {st}/{rst}")
        return hd, ha

    def launch(self) -> int:
        """pipeline=True: enqueue one step on the staged batch without waiting
        for it (the next batch's upload starts beside it); returns a ticket for
        result().  Keeping one launch ahead of result() hides the host's
        synchronise-to-launch gap between steps (at most two in flight: a
        ticket's answer is valid until the launch after next)."""
        if not self.pipeline:
            raise ValueError("launch() needs GraphedSearch(pipeline=True)")
        slot = self._slot
        self._run_pipelined(self.searcher.index.device)
        return slot

    def result(self, ticket: int):
        """Wait for the step of `ticket` (from launch()) -> (dists f64 [nq, w],
        anns uint32 [nq, w]): numpy views of that step's pinned answer."""
        ev = self._done_ev[ticket]
        if self.X:
            wait_event_with_deadline(ev, self.timeout_s)
        else:
            ev.synchronize()
        return self._answer(self.hs[ticket])

    def _upload(self, slot):
        """The staged block into d_blks[slot] on the copy stream, once the
        graph that last read that copy has finished."""
        cs = self._cs
        cs.wait_event(self._done_ev[slot])
        with torch.cuda.stream(cs):
            self.d_blks[slot].copy_(self.h_blks[self._last][self.rank_in_group], non_blocking=True)
        self._up_ev[slot].record(cs)
        self._fresh[slot] = True

    def _run_pipelined(self, dev):
        """Replay the current slot's graph; meanwhile upload the staged batch
        into the other slot for the next run when it will replay the same
        staged batch (the copy engine moves it while this step searches).  A
        caller that stages a new batch per run (run(q_nav, q_search)) uploads
        each batch into its slot just before that slot's replay: then the H2D
        is inside the step, not beside the previous one."""
        main = torch.cuda.current_stream(dev)
        slot = self._slot
        if not self._fresh[slot]:
            self._upload(slot)
        main.wait_event(self._up_ev[slot])
        self.graphs[slot].replay()
        self._done_ev[slot].record(main)
        self._fresh[slot] = False
        nxt = 1 - slot
        if not self._fresh[nxt] and self._prefetch:
            self._upload(nxt)
        self._slot = nxt

    def _eager(self, q_nav, q_search):
        dev = self.searcher.index.device
        self.searcher._qcheck = None
        # (float64 queries keep their dtype: Searcher.search answers them from
        # their float64 values, as the reference's float64 arithmetic does)
        qs = host_array(q_search)
        return self.searcher.search(_as_torch(host_array(q_nav), dev, torch.float32),
                                    _as_torch(qs, dev, torch.float64 if qs.dtype == np.float64
                                              else torch.float32),
                                    self.R, k=self.k, k_round=self.k_round,
                                    use_threshold=self.use_threshold, dist=self.dist)
