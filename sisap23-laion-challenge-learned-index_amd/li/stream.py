"""The batch stream: query batches through the search step as a four-stage
pipeline of captured graphs (Searcher.streamed -> StreamedSearch; the bench's
default step, DESIGN.md §5 "The batch stream").

The reference answers one host-resident batch per call (search.py:116-141;
its queries are host arrays, search.py:49, :85-87).  A server answers a
stream of such batches, and on a GPU the work of one batch -- H2D, router,
K2's plan, K2's scan, K2's chunk merge, the replay, D2H -- is one long
MFMA-bound scan between latency-bound chains.  Here every launch runs:

    R  batch t:   H2D of this rank's block of its staged host rows (copy
                  engine) -> router (K1)
    P  batch t:   the queries widened, K2's PLAN phase (fragments and norms,
                  the tile plan, the seed map, the tail split, the bounds)
    S  batch t-2: K2's SCAN phase (planned two launches earlier)
    F  batch t-3: K2's MERGE phase (+ the float64 refinement)
                  [-> all-gather + K3 at G > 1] -> replay (K4) -> D2H

on four streams ordered by per-slot events, and returns the answer of the
batch it finished; every batch passes every stage (the same kernels as
Searcher.search), so each answer equals Searcher.search of its batch bit for
bit.  The persistent scan holds every CU while it runs, so the R, P and F
chains start in its tail; the next launch's scan, enqueued ahead, waits on
the device for this launch's F, so the scans run back to back.

G > 1 ranks (the corpus striped, li.dist): each rank stages and uploads only
its block of the batch (1/G of the rows: the host-memory traffic of a new
batch does not grow with G) and routes it; the one collective per launch, in
F, all-gathers every rank's [lists of batch t-3 | query block and classes of
batch t] buffer, so the list exchange carries the next batch's queries.  F is
then three graphs: F1 (the merge phase, as soon as the scan is done), FX (the
all-gather, once batch t's block is routed), after which P of batch t unpacks
the gathered queries beside F2 (K3 + replay + D2H)."""
from __future__ import annotations

import ctypes as C
import os
import time
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._host import capture_underway, host_array, no_gc_capture, release_later, stage_rows_f16, \
    stage_rows_f32, wait_event_with_deadline
from .index import _SEED_ROUND0, answer_buffer, answer_views, bucket_topk, bucket_topk_f64, \
    global_band, replay_device


def _runs_beside(a, b, spin, wait_s):
    """True if a kernel on stream `b` finishes while a spinning one on stream
    `a` still runs (the two streams are on different hardware queues)."""
    ea, eb = torch.cuda.Event(), torch.cuda.Event()
    with torch.cuda.stream(a):
        torch.cuda._sleep(spin)
    ea.record(a)
    with torch.cuda.stream(b):
        torch.cuda._sleep(1)
    eb.record(b)
    t0 = time.perf_counter()
    beside = False
    while time.perf_counter() - t0 < wait_s:
        if eb.query():
            beside = not ea.query()
            break
    ea.synchronize()
    eb.synchronize()
    return beside


def _spin_cycles(stream, ms_target: float) -> int:
    """torch.cuda._sleep's argument (device clock cycles) for a spin of at
    least `ms_target` ms on `stream`, measured."""
    spin, ms = 1 << 18, 0.0
    while ms < ms_target / 2 and spin < (1 << 34):
        spin *= 4
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        with torch.cuda.stream(stream):
            torch.cuda._sleep(spin)
        e1.record(stream)
        e1.synchronize()
        ms = e0.elapsed_time(e1)
    return int(spin * max(1.0, ms_target / max(ms, 1e-3)))


def queue_streams(dev, n: int):
    """`n` new streams of `dev` whose work runs beside the current stream's
    and beside each other's.  HIP maps the streams of a process onto
    GPU_MAX_HW_QUEUES (4) hardware queues and serialises the streams that
    share one: a finish stream that lands on the scan's queue waits for the
    next scan instead of running in its tail (a float64 stream step measured
    636 µs between scans that way against 196 for float32, whose finish
    stream had landed elsewhere).  Each candidate stream is
    tested with a spinning kernel on the others (≈ 10 ms per test); with
    fewer free queues the rest share.  Every caller gets streams of its own:
    a stream the graphs of an object still alive (or not yet collected) were
    launched on is not handed out again on purpose."""
    dev = torch.device(dev)
    main = torch.cuda.current_stream(dev)
    spin, wait_s = _spin_cycles(main, 10.0), 5e-3
    have, tries = [], 0
    while len(have) < n and tries < 4 * n + 4:
        s = torch.cuda.Stream(dev)
        tries += 1
        if all(_runs_beside(o, s, spin, wait_s) for o in [main] + have):
            have.append(s)
    while len(have) < n:
        have.append(torch.cuda.Stream(dev))
    return have


def stream_reserve() -> int:
    """The default `reserve_cus` of a StreamedSearch: LMI_STREAM_RESERVE if set,
    else 0.  Measured (10M, W = 1, profiles/r06p_reserve_ab.txt): leaving 2,
    4 or 8 CUs to the finish made the float32 step 7.41-7.47 ms against
    7.20-7.25 with none -- the route, the plan and the finish of a launch then
    share those few CUs and outlast the ~7 ms scan -- and at W = 8 (a ~1 ms
    stripe scan) 1.34-1.51 against 1.26 ms (profiles/r06o_*); float64 and
    the split mode's finish are heavier still."""
    env = os.environ.get("LMI_STREAM_RESERVE")
    return int(env) if env is not None else 0


class QueryNotF16(RuntimeError):
    """A streamed batch held clip768 values that fp16 cannot represent: the
    phased scan (fp16 MFMA) cannot answer it; Searcher.search can (exact fp32
    MFMA).  Raised on every rank at the same launch (the flag rides the
    gathered blocks into the scan's status word)."""


class StreamedSearch:
    """See the module docstring.  `capture=False` launches the same stage
    functions eagerly (the gloo rehearsal of the G > 1 path: gloo cannot be
    captured).  `lookahead` (default True): the next launch's scan is enqueued
    at the end of each launch, waiting on the device for its plan (one launch
    earlier) and, unless `reserve_cus` > 0, for this launch's F; False
    enqueues each scan at the start of its own launch.  `reserve_cus` (None:
    stream_reserve's default): CUs the scan's persistent grid leaves to the
    finish chain, which then runs beside the next scan.  fp16 index and
    fp16-exact query batches (the phased scan
    is the fp16 scan; other batches go through Searcher.search), or the split
    mode (storage f32x, k_round <= 10, float32 batches: its SCAN phase is the
    sample scan, the bound and the collect scan, its MERGE phase the exact
    re-score; ABI 11)."""

    NS = 4

    def __init__(self, searcher, q_nav, q_search, R: int, k: int = 10, *,
                 k_round: int = 10, use_threshold: bool = True, dist: str = "f32",
                 capture: bool = True, lookahead: bool = True, kth_peers=None,
                 reserve_cus: Optional[int] = None):
        s = searcher
        ix = s.index
        dev = ix.device
        lib = _lib.load()
        self.searcher, self.R, self.k, self.k_round = s, R, k, k_round
        self.use_threshold, self.dist = use_threshold, dist
        # the list exchange spans the process group's ranks (Searcher.exchange;
        # a stripe of a G-way index in a process without a group: the rank's
        # own lists).  X: the exchange branch -- G > 1, or a one-rank group
        # under LMI_FORCE_EXCHANGE=1 (the same graphs, RCCL over one rank)
        self.X = X = s.exchange
        self.G = G = torch.distributed.get_world_size(s.group) if X else 1
        self.g = g = torch.distributed.get_rank(s.group) if X else 0
        if k_round > _lib.LMI_MAX_K:
            raise ValueError("the phased scan needs k_round <= 16")
        if capture and X and torch.distributed.get_backend(s.group) != "nccl":
            raise ValueError("graph capture needs RCCL collectives (capture=False runs the "
                             "stages eagerly, e.g. over gloo)")
        if lookahead not in (True, False):
            raise ValueError("lookahead must be True or False")
        nav, qs = host_array(q_nav), host_array(q_search)
        nq, d, dn = int(qs.shape[0]), ix.d, int(nav.shape[1])
        if qs.shape != (nq, d) or nav.shape[0] != nq:
            raise ValueError("query shapes do not match the index")
        # (the split mode, storage f32x: float32 batches, its phases need
        # k_round <= 10, ABI 11)
        self.split = split = ix.storage == "f32x"
        if split and k_round > 10:
            raise ValueError("the split mode's batch stream needs k_round <= 10")
        if not (split or (ix.storage == "f16" and d % 2 == 0)):
            raise ValueError("the batch stream needs an fp16 index with an even d, or the split mode")
        self.nq, self.d, self.dn = nq, d, dn
        f64 = dist == "f64"
        self.w = k_round if R == 1 else k
        kl = k_round
        NS, X = self.NS, self.X
        self.per = per = -(-nq // G)                 # rows of a rank's block
        self.lo, self.hi = min(nq, g * per), min(nq, (g + 1) * per)
        wq = d if split else d // 2                  # int32 words per fp16 (split: float32) row
        # a rank's block, int32 words: [pca96 f32 per*dn | clip768 f16 per*wq |
        # not-fp16 flag, pad | classes per*R (G > 1)]; stage() writes and the
        # H2D moves everything before the classes
        self.o_q, self.o_flag = per * dn, per * (dn + wq)
        self.o_cls = self.staged_words = self.o_flag + 2
        self.bw = self.o_cls + (per * R if X else 0)
        pin = torch.cuda.is_available()
        self.h_stage = [torch.zeros((self.bw,), dtype=torch.int32, pin_memory=pin) for _ in range(NS)]
        self.q32 = [torch.empty((G * per, d), dtype=torch.float32, device=dev) for _ in range(NS)]
        self.cls = [torch.empty((G * per, R), dtype=torch.int32, device=dev) for _ in range(NS)]
        wsb = (lib.lmi_scan_f64_workspace_bytes if f64 else lib.lmi_scan_workspace_bytes)(
            C.byref(ix.desc), nq, R, kl, _lib.LMI_Q_F16)
        self.ws = [torch.empty(max(int(wsb), 256), dtype=torch.uint8, device=dev) for _ in range(NS)]
        self.ans = [answer_buffer(nq, self.w, dev) for _ in range(NS)]
        self.h_ans = [torch.empty((3 * nq * self.w + 2,), dtype=torch.int32, pin_memory=pin)
                      for _ in range(NS)]
        ldt = torch.float64 if f64 else torch.float32
        if X:
            # exchange buffer j: [packed lists of slot j (lmi_packed_rank_words)
            # | the block of slot j-1]; gathered into xall[j] by F1 of slot j
            wl = int(lib.lmi_packed_rank_words(nq * R, kl, int(f64)))
            self.wl = wl
            self.W = W = wl + self.bw + (self.bw & 1)
            self.xb = [torch.zeros((W,), dtype=torch.int32, device=dev) for _ in range(NS)]
            self.xall = [torch.zeros((G * W,), dtype=torch.int32, device=dev) for _ in range(NS)]
            n = nq * R * kl
            nd = n * (2 if f64 else 1)
            self.lists = [(b[:nd].view(ldt).view(nq, R, kl), b[nd:nd + n].view(nq, R, kl),
                           b[nd + n:nd + n + 1]) for b in self.xb]
            self.d_blk = [self.xb[(j + 1) % NS][wl:wl + self.bw] for j in range(NS)]
        else:
            self.xb = self.xall = None
            self.d_blk = [torch.zeros((self.bw,), dtype=torch.int32, device=dev) for _ in range(NS)]
            self.lists = [(torch.empty((nq, R, kl), dtype=ldt, device=dev),
                           torch.empty((nq, R, kl), dtype=torch.int32, device=dev),
                           self.ans[j][3][0:1]) for j in range(NS)]
        bsz, p2id = s._device_tables()
        # the replay's workspace per slot: its GROUPS phase (every round's
        # groups, from the classes) runs in the plan stage, beside the scan;
        # its ROUNDS phase in the finish
        rwb = int(lib.lmi_replay_device_workspace_bytes(nq, R, kl, k_round, k, int(bsz.numel())))
        self.rws = [torch.empty(max(rwb, 256), dtype=torch.uint8, device=dev) for _ in range(NS)]
        seed = use_threshold and k <= k_round and _SEED_ROUND0
        scan_fn = bucket_topk_f64 if f64 else bucket_topk
        self.timeout_s = float(os.environ.get("LMI_DIST_TIMEOUT_S", "300"))
        NF = _lib.LMI_STATUS_QUERY_NOT_F16

        # float64 at G > 1 (ABI 10): the band decided over every rank's lists
        # -- the MERGE phase writes the pairs' k smallest d32 (kth), F1
        # all-gathers them (kall) before the REFINE phase, so each rank
        # refines only its rows of the merged band (Searcher._scan's form)
        # (`kth_peers`, measurement only: a one-rank rehearsal of one stripe
        # of a G'-rank index, tools/stream_steps.py -- the other stripes' kth
        # blocks of the batch, [G' - 1, nq*R*k], held beside the gathered one,
        # so the REFINE phase sees the G'-rank band)
        self.gband = gband = f64 and X and global_band(ix, nq, R, kl, _lib.LMI_Q_F16)
        Gk = G
        if gband:
            nk = nq * R * kl
            if kth_peers is not None:
                if G != 1 or tuple(kth_peers.shape[1:]) != (nk,):
                    raise ValueError("kth_peers needs a one-rank group and [G' - 1, nq*R*k] blocks")
                Gk = 1 + int(kth_peers.shape[0])
            self.kth = [torch.empty((nk,), dtype=torch.float32, device=dev) for _ in range(NS)]
            self.kall = [torch.empty((Gk * nk,), dtype=torch.float32, device=dev) for _ in range(NS)]
            if kth_peers is not None:
                for kall in self.kall:
                    kall[nk:].copy_(kth_peers.reshape(-1))

        def phase(j, ph, band_x=None):
            dl, pl, st = self.lists[j]
            kw = {} if band_x is None else {"band_x": band_x}
            scan_fn(ix, self.q32[j][:nq], self.cls[j][:nq], kl, qmode=_lib.LMI_Q_F16,
                    out=(dl, pl, st), ws=self.ws[j], seed_round0=seed, phases=ph, **kw)

        def upload(j):
            self.d_blk[j][:self.staged_words].copy_(self.h_stage[j][:self.staged_words],
                                                    non_blocking=True)

        def route(j):
            # (the staged rows are in d_blk[j]: upload(j) ran before, on the
            # copy stream in a launch); G > 1: this rank's block, its classes
            # into the block (gathered with it)
            blk = self.d_blk[j]
            nav_d = blk[:self.o_q].view(torch.float32).view(per, dn)
            if not X:
                s.router.topr(nav_d, R, out=self.cls[j])
            else:
                s.router.topr(nav_d, R, out=blk[self.o_cls:self.o_cls + per * R])

        def xgather(j):
            from .dist import _all_gather
            _all_gather(self.xall[j], self.xb[j], s.group)

        def plan(j):
            st = self.lists[j][2]
            qdt = torch.float32 if split else torch.float16
            if not X:
                blk = self.d_blk[j]
                self.q32[j].copy_(blk[self.o_q:self.o_flag].view(qdt).view(nq, d))
                # the scan's status word starts with the staged block's
                # not-fp16 flag (the scan only ORs bits into it)
                st.copy_(blk[self.o_flag:self.o_flag + 1])
            else:
                xa = self.xall[(j + 1) % NS].view(G, self.W)[:, self.wl:self.wl + self.bw]
                self.q32[j].view(G, per, d).copy_(
                    xa[:, self.o_q:self.o_flag].view(qdt).view(G, per, d))
                self.cls[j].view(G, per, R).copy_(xa[:, self.o_cls:].view(G, per, R))
                torch.amax(xa[:, self.o_flag:self.o_flag + 1], dim=0, out=st)
            phase(j, _lib.LMI_Q_PHASE_PLAN)
            _, ad, aa, ast = self.ans[j]
            replay_device(self.cls[j][:nq], None, None, k_round=k_round, k_final=k, bucket_size=bsz,
                          pos_to_id=p2id, use_threshold=use_threshold, out=(ad, aa, ast[1:2]),
                          phases=_lib.LMI_REPLAY_PHASE_GROUPS, ws=self.rws[j], k_list=kl)

        def scan(j):
            if not self.scan_wgs:
                phase(j, _lib.LMI_Q_PHASE_SCAN)
                return
            prev = lib.lmi_scan_set_workgroups(self.scan_wgs)
            try:
                phase(j, _lib.LMI_Q_PHASE_SCAN)
            finally:
                lib.lmi_scan_set_workgroups(prev)

        def finish1(j):
            if gband:
                from .dist import _all_gather
                phase(j, _lib.LMI_Q_PHASE_MERGE, band_x=(self.kth[j], None, G))
                _all_gather(self.kall[j][:G * self.kth[j].numel()], self.kth[j], s.group)
                phase(j, _lib.LMI_Q_PHASE_REFINE, band_x=(None, self.kall[j], Gk))
            else:
                phase(j, _lib.LMI_Q_PHASE_MERGE)

        def finish2(j):
            buf, ad, aa, ast = self.ans[j]
            # (the replay status word was zeroed by the plan's GROUPS phase)
            if X:
                dd = torch.empty((nq * R, kl), dtype=ldt, device=dev) if self._mdd[j] is None \
                    else self._mdd[j]
                pp = torch.empty((nq * R, kl), dtype=torch.int32, device=dev) if self._mpp[j] is None \
                    else self._mpp[j]
                self._mdd[j], self._mpp[j] = dd, pp
                _lib.check("lmi_merge_topk_packed", lib.lmi_merge_topk_packed(
                    _lib.ptr(self.xall[j]), G, self.W, nq * R, kl, int(f64), _lib.ptr(dd),
                    _lib.ptr(pp), _lib.ptr(ast[0:1]), _lib.stream_handle(dev)))
                dd, pp = dd.view(nq, R, kl), pp.view(nq, R, kl)
            else:
                dd, pp = self.lists[j][0], self.lists[j][1]
            replay_device(self.cls[j][:nq], dd, pp, k_round=k_round, k_final=k, bucket_size=bsz,
                          pos_to_id=p2id, use_threshold=use_threshold, out=(ad, aa, ast[1:2]),
                          phases=_lib.LMI_REPLAY_PHASE_ROUNDS, ws=self.rws[j])
            self.h_ans[j].copy_(buf, non_blocking=True)

        def finish(j):
            finish1(j)
            if X:
                xgather(j)
            finish2(j)

        self._mdd, self._mpp = [None] * NS, [None] * NS
        # (F1: the merge phase [float64: + the kth exchange and the REFINE
        # phase]; FX: the all-gather of slot j's lists with the next batch's
        # block, which waits for that block's route; F2: K3 + replay + D2H)
        self._f = dict(U=upload, R=route, X=xgather, P=plan, S=scan, F=finish, F1=finish1,
                       FX=xgather, F2=finish2)
        # four streams: the finish, the plan, the upload + route (the H2D on
        # the copy engine, then the router), and the scan on the caller's
        # stream, each on its own hardware queue (queue_streams); per-slot
        # events order them across launches
        self._fs, self._ps, self._rs = queue_streams(dev, 3)
        self._cs = self._rs
        ev = lambda: [torch.cuda.Event() for _ in range(NS)]
        self._up, self._rdone, self._pdone, self._sdone = ev(), ev(), ev(), ev()
        self._gdone, self._fdone = ev(), ev()
        self.graphs = None
        self._closed = False
        self._t = None  # launch counter once primed
        self.launches = 0  # step() calls so far (all primes)
        # measurement only: HIP events on the scan's stream around every scan
        # graph step() launches (the SCAN phase is the one scan kernel)
        self.time_scans = False
        self._scan_ev = []
        self.lookahead = lookahead
        # reserve_cus > 0: the scan's persistent grid leaves that many CUs to
        # the finish chain (lmi_scan_set_workgroups, ABI 12), and the
        # lookahead scan does not wait for this launch's finish (its slot is
        # not the finish's), so the finish runs beside the next scan instead
        # of between two scans (DESIGN.md §5 "The finish beside the scan")
        self.reserve_cus = r = stream_reserve() if reserve_cus is None else int(reserve_cus)
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        if not 0 <= r < ncu:
            raise ValueError(f"reserve_cus={r} outside [0, {ncu})")
        self.scan_wgs = ncu - r if r > 0 else 0
        self.overlap = r > 0
        self._s_ahead = False  # the next launch's scan is already enqueued
        for j in range(NS):
            if not self.stage(nav, qs, slot=j):
                raise ValueError("the batch stream needs fp16-exact query batches")
        # warm-up: one eager pass of every stage on every slot (allocations,
        # kernel attributes, communicators), in pipeline order, on a side
        # stream; every rank runs the same collectives in the same order
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        err = None
        try:
            with torch.cuda.stream(side):
                for j in range(NS):
                    self._fill(j, "F")
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
        except Exception as e:  # noqa: BLE001 (re-raised below on every rank)
            err = e
        if X:
            ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
            torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN, group=s.group)
            if int(ok.item()) == 0:
                raise RuntimeError(f"stream warm-up failed on some rank: {err!r}")
        elif err is not None:
            raise err
        if capture:
            # one graph per (stage, slot); F is F1 + FX + F2 at G > 1 (the garbage
            # collector off meanwhile: li._host "graph lifetime")
            names = ("R", "P", "S") + (("F1", "FX", "F2") if X else ("F",))
            self.graphs = {}
            with no_gc_capture():
                for name in names:
                    for j in range(NS):
                        gr = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                            self._f[name](j)
                        self.graphs[name, j] = gr
            torch.cuda.synchronize(dev)

    # -- lifetime ------------------------------------------------------------
    def drain(self):
        """Wait for every piece of work this object enqueued: its finish, plan
        and route streams, and the scans it launched on the caller's stream
        (with `lookahead` the next launch's scan is still in flight when
        step() returns)."""
        if getattr(self, "_closed", True) or capture_underway():
            return
        for evs in (self._up, self._rdone, self._pdone, self._sdone, self._gdone, self._fdone):
            for e in evs:
                e.synchronize()
        for st in (self._fs, self._ps, self._rs):
            st.synchronize()

    def close(self):
        """drain(), then release the captured graphs (and with them their
        private memory pools and kernel-argument buffers): a StreamedSearch
        dropped right after step() still has its lookahead scan graph queued
        on the device, and destroying that executable and handing its pool's
        blocks to the caching allocator while the GPU still uses them is
        unsafe.  Inside another object's capture nothing is synchronised or
        destroyed: the graphs are parked (li._host "graph lifetime", the
        root cause of round 5's abort).  Idempotent; step() after close()
        raises."""
        if getattr(self, "_closed", True):
            return
        if capture_underway():
            # (a finaliser inside another capture: park the graphs, li._host)
            release_later(self.graphs, self.ws, self.rws, self.lists, self.xall)
        else:
            self.drain()
        self.graphs = None
        self._closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown: torch may be gone)
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- staging -------------------------------------------------------------
    def stage(self, q_nav, q_search, slot: Optional[int] = None) -> bool:
        """Write this rank's block of a batch (host arrays of the stream's
        shape; rows [g*per, (g+1)*per) at G > 1) into the pinned staging rows
        of `slot` (default: the slot the next launch routes), on the host
        cores (lmi_host_stage_f16: float32 -> fp16 with the exactness check in
        one pass; float16 rows are copied).  Returns False when a clip768
        value of the block is not fp16-representable: the block still goes
        in, flagged, and the launch that finishes the batch raises
        QueryNotF16 on every rank (stream() then answers it eagerly)."""
        nav, qs = host_array(q_nav), host_array(q_search)
        nq, d, dn, per = self.nq, self.d, self.dn, self.per
        if nav.shape != (nq, dn) or qs.shape != (nq, d):
            raise ValueError("a staged batch must have the stream's shape")
        if slot is None:
            slot = (self._t or 0) % self.NS
        lo, hi = self.lo, self.hi
        blk = self.h_stage[slot].numpy()
        stage_rows_f32(blk[:(hi - lo) * dn].view(np.float32).reshape(hi - lo, dn), nav[lo:hi])
        if self.split:  # (float32 rows as given: the split mode rounds them itself)
            stage_rows_f32(blk[self.o_q:self.o_q + (hi - lo) * d].view(np.float32).reshape(hi - lo, d),
                           qs[lo:hi])
            blk[self.o_flag] = 0
            return True
        ok = stage_rows_f16(blk[self.o_q:self.o_q + (hi - lo) * (d // 2)].view(np.float16)
                            .reshape(hi - lo, d), qs[lo:hi])
        blk[self.o_flag] = 0 if ok else _lib.LMI_STATUS_QUERY_NOT_F16
        return ok

    def upload_bytes(self) -> int:
        """Bytes this rank moves host -> device per launch (its block)."""
        return 4 * self.staged_words

    # -- launches --------------------------------------------------------------
    def _fill(self, j, upto):
        """Slot j's stages eagerly, in order, up to `upto` (fill and drain)."""
        order = ("U", "R") + (("X",) if self.X else ()) + ("P", "S", "F")
        for name in order:
            if name == "X":
                self._f["X"]((j + 1) % self.NS)  # the exchange buffer holding slot j's block
            else:
                self._f[name](j)
            if name == upto:
                return

    def prime(self):
        """Fill the pipeline with the staged rows of slots 1, 2 and 3 (eagerly:
        slot 1 up to its scan, slots 2 and 3 up to their plans): the next
        launch answers slot 1."""
        dev = self.searcher.index.device
        for j, upto in ((1, "S"), (2, "P"), (3, "P")):
            self._fill(j, upto)
        torch.cuda.current_stream(dev).synchronize()
        self._t = 0
        self._s_ahead = False

    def _run(self, name, j):
        if self.graphs is not None:
            self.graphs[name, j].replay()
        else:
            self._f[name](j)

    def _run_scan(self, j, main):
        if self.time_scans:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            self._run("S", j)
            e1.record(main)
            self._scan_ev.append((e0, e1))
        else:
            self._run("S", j)
        self._sdone[j].record(main)

    def scan_ms(self):
        """Durations (ms) of the scans step() launched while `time_scans` was
        set (HIP events on the scan's stream, outside the captured graphs),
        in launch order; clears the record."""
        out = []
        for e0, e1 in self._scan_ev:
            e1.synchronize()
            out.append(e0.elapsed_time(e1))
        self._scan_ev = []
        return out

    def step(self):
        """One launch -> (dists f64 [nq, w], anns uint32 [nq, w]) of the batch
        it finished (numpy views, valid for the next three launches).  Slot
        t mod 4 is uploaded, routed and planned (stage() before step() streams
        a new batch; without it the slot's previous rows are used again), slot
        t + 2 scanned and t + 1 finished (mod 4), on four streams (each on its
        own hardware queue, queue_streams; the upload and the route share one):

            copy:   H2D of this rank's block of slot t      (the copy engine)
            route:  wait H2D -> router (slot t)
            scan:   wait plan(two launches ago) -> K2 SCAN (slot t+2)
            finish: wait scan(last launch) [and route] -> merge phase
                    [-> all-gather -> K3] -> replay -> D2H (slot t+1)
            plan:   wait route [G > 1: the all-gather] -> widen, K2 PLAN (slot t)

        With `lookahead` the next launch's scan (slot t+3, planned a launch
        earlier) is enqueued too, behind this launch's finish on the device."""
        if self._closed:
            raise RuntimeError("StreamedSearch: step() after close()")
        if self._t is None:
            self.prime()
        dev = self.searcher.index.device
        NS, X = self.NS, self.X
        t = self._t % NS
        jr, js, jf = t, (t + 2) % NS, (t + 1) % NS
        main = torch.cuda.current_stream(dev)
        # (slot jr's device block was last read by the plan -- at G > 1 the
        # all-gather -- of four launches ago, which the finish the host waited
        # for at the end of the last launch depended on)
        with torch.cuda.stream(self._cs):
            self._f["U"](jr)
        self._up[jr].record(self._cs)
        if not self._s_ahead:
            main.wait_event(self._pdone[js])
            self._run_scan(js, main)
        self._rs.wait_event(self._up[jr])
        with torch.cuda.stream(self._rs):
            self._run("R", jr)
        self._rdone[jr].record(self._rs)
        if not X:
            self._ps.wait_event(self._rdone[jr])
            with torch.cuda.stream(self._ps):
                self._run("P", jr)
            self._pdone[jr].record(self._ps)
        self._fs.wait_event(self._sdone[jf])
        if not X:
            with torch.cuda.stream(self._fs):
                self._run("F", jf)
        else:
            # F1, the merge phase, runs as soon as the scan is done; FX gathers
            # slot jf's lists with slot jr's block (exchange buffer jf), so it
            # also waits for that block's route (the router, starved by the
            # scan's persistent grid, ends ~50 us after it: round 6 moved the
            # merge phase out from behind it)
            with torch.cuda.stream(self._fs):
                self._run("F1", jf)
            self._fs.wait_event(self._rdone[jr])
            with torch.cuda.stream(self._fs):
                self._run("FX", jf)
            self._gdone[jf].record(self._fs)
            with torch.cuda.stream(self._fs):
                self._run("F2", jf)
            self._ps.wait_event(self._gdone[jf])
            with torch.cuda.stream(self._ps):
                self._run("P", jr)
            self._pdone[jr].record(self._ps)
        self._fdone[jf].record(self._fs)
        if self.lookahead:
            jn = (t + 3) % NS
            main.wait_event(self._pdone[jn])
            if not self.overlap:
                main.wait_event(self._fdone[jf])
            self._run_scan(jn, main)
        self._s_ahead = bool(self.lookahead)
        self._t += 1
        self.launches += 1
        if X and self.graphs is not None:
            wait_event_with_deadline(self._fdone[jf], self.timeout_s)
        else:
            self._fdone[jf].synchronize()
        return self._answer(jf)

    def _answer(self, j):
        hd, ha, st, rst = answer_views(self.h_ans[j], self.nq, self.w)
        if st & _lib.LMI_STATUS_INTERNAL or rst:
            raise RuntimeError(f"stream: status {st}/{rst}")
        if st & _lib.LMI_STATUS_QUERY_NOT_F16:
            raise QueryNotF16("a streamed batch is not fp16-exact")
        return hd, ha

    def _eager(self, batch):
        """A batch the stream cannot answer (not fp16-exact), by
        Searcher.search; every rank calls it at the same batch."""
        s = self.searcher
        dev = s.index.device
        torch.cuda.synchronize(dev)  # (no captured collective in flight)
        nav, qs = host_array(batch[0]), host_array(batch[1])
        return s.search(torch.from_numpy(np.ascontiguousarray(nav, dtype=np.float32)).to(dev),
                        torch.from_numpy(np.ascontiguousarray(qs)).to(dev), self.R, k=self.k,
                        k_round=self.k_round, use_threshold=self.use_threshold, dist=self.dist)

    def _take(self, j, batch):
        try:
            return tuple(a.copy() for a in self._answer(j))
        except QueryNotF16:
            return self._eager(batch)

    def stream(self, batches):
        """Answer an iterable of (q_nav, q_search) batches in order, yielding
        (dists, anns) copies per batch: three batches fill the pipeline, then
        one launch per batch, then the last three finish eagerly.  A batch
        that is not fp16-exact is answered by Searcher.search instead."""
        dev = self.searcher.index.device
        NS, X = self.NS, self.X
        sync = lambda: torch.cuda.current_stream(dev).synchronize()
        it = iter(batches)
        held = {}
        first = []
        for b in it:
            first.append(b)
            if len(first) == NS - 1:
                break
        for j, b in zip(range(1, NS), first):
            self.stage(*b, slot=j)
            held[j] = b
        if len(first) < NS - 1:
            for j in range(1, 1 + len(first)):
                self._fill(j, "F")
                sync()
                yield self._take(j, held[j])
            return
        self.prime()
        for b in it:
            j = self._t % NS
            self.stage(*b, slot=j)
            held[j] = b
            jf = (self._t + 1) % NS
            try:
                out = self.step()
                yield tuple(a.copy() for a in out)
            except QueryNotF16:
                yield self._eager(held[jf])
        # drain: slot t+1 is scanned, t+2 and t+3 planned (mod 4; t+2's scan
        # enqueued when lookahead), t the launch count
        torch.cuda.synchronize(dev)  # (every stream of the last launch)
        t = self._t
        j1, j2, j3 = (t + 1) % NS, (t + 2) % NS, (t + 3) % NS
        self._f["F"](j1)
        sync()
        yield self._take(j1, held[j1])
        if not self._s_ahead:
            self._f["S"](j2)
        self._f["F"](j2)
        sync()
        yield self._take(j2, held[j2])
        self._f["S"](j3)
        self._f["F"](j3)
        sync()
        self.drain()
        yield self._take(j3, held[j3])
        self._t = None
        self._s_ahead = False
