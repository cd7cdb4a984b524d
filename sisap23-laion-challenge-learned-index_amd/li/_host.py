"""Host-side helpers of the captured search steps (li.graphed, li.stream):
query batches as host arrays, staging them into pinned memory on the host
cores (liblmi's lmi_host_stage_f16 / lmi_host_copy, ABI 8), and bounded waits
for steps whose collectives are outside the process group's watchdog.

The reference's queries are host arrays (search.py:49, :85-87) and its timer
(search.py:116-141) starts with them in host memory; a step that streams new
batches has to write each one into the pinned rows its H2D copy reads."""
from __future__ import annotations

import time

import numpy as np
import torch

from . import _lib


def host_array(x) -> np.ndarray:
    """A query batch (numpy, or a torch tensor on any device) as a host array."""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def np_fp16_exact(x: np.ndarray) -> bool:
    """True when every value of a host array round-trips through fp16."""
    x = np.asarray(x)
    if x.dtype == np.float16:
        return True
    x32 = x.astype(np.float32, copy=False)
    if x.dtype != np.float32 and not np.array_equal(x32.astype(x.dtype), x):
        return False
    return bool(np.array_equal(x32.astype(np.float16).astype(np.float32), x32))


def stage_rows_f32(dst: np.ndarray, src: np.ndarray, threads: int = 0) -> None:
    """dst[:] = src (float32 rows, same shape) on the host cores."""
    src = np.ascontiguousarray(src, dtype=np.float32)
    if src.shape != dst.shape or dst.dtype != np.float32 or not dst.flags.c_contiguous:
        raise ValueError("stage_rows_f32: shape/dtype mismatch")
    _lib.check("lmi_host_copy", _lib.load().lmi_host_copy(dst.ctypes.data, src.ctypes.data,
                                                          src.nbytes, threads))


def stage_rows_f16(dst: np.ndarray, src: np.ndarray, threads: int = 0) -> bool:
    """dst[:] = src as fp16 rows on the host cores; True when every value of
    src is fp16-representable (the fp16 scan's precondition).  float16 input
    is copied as it is (exact by construction); float64 input must also be
    exact in float32."""
    if dst.dtype != np.float16 or not dst.flags.c_contiguous:
        raise ValueError("stage_rows_f16: dst must be a contiguous float16 array")
    src = np.asarray(src)
    if src.shape != dst.shape:
        raise ValueError("stage_rows_f16: shape mismatch")
    lib = _lib.load()
    if src.dtype == np.float16:
        src = np.ascontiguousarray(src)
        _lib.check("lmi_host_copy", lib.lmi_host_copy(dst.ctypes.data, src.ctypes.data,
                                                      src.nbytes, threads))
        return True
    ok = True
    if src.dtype != np.float32:
        s32 = src.astype(np.float32)
        ok = bool(np.array_equal(s32.astype(src.dtype), src))
        src = s32
    src = np.ascontiguousarray(src)
    r = int(lib.lmi_host_stage_f16(src.ctypes.data, src.size, dst.ctypes.data, threads))
    if r < 0:
        _lib.check("lmi_host_stage_f16", -r)
    return ok and r == 1


def wait_event_with_deadline(ev, timeout_s: float) -> None:
    """Wait for a recorded event, raising after `timeout_s`: a graph replay
    whose all-gather waits for a rank that died never completes, and RCCL
    kernels captured in a graph are outside the process group's watchdog
    (li.dist.init_from_env).  The caller should end the process: the stalled
    kernels stay queued on the device until its context is torn down."""
    deadline = time.monotonic() + timeout_s
    spins = 0
    while not ev.query():
        spins += 1
        if spins > 1000:
            if time.monotonic() > deadline:
                raise RuntimeError(f"search step not finished after {timeout_s:.0f} s: a peer rank "
                                   "stopped inside the step's collectives; end this process")
            time.sleep(1e-4)


def wait_with_deadline(dev, timeout_s: float) -> None:
    """wait_event_with_deadline on the current stream's work."""
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    wait_event_with_deadline(ev, timeout_s)


# ---- graph lifetime ---------------------------------------------------------
# The round-5 abort, root-caused in round 6 (DESIGN.md §5 "Graph lifetime"):
# a StreamedSearch holds its stage closures, which hold the object -- a
# reference cycle -- so a dropped object is freed by the cyclic garbage
# collector, at whatever allocation triggers it.  When that allocation sat
# inside ANOTHER object's graph capture, the collector ran the old object's
# finalisers there: destroying a graph executable and releasing its private
# memory pool (or synchronising an event) while a stream capture is underway
# aborts the process.  So: (1) captures run with the collector off
# (`no_gc_capture`), and (2) a finaliser that runs while a capture is
# underway anyway (another library's capture) parks the graphs instead of
# destroying them (`release_later`); they are destroyed at the next safe
# point (`flush_released`, after a device synchronisation).
_PARKED = []


def capture_underway() -> bool:
    """True while the current stream is capturing a graph."""
    try:
        return bool(torch.cuda.is_available() and torch.cuda.is_current_stream_capturing())
    except Exception:  # noqa: BLE001
        return False


def release_later(*objs) -> None:
    """Keep `objs` (graphs, their buffers) alive until flush_released()."""
    _PARKED.append(objs)


def flush_released() -> None:
    """Destroy the parked graphs once no capture is underway (after a device
    synchronisation: their last replays may still be queued)."""
    if _PARKED and not capture_underway():
        torch.cuda.synchronize()
        _PARKED.clear()


class no_gc_capture:
    """Context manager around a block of graph captures: the cyclic garbage
    collector is off inside (torch.cuda.graph itself collects before each
    capture begins), so no finaliser runs mid-capture.  The captures
    themselves use capture_error_mode="thread_local": with an RCCL process
    group the watchdog thread queries its collectives' events at any moment,
    and in the default global mode such a query from another thread during a
    capture invalidates it and kills the watchdog, which aborts the process
    (round 6: tools/stream_steps.py aborted building its eighth stream object
    that way, gpurun_out r6d)."""

    def __enter__(self):
        import gc
        flush_released()
        self._was = gc.isenabled()
        gc.disable()
        return self

    def __exit__(self, *exc):
        import gc
        if self._was:
            gc.enable()
