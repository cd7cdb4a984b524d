"""ctypes binding of liblmi_hip.so (the C-ABI declared in include/lmi_hip.h).

The library is the product path: there is no Python or CPU fallback for any
kernel.  If the shared object is missing or fails to load, every entry point
raises ``LmiUnavailable`` loudly.

torch is imported before the library is opened so that the process has ONE
HIP runtime: torch's ``libamdhip64.so`` carries the soname ``libamdhip64.so.7``
that liblmi_hip.so needs, so the dynamic linker reuses it instead of loading
``/opt/rocm/lib``'s copy (device pointers and streams are then shared).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (must precede the dlopen: one HIP runtime per process)

LIB_NAME = os.environ.get("LMI_LIB_NAME", "liblmi_hip.so")  # diagnostic builds only
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

LMI_OK = 0
LMI_E_INVALID = 1001
LMI_E_UNSUPPORTED = 1002
LMI_E_WORKSPACE = 1003
LMI_E_HIP = 1004
LMI_STATUS_QUERY_NOT_F16 = 1
LMI_STATUS_INTERNAL = 2

LMI_F32 = 0
LMI_F16 = 1
LMI_ROUTER_TOPR = 0
LMI_ROUTER_ARGMAX = 1
LMI_Q_F16 = 0
LMI_Q_F32 = 1
LMI_Q_SEED_ROUND0 = 0x100
LMI_Q_PHASE_PLAN = 0x200
LMI_Q_PHASE_SCAN = 0x400
LMI_Q_PHASE_MERGE = 0x800
LMI_Q_PHASE_REFINE = 0x1000
LMI_REPLAY_PHASE_GROUPS = 1
LMI_REPLAY_PHASE_ROUNDS = 2
LMI_MAX_LAYERS = 8
LMI_MAX_K = 16
LMI_MAX_K_PASSES = 1024
LMI_MAX_K_F64 = 240
LMI_REPLAY_DEVICE_MAX_KR = 32
LMI_REPLAY_DEVICE_MAX_K = 64
LMI_KMEANS_MAX_D = 128
LMI_REFINE_EPS = 2.0 ** -16

# every symbol include/lmi_hip.h declares (tests check the export table)
EXPORTS = (
    "lmi_router",
    "lmi_plan_chunks",
    "lmi_scan_workspace_bytes",
    "lmi_bucket_topk",
    "lmi_merge_topk",
    "lmi_scan_f64_workspace_bytes",
    "lmi_bucket_topk_f64",
    "lmi_bucket_topk_f64q",
    "lmi_f64_global_band",
    "lmi_bucket_topk_f64g",
    "lmi_refine_fallback_count",
    "lmi_split_sample_fallback_count",
    "lmi_split_eps",
    "lmi_split_normalize",
    "lmi_replay_device_phase",
    "lmi_merge_topk_f64",
    "lmi_packed_rank_words",
    "lmi_merge_topk_packed",
    "lmi_replay",
    "lmi_replay_f64",
    "lmi_replay_device_workspace_bytes",
    "lmi_replay_device",
    "lmi_replay_device_f64",
    "lmi_kmeans_assign",
    "lmi_kmeans_workspace_bytes",
    "lmi_kmeans_update",
    "lmi_timing_enable",
    "lmi_timing_read",
    "lmi_last_error",
    "lmi_abi_version",
    "lmi_config_reload",
    "lmi_scan_set_workgroups",
    "lmi_host_hash64",
    "lmi_host_stage_f16",
    "lmi_host_copy",
)


class LmiUnavailable(RuntimeError):
    """liblmi_hip.so is missing or unusable; there is no fallback path."""


class LmiError(RuntimeError):
    def __init__(self, fn: str, rc: int, msg: str):
        super().__init__(f"{fn} failed with code {rc}: {msg}")
        self.rc = rc


class MlpDesc(C.Structure):
    _fields_ = [
        ("n_layers", C.c_int32),
        ("dims", C.c_int32 * (LMI_MAX_LAYERS + 1)),
        ("W", C.c_void_p * LMI_MAX_LAYERS),
        ("b", C.c_void_p * LMI_MAX_LAYERS),
    ]


ABI_VERSION = 13


class IndexDesc(C.Structure):
    _fields_ = [
        ("corpus", C.c_void_p),
        ("dtype", C.c_int32),
        ("d", C.c_int32),
        ("d_pad", C.c_int32),
        ("n_rows", C.c_int64),
        ("inv_norm", C.c_void_p),
        ("gpos", C.c_void_p),
        ("n_buckets", C.c_int32),
        ("bucket_off", C.c_void_p),
        ("chunk_rows", C.c_int32),
        ("chunk_first", C.c_void_p),
        ("n_chunks", C.c_int32),
        ("max_chunks", C.c_int32),
        ("chunk_centroid", C.c_void_p),  # ABI 2
        ("corpus64", C.c_void_p),        # ABI 6
        ("corpus32", C.c_void_p),        # ABI 9
        ("bucket_rows", C.c_void_p),     # ABI 10
        ("corpus32n", C.c_void_p),       # ABI 11
    ]


_P = C.c_void_p
_I32 = C.c_int32
_I64 = C.c_int64

_SIGNATURES = {
    "lmi_router": (C.c_int, [_P, _I32, _I32, C.POINTER(MlpDesc), _I32, _I32, _P, _P, _P]),
    "lmi_plan_chunks": (C.c_int32, [_P, _I32, _I32, _P]),
    "lmi_scan_workspace_bytes": (C.c_size_t, [C.POINTER(IndexDesc), _I32, _I32, _I32, _I32]),
    "lmi_bucket_topk": (C.c_int, [C.POINTER(IndexDesc), _P, _I32, _I32, _P, _I32, _I32, _I32,
                                  _P, _P, _P, _P, C.c_size_t, _P]),
    "lmi_merge_topk": (C.c_int, [_P, _P, _I32, _I64, _I32, _P, _P, _P]),
    "lmi_scan_f64_workspace_bytes": (C.c_size_t, [C.POINTER(IndexDesc), _I32, _I32, _I32, _I32]),
    "lmi_bucket_topk_f64": (C.c_int, [C.POINTER(IndexDesc), _P, _I32, _I32, _P, _I32, _I32, _I32,
                                      C.c_double, _P, _P, _P, _P, C.c_size_t, _P]),
    "lmi_bucket_topk_f64q": (C.c_int, [C.POINTER(IndexDesc), _P, _I32, _I32, _P, _I32, _P, _I32,
                                       _I32, _I32, C.c_double, _P, _P, _P, _P, C.c_size_t, _P]),
    "lmi_f64_global_band": (C.c_int, [C.POINTER(IndexDesc), _I32, _I32, _I32, _I32]),
    "lmi_bucket_topk_f64g": (C.c_int, [C.POINTER(IndexDesc), _P, _I32, _I32, _P, _I32, _P, _I32,
                                       _I32, _I32, C.c_double, _P, _P, _I32, _I64, _P, _P, _P, _P,
                                       C.c_size_t, _P]),
    "lmi_split_eps": (C.c_double, [_I32]),
    "lmi_split_normalize": (C.c_int, [_P, _I64, _I32, _I32, _P, _P]),
    "lmi_replay_device_phase": (C.c_int, [_I32, _I32, _P, _I32, _I32, _I32, _P, _P, _I32, _I32, _P, _I32,
                                          _P, _I64, _I32, _P, _P, _P, _P, _P, C.c_size_t, _P]),
    "lmi_refine_fallback_count": (C.c_int, [_P, C.POINTER(IndexDesc), _I32, _I32, _I32, _I32, _P,
                                            _P]),
    "lmi_split_sample_fallback_count": (C.c_int, [_P, C.POINTER(IndexDesc), _I32, _I32, _I32, _P, _P]),
    "lmi_merge_topk_f64": (C.c_int, [_P, _P, _I32, _I64, _I32, _P, _P, _P]),
    "lmi_packed_rank_words": (C.c_int64, [_I64, _I32, _I32]),
    "lmi_merge_topk_packed": (C.c_int, [_P, _I32, _I64, _I64, _I32, _I32, _P, _P, _P, _P]),
    "lmi_replay": (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _I32, _I32, _P, _I32, _P, _I64, _I32,
                             _P, _P, _P, _P]),
    "lmi_replay_f64": (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _I32, _I32, _P, _I32, _P, _I64,
                                 _I32, _P, _P, _P, _P]),
    "lmi_replay_device_workspace_bytes": (C.c_size_t, [_I32, _I32, _I32, _I32, _I32, _I32]),
    "lmi_replay_device": (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _I32, _I32, _P, _I32, _P, _I64,
                                    _I32, _P, _P, _P, _P, _P, C.c_size_t, _P]),
    "lmi_replay_device_f64": (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _I32, _I32, _P, _I32, _P,
                                        _I64, _I32, _P, _P, _P, _P, _P, C.c_size_t, _P]),
    "lmi_kmeans_assign": (C.c_int, [_P, _I64, _I32, _P, _I32, _P, _P, _P]),
    "lmi_kmeans_workspace_bytes": (C.c_size_t, [_I64, _I32, _I32]),
    "lmi_kmeans_update": (C.c_int, [_P, _I64, _I32, _P, _I32, _P, _P, _P, _P, C.c_size_t, _P]),
    "lmi_timing_enable": (C.c_int, [_I32]),
    "lmi_timing_read": (C.c_int32, [_P, _I32]),
    "lmi_last_error": (C.c_char_p, []),
    "lmi_abi_version": (C.c_int32, []),
    "lmi_config_reload": (C.c_int, []),
    "lmi_scan_set_workgroups": (C.c_int32, [_I32]),
    "lmi_host_hash64": (C.c_uint64, [_P, C.c_uint64, _I32]),
    "lmi_host_stage_f16": (C.c_int32, [_P, C.c_uint64, _P, _I32]),
    "lmi_host_copy": (C.c_int, [_P, _P, C.c_uint64, _I32]),
}

_lock = threading.Lock()
_lib = None


def load() -> C.CDLL:
    """Open liblmi_hip.so once; raise LmiUnavailable if it cannot be used."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise LmiUnavailable(
                f"{LIB_PATH} not found: build it with `make -C csrc` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        try:
            lib = C.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the host
            raise LmiUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.lmi_abi_version() != ABI_VERSION:
            raise LmiUnavailable("liblmi_hip.so ABI version mismatch")
        _lib = lib
        return lib


def check(fn: str, rc: int) -> None:
    if rc != LMI_OK:
        msg = load().lmi_last_error().decode(errors="replace")
        raise LmiError(fn, rc, msg)


def ptr(t) -> int:
    """Device (or host) address of a torch tensor / numpy array, 0 for None."""
    if t is None:
        return 0
    if isinstance(t, torch.Tensor):
        return t.data_ptr()
    return t.ctypes.data  # numpy


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(device=None) -> int:
    """hipStream_t of torch's current stream on `device` (the raw-pointer query
    when torch has it: a few microseconds cheaper per call on the hot path)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            d = torch.device(device)
            idx = d.index if d.index is not None else torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream
