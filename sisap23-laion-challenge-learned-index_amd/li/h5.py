"""ctypes binding of liblmi_h5.so (include/lmi_h5.h): the HDF5 files around the
hot path, native over the image's libhdf5 (h5py is not installed here).

  read_dataset(path, key)        np.array(h5py.File(path, "r")[key])
                                 (search.py:48-49, :79-87): the stored floating
                                 type (float16 'emb' stays float16), or
                                 converted by HDF5 with dtype=np.float32
  write_results(dst, ...)        store_results (utils.py:85-97), eval/'s format
  write_dataset(path, key, x)    lay synthetic data out as data/<kind>/<size>/*.h5
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

# LMI_H5_LIB_NAME: the host-sanitizer build (csrc `make asan`: liblmi_h5_asan.so)
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        os.environ.get("LMI_H5_LIB_NAME", "liblmi_h5.so"))
F32, F16, F64, U32, I64 = 0, 1, 2, 3, 4
EXPORTS = ("lmi_h5_dataset_info", "lmi_h5_read_f32", "lmi_h5_read_stored", "lmi_h5_write_results",
           "lmi_h5_write_f32", "lmi_h5_write_stored", "lmi_h5_last_error")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} missing: build it (make -C csrc) against libhdf5")
        lib = C.CDLL(LIB_PATH)
        lib.lmi_h5_dataset_info.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p, C.c_void_p]
        lib.lmi_h5_read_f32.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.c_int64, C.c_void_p]
        lib.lmi_h5_read_stored.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.c_int64, C.c_int32,
                                           C.c_void_p]
        lib.lmi_h5_write_results.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32,
                                             C.c_char_p, C.c_char_p, C.c_double, C.c_double,
                                             C.c_char_p, C.c_char_p]
        lib.lmi_h5_write_f32.argtypes = [C.c_char_p, C.c_char_p, C.c_int32, C.c_int64, C.c_int64,
                                         C.c_void_p, C.c_int32]
        lib.lmi_h5_write_stored.argtypes = [C.c_char_p, C.c_char_p, C.c_int32, C.c_int64, C.c_int64,
                                            C.c_void_p, C.c_int32]
        lib.lmi_h5_last_error.restype = C.c_char_p
        _lib = lib
    return _lib


def _check(rc, what):
    if rc != 0:
        raise OSError(f"{what}: {load().lmi_h5_last_error().decode()} (code {rc})")


def _b(s) -> bytes:
    return str(s).encode()


def dataset_info(path: str, key: str):
    """((rows, cols), dtype code) of a rank-1/2 dataset."""
    dims = np.zeros(2, np.int64)
    dt = C.c_int32(0)
    _check(load().lmi_h5_dataset_info(_b(path), _b(key), dims.ctypes.data, C.byref(dt)),
           f"{path}[{key}]")
    return (int(dims[0]), int(dims[1])), dt.value


_STORED = {F16: np.float16, F32: np.float32, F64: np.float64, U32: np.uint32, I64: np.int64}


def read_dataset(path: str, key: str, row0: int = 0, nrows: int = None, dtype=None) -> np.ndarray:
    """Rows of a dataset [nrows, cols] in its stored type (float16/32/64, or
    the result files' uint32 knns / int64), as
    np.array(h5py.File(path)[key]) gives them (the fp16 clip768 'emb' stays
    float16: the reference then computes float64 distances, utils.py:11);
    dtype=np.float32 converts through HDF5 instead (fp16 widened exactly)."""
    (n, d), code = dataset_info(path, key)
    nrows = n - row0 if nrows is None else nrows
    if dtype is None and code in _STORED:
        out = np.empty((nrows, d), _STORED[code])
        _check(load().lmi_h5_read_stored(_b(path), _b(key), row0, nrows, out.itemsize,
                                         out.ctypes.data), f"{path}[{key}]")
        return out
    if dtype not in (None, np.float32):
        raise ValueError("read_dataset: dtype must be None (stored) or np.float32")
    out = np.empty((nrows, d), np.float32)
    _check(load().lmi_h5_read_f32(_b(path), _b(key), row0, nrows, out.ctypes.data),
           f"{path}[{key}]")
    return out


def write_dataset(path: str, key: str, x: np.ndarray, *, fp16: bool, append: bool = False):
    """A rank-2 dataset stored as float16 (fp16=True) or float32; a float16
    array with fp16=True is written as it is (no conversion)."""
    if fp16 and np.asarray(x).dtype == np.float16:
        x = np.ascontiguousarray(x)
        if x.ndim != 2:
            raise ValueError("write_dataset: 2-D arrays only")
        _check(load().lmi_h5_write_stored(_b(path), _b(key), 2, x.shape[0], x.shape[1], x.ctypes.data,
                                          int(append)), f"{path}[{key}]")
        return
    x = np.ascontiguousarray(x, dtype=np.float32)
    if x.ndim != 2:
        raise ValueError("write_dataset: 2-D arrays only")
    _check(load().lmi_h5_write_f32(_b(path), _b(key), F16 if fp16 else F32, x.shape[0], x.shape[1],
                                   x.ctypes.data, int(append)), f"{path}[{key}]")


def write_results(dst: str, algo, kind, dists, anns, buildtime, querytime, params, size):
    """store_results (utils.py:85-97): knns uint32 and dists float64 [nq, k]."""
    anns = np.ascontiguousarray(anns)
    dists = np.ascontiguousarray(dists, dtype=np.float64)
    if anns.dtype != np.uint32:
        # the reference writes anns.dtype as is; its search returns uint32
        if anns.dtype.kind not in "iu" or (anns.size and (anns.min() < 0 or anns.max() > 2**32 - 1)):
            raise TypeError(f"knns must be uint32-representable ids (got {anns.dtype})")
        anns = anns.astype(np.uint32)
    if anns.shape != dists.shape or anns.ndim != 2:
        raise ValueError("knns and dists must both be [nq, k]")
    _check(load().lmi_h5_write_results(_b(dst), anns.ctypes.data, dists.ctypes.data, anns.shape[0],
                                       anns.shape[1], _b(algo), _b(kind), float(buildtime),
                                       float(querytime), _b(size), _b(params)), dst)
