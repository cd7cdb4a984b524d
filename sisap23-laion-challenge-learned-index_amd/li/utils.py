"""I/O helpers of the reference's search/li/utils.py that sit around the hot path.

The distance helpers of the reference (pairwise_cosine, utils.py:10-11, and
pairwise_cosine_threshold, :14-43) are replaced as a whole by the GPU scan
(lmi_bucket_topk) plus the host replay; they are not re-exported here so that
no CPU distance path exists in the product package.
"""
from __future__ import annotations

import os
import pickle
from pathlib import Path


def save_as_pickle(filename: str, obj):
    """utils.py:46-60 (in a process group, rank 0 writes the file)."""
    from .dist import is_writer
    if not is_writer():
        return
    with open(filename, "wb") as f:
        pickle.dump(obj, f)


def prepare(kind, size):
    """utils.py:71-82 downloads the SISAP'23 files; offline builds only accept
    files that are already in place."""
    for version in ("query", "dataset"):
        target = os.path.join("data", kind, size, f"{version}.h5")
        if not os.path.exists(target):
            raise FileNotFoundError(
                f"{target} missing: this build has no network access (utils.py:63-82 would download it)")


def store_results(dst, algo, kind, dists, anns, buildtime, querytime, params, size):
    """utils.py:85-97: HDF5 with attrs algo/data/buildtime/querytime/size/params
    and datasets knns (uint32) and dists (float64), read by eval/ — written by
    the native libhdf5 shim (li.h5, liblmi_h5.so).  In a process group every
    rank holds the same answer and rank 0 writes the file."""
    from . import h5
    from .dist import is_writer
    if not is_writer():
        return
    os.makedirs(Path(dst).parent, exist_ok=True)
    h5.write_results(dst, algo, kind, dists, anns, buildtime, querytime, params, size)
