"""Exact brute-force k-NN (reference search/li/Baseline.py:7-25) on the GPU.

The whole corpus is one bucket of the K2 scan: the exact
top-k by (distance, row) is what `pairwise_cosine(data, queries).T.argsort()`
and `np.sort` give on tie-free inputs (Baseline.py:17-19).  As in the
reference, the distances are float32 when data and queries are both float32
and float64 otherwise (sklearn's dtype rule, utils.py:11); the float64 case
runs lmi_bucket_topk_f64.  k <= LMI_MAX_K_PASSES (float32) / LMI_MAX_K_F64 (float64); k > 16 runs the
scan's lower-bound passes.
"""
import time

import numpy as np
import torch

from . import _lib
from .Logger import Logger


class Baseline(Logger):
    def __init__(self):
        self._index = None
        self._key = None

    def search(self, queries, data, k=10):
        from .LearnedIndex import _upload_queries, content_key, dist_dtype
        from .index import DeviceIndex, Searcher
        s = time.time()
        key = content_key(data)
        if self._index is None or self._key != key:
            n = np.shape(data)[0]
            self._index = DeviceIndex(data, np.zeros(n, np.int64), 1)
            self._key = key
        ix = self._index
        q = _upload_queries(queries, ix.device)
        classes = torch.zeros((q.shape[0], 1), dtype=torch.int32, device=ix.device)
        dist = dist_dtype(data, queries)
        _, d, pos, st = Searcher(ix, None, exchange=False).lists(None, q, 1, k, classes=classes, dist=dist)
        if int(st.item()) & _lib.LMI_STATUS_INTERNAL:
            raise RuntimeError(f"Baseline.search: scan status {int(st.item())}")
        dists = d[:, 0].cpu().numpy()  # float32 or float64, as 1 - cosine_similarity
        nns = ix.pos_to_id[np.maximum(pos[:, 0].cpu().numpy(), 0)]
        return dists, nns, time.time() - s

    def build(self, data):
        s = time.time()
        self.logger.info('No build method implemented for baseline.')
        return time.time() - s
