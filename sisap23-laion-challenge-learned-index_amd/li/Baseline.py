"""Exact brute-force k-NN (reference search/li/Baseline.py:7-25) on the GPU.

The whole corpus is one bucket of the K2 scan: the exact
top-k by (distance, row) is what `pairwise_cosine(data, queries).T.argsort()`
and `np.sort` give on tie-free inputs (Baseline.py:17-19).  k <= LMI_MAX_K.
"""
import time

import numpy as np
import torch

from .Logger import Logger


class Baseline(Logger):
    def __init__(self):
        self._index = None

    def search(self, queries, data, k=10):
        from .index import DeviceIndex, bucket_topk
        s = time.time()
        n = np.shape(data)[0]
        if self._index is None or self._index.n_total != n:
            self._index = DeviceIndex(data, np.zeros(n, np.int64), 1)
        ix = self._index
        q = torch.from_numpy(np.ascontiguousarray(queries, dtype=np.float32)).to(ix.device)
        classes = torch.zeros((q.shape[0], 1), dtype=torch.int32, device=ix.device)
        d, pos, st = bucket_topk(ix, q, classes, k)
        if int(st.item()):
            from . import _lib
            d, pos, _ = bucket_topk(ix, q, classes, k, qmode=_lib.LMI_Q_F32)
        dists = d[:, 0].cpu().numpy()  # fp32, like 1 - cosine_similarity of fp32 inputs
        nns = ix.pos_to_id[np.maximum(pos[:, 0].cpu().numpy(), 0)]
        return dists, nns, time.time() - s

    def build(self, data):
        s = time.time()
        self.logger.info('No build method implemented for baseline.')
        return time.time() - s
