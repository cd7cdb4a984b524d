"""Drop-in for the reference's search/li/LearnedIndex.py on MI355X.

`LearnedIndex.search` / `search_single` keep the reference's signatures,
argument meaning, side effects and return types (LearnedIndex.py:22-195):

  search(data_navigation, queries_navigation, data_search, queries_search,
         pred_categories, n_buckets=1, k=10, use_threshold=False)
      -> (dists float64 (nq, w), anns uint32 (nq, w)); w = 10 if n_buckets == 1
         else k (search() never passes k to search_single, :75-81)
  search_single(data_navigation, data_search, queries_search, pred_categories,
                k=10, threshold_dist=None) -> (dists float64 (nq, k), anns uint32)

Work split: the router (K1), the per-(query, probe) exact bucket top-k (K2)
and its merge run on the GPU through liblmi_hip.so; the reference's
threshold/grouping/padding procedure is replayed from the k-lists on the GPU
(lmi_replay_device; the host C++ lmi_replay is its bit-exact twin), which
reproduces its output exactly on tie-free inputs (tests/test_oracle_golden.py,
tests/test_gpu_golden.py, tests/test_gpu_replay.py).

The bucket-sorted corpus is built in HBM on first use and cached while
byte-identical data, ids and labels are passed again (`content_key`; the
reference re-gathers every bucket on every call: LearnedIndex.py:152-153, :168).
`attach` (an addition) builds it ahead of the timed calls and lets later
calls with the SAME objects skip the content hash: the caller promises not to
change those frames in place (or calls `attach` again).  search.py's CLI
attaches before its timed loop, as it never mutates its frames.

Process-group mode (an addition): one process per GPU, every
rank holding the same frames and making the same calls.  `use_process_group`
(automatic under a launcher that sets WORLD_SIZE > 1, e.g. torchrun or
`search.py --gpus N`; LMI_SHARD=0 turns that off) makes each rank build only
its stripe of every bucket (li.index.BucketLayout.shard) and run
`search` / `search_single` as li.index.Searcher's striped path: the router
sharded by queries, K2 on the stripe, one all-gather of the packed lists,
K3 and the replay on every rank -- so every rank returns the same answer,
bitwise the one-process answer.  `build` trains on rank 0 and broadcasts the
router and the object labels, so every rank indexes the same buckets.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from . import _lib
from .Logger import Logger
from .model import NeuralNetwork, data_X_to_torch, LIDataset

torch.manual_seed(2023)
np.random.seed(2023)

# LMI_AUTO_ATTACH=1: the first search / search_single call attaches its frames
# (LearnedIndex.attach), so an unchanged caller (the reference's own search.py)
# does not hash the corpus on every later call; the caller then must not change
# the frames in place.  Off by default: every call checks the content.
_AUTO_ATTACH = os.environ.get("LMI_AUTO_ATTACH") == "1"


def content_key(a) -> tuple:
    """Shape, dtype and a 64-bit hash of every byte of an array or DataFrame
    (its values in their own memory order, no copy of a contiguous block).

    Keys the HBM index cache: a cached corpus is reused only for byte-identical
    inputs, so a frame changed in place, or a new frame that happens to reuse
    a freed one's id(), is rebuilt rather than served stale.  The hash is
    liblmi's lmi_host_hash64 on all host cores (memory-bound; the python xxh3
    binding holds the GIL: ≈2.3 s on one core for 15 GB of fp16 clip768 at
    10M).  `LearnedIndex.attach` skips it for trusted objects."""
    v = a.to_numpy() if hasattr(a, "to_numpy") else np.asarray(a)
    if not v.flags.c_contiguous and v.T.flags.c_contiguous:
        mem, order = v.T, "F"
    else:
        mem, order = np.ascontiguousarray(v), "C"
    h = int(_lib.load().lmi_host_hash64(mem.ctypes.data if mem.nbytes else None, mem.nbytes, 0))
    return (v.shape, v.dtype.str, order, h)


def identity_key(a) -> tuple:
    """The object identity of an array, DataFrame or pandas Index: id(),
    shape, dtype and the addresses of its value arrays.  Cheap; it does not
    see values changed in place (that is what `attach` asks the caller to
    rule out)."""
    if hasattr(a, "_mgr") and hasattr(a._mgr, "arrays"):      # DataFrame
        arrs = tuple((x.__array_interface__["data"][0], x.shape, x.dtype.str)
                     for x in a._mgr.arrays if hasattr(x, "__array_interface__"))
        return ("frame", id(a), tuple(a.shape), arrs, id(a.index), id(a.columns))
    if isinstance(a, np.ndarray):
        return ("array", id(a), a.shape, a.dtype.str, a.__array_interface__["data"][0], a.strides)
    return ("object", id(a))


def _search_frame(data_search):
    """data_search as search_single sees it: without a 'category' column
    (LearnedIndex.py:140-141)."""
    if hasattr(data_search, "columns") and "category" in data_search.columns:
        return data_search.drop("category", axis=1, errors="ignore")
    return data_search


def _dtypes(a) -> set:
    if hasattr(a, "dtypes") and hasattr(a.dtypes, "__iter__"):
        return {np.dtype(t) for t in a.dtypes}
    return {np.asarray(a).dtype}


def dist_dtype(data_search, queries_search) -> str:
    """The arithmetic the reference's distances run in (utils.py:11, :19):
    sklearn's cosine_similarity works in float32 only when both operands are
    float32 (check_pairwise_arrays / _return_float_dtype) and in float64
    otherwise — the clip768 'emb' of the real data is float16, so 'f64'."""
    f32 = {np.dtype(np.float32)}
    return "f32" if _dtypes(_search_frame(data_search)) == f32 and \
        _dtypes(queries_search) == f32 else "f64"


def _upload_queries(queries_search, device) -> torch.Tensor:
    """The clip768 queries on the device: float16 input (the real 'emb')
    crosses PCIe as float16 (half the bytes) and is widened to float32 on the
    device (exact); float64 input stays float64 (the float64 mode computes on
    its values, utils.py:11); anything else as float32."""
    a = np.asarray(queries_search)
    if a.dtype == np.float16:
        return torch.from_numpy(np.ascontiguousarray(a)).to(device).float()
    if a.dtype == np.float64:
        return torch.from_numpy(np.ascontiguousarray(a)).to(device)
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(device)


class LearnedIndex(Logger):

    # class-level defaults for instances unpickled from the reference's
    # pickle (li.index_io.load_index), which hold only `model`
    _cache_key = None
    _index = None
    _trusted = None
    _searcher = None
    _attached_labels = None
    _cat_written = None
    _pg = None        # process-group mode: (group, rank, world, chunk_rows)

    def __init__(self):
        self.model = None
        self._cache_key = None
        self._index = None
        self._trusted = None
        self._searcher = None

    def __getstate__(self):
        """Pickle (save_as_pickle, utils.py:46-60) what the reference pickles:
        the model; the HBM index and its caches stay out of the file."""
        st = dict(self.__dict__)
        for key in ("_index", "_cache_key", "_trusted", "_searcher", "_attached_labels", "_cat_written",
                    "_pg", "_n_builds"):
            st.pop(key, None)
        return st

    # ---- process-group mode --------------------------------------------------
    def use_process_group(self, group=None, chunk_rows=None):
        """Shard this index over the ranks of `group` (default: the default
        process group, which must be initialised: li.dist.init_from_env).
        Rank g builds slice g of every bucket; search / search_single return
        the whole answer on every rank.  `chunk_rows`: the scan's chunk of a
        stripe (default li.index.default_chunk_rows(world, rows) when the
        index is built)."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("use_process_group: torch.distributed is not initialised "
                               "(li.dist.init_from_env)")
        world = dist.get_world_size(group)
        self._pg = (group, dist.get_rank(group), world, int(chunk_rows) if chunk_rows else None)
        self._index = self._searcher = self._cache_key = self._trusted = None
        self._cat_written = None
        return self

    def _proc_group(self):
        """The process-group mode's (group, rank, world, chunk_rows), or None.
        Entered on first use when a launcher set WORLD_SIZE > 1 (torchrun,
        search.py --gpus N), unless LMI_SHARD=0."""
        if self._pg is None and int(os.environ.get("WORLD_SIZE", "1")) > 1 and \
                os.environ.get("LMI_SHARD", "1") != "0":
            from .dist import init_from_env
            init_from_env()
            self.use_process_group()
        return self._pg

    # ---- index ------------------------------------------------------------
    def _identity(self, data_navigation, data_search, labels):
        return (identity_key(data_search), identity_key(labels), identity_key(data_navigation.index))

    def _is_attached(self, data_navigation, data_search, labels) -> bool:
        """The attached objects themselves (held by strong references, so no
        freed object's id() or buffer can be taken for them), with their value
        arrays still where they were at attach time."""
        t = self._trusted
        if t is None or self._index is None or t[1] != self._cache_key:
            return False
        refs = t[2]
        return (refs[0] is data_search and refs[1] is labels and refs[2] is data_navigation.index
                and t[0] == self._identity(data_navigation, data_search, labels))

    def attach(self, data_navigation, data_search, pred_categories):
        """Build the HBM index of data_search (rows in data_navigation's id
        order, bucket labels `pred_categories`) now, outside any timed call,
        and trust these objects: later search / search_single calls that pass
        the same objects (same id, shape, dtype and value arrays) reuse it
        without hashing their bytes.  The caller must not change them in
        place afterwards (or must call attach again).  An addition; the
        reference has no such step (it re-gathers every bucket per call)."""
        self._trusted = None
        self._cat_written = None
        self._device_index(data_navigation, data_search, pred_categories)
        # strong references to the trusted objects: while they are held, their
        # id()s and buffers cannot be reused by new objects
        self._trusted = (self._identity(data_navigation, data_search, pred_categories),
                         self._cache_key, (data_search, pred_categories, data_navigation.index))
        self._attached_labels = pred_categories if isinstance(pred_categories, np.ndarray) else None
        return self._index

    def detach(self):
        """Stop trusting the attached objects (the next call hashes them)."""
        self._trusted = None
        self._cat_written = None

    def _device_index(self, data_navigation, data_search, labels):
        """DeviceIndex of data_search rows in data_navigation order."""
        from .index import DeviceIndex
        if self._is_attached(data_navigation, data_search, labels):
            return self._index
        labels = np.asarray(labels).astype(np.int64)
        ds = _search_frame(data_search)
        ids = np.asarray(data_navigation.index)
        key = (content_key(ds), content_key(labels), content_key(ids),
               content_key(np.asarray(ds.index)) if hasattr(ds, "index") else None)
        if self._index is not None and self._cache_key == key:
            return self._index
        # fp16 data (the real clip768 'emb') stays fp16 on its way to HBM;
        # float64 data keeps its float64 values for the float64 mode
        # (DeviceIndex.corpus64: sklearn computes on them, utils.py:11)
        dts = _dtypes(ds)
        dt = np.float16 if dts == {np.dtype(np.float16)} else \
            np.float64 if np.dtype(np.float64) in dts else np.float32
        if hasattr(ds, "index") and not ds.index.equals(data_navigation.index):
            rows = ds.loc[data_navigation.index].to_numpy(dtype=dt)  # :152-153, :168
        else:
            rows = np.asarray(ds, dtype=dt)
        n_buckets = self._n_buckets(labels)
        self._index = None
        self._searcher = None
        pg = self._proc_group()
        shard = {} if pg is None else dict(rank=pg[1], world=pg[2], chunk_rows=pg[3])
        self._index = DeviceIndex(rows, labels, n_buckets, ids=ids, **shard)
        self._cache_key = key
        return self._index

    def _get_searcher(self, index):
        """One Searcher per cached index (its device tables -- bucket sizes and
        the 80 MB position -> id map at 10M -- are uploaded once)."""
        from .index import Searcher
        router = self.model.router() if self.model is not None else None
        s = self._searcher
        if s is None or s.index is not index or s.router is not router:
            pg = self._proc_group()
            s = self._searcher = Searcher(index, router, None if pg is None else pg[0])
        return s

    def _n_buckets(self, labels):
        if labels.size and labels.min() < 0:
            raise ValueError("categories must be non-negative integers")
        c = int(labels.max()) + 1 if labels.size else 1
        if self.model is not None:
            c = max(c, int(self.model.model.n_output_neurons))
        return c

    # ---- search -------------------------------------------------------------
    def search(self, data_navigation, queries_navigation, data_search, queries_search,
               pred_categories, n_buckets=1, k=10, use_threshold=False, semantics="reference"):
        """Search for k nearest neighbors of each query (LearnedIndex.py:22-101).
        `semantics="exact"` (an addition; default off) returns the exact top-k of
        the union of the probed buckets instead of the reference's round merge."""
        assert self.model is not None, 'Model is not trained, call `build` first.'
        if _AUTO_ATTACH and self._trusted is None:
            self.attach(data_navigation, data_search, pred_categories)
        self._set_category(data_navigation, pred_categories)   # :67 (caller-visible side effect)
        index = self._device_index(data_navigation, data_search, pred_categories)
        q_nav = data_X_to_torch(queries_navigation).to(index.device)
        return self._get_searcher(index).search(q_nav, _upload_queries(queries_search, index.device),
                                                n_buckets, k=k, k_round=10,
                                                use_threshold=use_threshold, semantics=semantics,
                                                dist=dist_dtype(data_search, queries_search))

    def search_single(self, data_navigation, data_search, queries_search, pred_categories,
                      k=10, threshold_dist=None):
        """One bucket per query (LearnedIndex.py:103-195).  `pred_categories`
        is the per-query bucket; object labels come from
        data_navigation['category'] as in the reference's groupby (:143)."""
        from .index import replay, replay_device
        if _AUTO_ATTACH and self._trusted is None:
            self.attach(data_navigation, data_search, np.asarray(data_navigation['category']))
        index = self._device_index(data_navigation, data_search,
                                   data_navigation['category'] if self._trusted is None
                                   else self._labels_of(data_navigation))
        dev = index.device
        q = _upload_queries(queries_search, dev)
        cls = np.asarray(pred_categories).astype(np.int32).reshape(-1, 1)
        classes = torch.from_numpy(cls).to(dev)
        _, d, pos, st = self._get_searcher(index).lists(None, q, 1, k, classes=classes,
                                                        dist=dist_dtype(data_search, queries_search))
        if int(st.item()) & _lib.LMI_STATUS_INTERNAL:
            raise RuntimeError(f"search_single: scan status {int(st.item())}")
        if k > _lib.LMI_REPLAY_DEVICE_MAX_KR:
            # rows wider than the device replay holds: the host replay (C++)
            return replay(cls, d.cpu().numpy(), pos.cpu().numpy(), k_round=k, k_final=k,
                          bucket_size=index.bucket_size, pos_to_id=index.pos_to_id,
                          use_threshold=False, thr_round0=threshold_dist)
        thr = None if threshold_dist is None else torch.from_numpy(
            np.ascontiguousarray(np.asarray(threshold_dist, dtype=np.float64).ravel())).to(dev)
        bsz, p2id = self._get_searcher(index)._device_tables()
        dd, aa, rst = replay_device(classes, d, pos, k_round=k, k_final=k, bucket_size=bsz,
                                    pos_to_id=p2id, use_threshold=False, thr_round0=thr)
        if int(rst.item()):
            raise RuntimeError(f"search_single: replay status {int(rst.item())}")
        return dd.cpu().numpy(), aa.cpu().numpy().view(np.uint32)

    def _set_category(self, data_navigation, pred_categories):
        """data_navigation['category'] = pred_categories (LearnedIndex.py:67),
        except when this call would rewrite the very values the previous call
        wrote: the frame and the labels are the attached objects (attach's
        contract: not changed in place) and the column still holds the array
        written then.  At 10M rows the assignment copies 80 MB inside pandas
        (~10-30 ms), a third of the CLI's querytime."""
        col = lambda: (id(data_navigation),
                       np.asarray(data_navigation["category"]).__array_interface__["data"][0])
        mark = (identity_key(pred_categories), identity_key(data_navigation.index))
        if self._trusted is not None and self._cat_written is not None and \
                pred_categories is self._attached_labels and \
                "category" in getattr(data_navigation, "columns", ()) and \
                self._cat_written == (mark, col()):
            return
        data_navigation['category'] = pred_categories
        self._cat_written = (mark, col()) if self._trusted is not None else None

    def _labels_of(self, data_navigation):
        """data_navigation['category'] as search_single reads it (:143), but
        the attached labels object itself when its values are the attached
        ones (the column is a fresh Series per access, so its identity never
        matches; its values are compared instead: 80 MB at 10M, a memcmp)."""
        col = np.asarray(data_navigation['category'])
        lab = self._attached_labels
        if lab is not None and lab.shape == col.shape and np.array_equal(lab, col):
            return lab
        return col

    # ---- build (outside the hot path) -------------------------------------
    def build(self, data, n_categories=100, epochs=100, lr=0.1, model_type='MLP'):
        """LearnedIndex.py:197-240: cluster, train the router, label the data
        with the router's argmax (predict on the GPU router kernel)."""
        s = time.time()
        pg = self._proc_group()
        if pg is None or pg[1] == 0:
            try:
                _, labels = self.cluster(data, n_categories)
                dataset = LIDataset(data, labels)
                train_loader = torch.utils.data.DataLoader(
                    dataset, batch_size=256,
                    sampler=torch.utils.data.SubsetRandomSampler(data.index.values.tolist()))
                nn = NeuralNetwork(input_dim=data.shape[1], output_dim=n_categories, lr=lr,
                                   model_type=model_type)
                nn.train_batch(train_loader, epochs=epochs, logger=self.logger)
                self.model = nn
                pred = nn.predict(data_X_to_torch(data))
            except BaseException as e:
                if pg is not None:
                    self._build_done(pg, repr(e)[:500])
                raise
        if pg is not None:
            # the other ranks wait for rank 0's build on the rendezvous store,
            # outside any collective: the build (k-means + 100 epochs of
            # training) may take far longer than the process group's timeout
            # (LMI_DIST_TIMEOUT_S), which then bounds only the broadcast
            self._build_done(pg, None)
            # every rank must index the same buckets: rank 0's router and
            # labels, broadcast (GPU training is not promised bit-reproducible)
            pred = self._share_build(pg, None if pg[1] else (self.model, pred),
                                     data.shape[1], n_categories, lr, model_type)
        return pred, time.time() - s

    def _build_done(self, pg, error):
        """Rank 0: publish that the build ended (`error`: its message, or None).
        Other ranks: wait for that key on the default group's store, polling,
        for at most LMI_BUILD_TIMEOUT_S (default 86400 s), and raise rank 0's
        error if it failed.  A store key per build call (builds are called in
        the same order on every rank)."""
        import torch.distributed as dist
        store = dist.distributed_c10d._get_default_store()
        self._n_builds = getattr(self, "_n_builds", 0) + 1
        key = f"lmi_build_{self._n_builds}"
        if pg[1] == 0:
            store.set(key, "ok" if error is None else "ERR " + error)
            return
        deadline = time.monotonic() + float(os.environ.get("LMI_BUILD_TIMEOUT_S", "86400"))
        while not store.check([key]):
            if time.monotonic() > deadline:
                raise RuntimeError(f"rank {pg[1]}: rank 0's build did not finish in time")
            time.sleep(0.2)
        got = store.get(key).decode()
        if got != "ok":
            raise RuntimeError(f"rank 0's build failed: {got[4:]}")

    def _share_build(self, pg, built, input_dim, n_categories, lr, model_type):
        """Broadcast rank 0's trained router (state_dict) and object labels to
        every rank of the process group; returns the labels."""
        import torch.distributed as dist
        group = pg[0]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        if built is not None:
            nn, pred = built
            state = {k: v.detach().cpu().numpy() for k, v in nn.model.state_dict().items()}
            obj = [(state, np.asarray(pred), nn.model.n_output_neurons)]
        else:
            obj = [None]
        dist.broadcast_object_list(obj, src=src, group=group)
        state, pred, n_out = obj[0]
        if built is None:
            nn = NeuralNetwork(input_dim=input_dim, output_dim=n_out, lr=lr, model_type=model_type)
            nn.model.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})
            self.model = nn
        return pred

    def cluster(self, data, n_clusters):
        """LearnedIndex.py:242-282: k-means labels of the navigation data.  The
        reference's faiss.Kmeans(d, k, seed=2023) is replaced by li.kmeans.Kmeans
        (same API and defaults, GPU kernels csrc/lmi_kmeans.hip)."""
        from .kmeans import Kmeans
        if data.shape[0] < 2:
            return None, np.zeros_like(data.shape[0])
        if data.shape[0] < n_clusters:
            n_clusters = data.shape[0] // 5
            if n_clusters < 2:
                n_clusters = 2
        X = np.array(data).astype(np.float32)
        kmeans = Kmeans(d=X.shape[1], k=n_clusters, verbose=False, seed=2023)
        kmeans.train(X)
        return kmeans, kmeans.index.search(X, 1)[1].T[0]
