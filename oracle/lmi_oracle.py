"""CPU restatement of the reference's LMI search hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker (or as the
timed CPU baseline "port").  The product path (li/, liblmi_hip.so) never
calls it; there is no CPU fallback.

Every function restates a piece of TerkaSlan/sisap23-laion-challenge-learned-index
(paths relative to that repository) with numpy, in the reference's dtypes:

  normalize            sklearn.preprocessing.normalize as used by
                       utils.py:10-11 (cosine_similarity) and search.py:50-52
  pairwise_cosine      utils.py:10-11
  pairwise_cosine_threshold  utils.py:14-43
  blas32_*             utils.py:10-11's float32 arithmetic operation by
                       operation (numpy einsum + OpenBLAS sgemm orders, round 6)
  mlp_forward / predict_proba / predict   model.py:15-83, :201-229
  search_single_direct / search_direct   LearnedIndex.py:22-195, restated
                       line by line (full distance matrices, no shortcut)
  bucket_lists + replay  the decomposition the GPU path implements
                       

Parity is pinned: tests/test_oracle_golden.py checks search_direct and the
router against fixtures produced by running the reference itself
(tests/golden/gen_golden.py), and checks bucket_lists + replay against
search_direct.
"""
from __future__ import annotations

import numpy as np

FILL = 10_000.0  # LearnedIndex.py:138, utils.py:35


# ---------------------------------------------------------------------------
# distances (utils.py)
# ---------------------------------------------------------------------------
def _float_dtype(x, y):
    # sklearn _return_float_dtype: float32 only if both are float32
    return np.float32 if (x.dtype == np.float32 and y.dtype == np.float32) else np.float64


def normalize(x: np.ndarray) -> np.ndarray:
    """sklearn normalize(norm='l2'): x / sqrt(einsum(x*x)), norms < 10*eps -> 1."""
    x = np.array(x, copy=True)
    norms = np.sqrt(np.einsum("ij,ij->i", x, x))
    norms[norms < 10 * np.finfo(norms.dtype).eps] = 1.0
    x /= norms[:, None]
    return x


def pairwise_cosine(x, y):
    """utils.py:10-11: 1 - cosine_similarity(x, y)."""
    dt = _float_dtype(np.asarray(x), np.asarray(y))
    xn = normalize(np.asarray(x, dtype=dt))
    yn = normalize(np.asarray(y, dtype=dt))
    return 1 - xn @ yn.T


def pairwise_cosine_threshold(x, y, threshold, cat_idxs, k=10):
    """utils.py:14-43 (returns (None, t) when nothing beats the threshold)."""
    result = pairwise_cosine(x, y)
    thresh_consistent = np.repeat(threshold[cat_idxs, np.newaxis], result.shape[1], 1)
    relevant_dists = np.where(result < thresh_consistent)
    relevant_object_ids = np.unique(relevant_dists[1])
    max_idx = relevant_object_ids.shape[0]
    if max_idx == 0:
        return None, 0.0
    max_idx = max_idx if max_idx > k else k
    output_arr = np.full(shape=(result.shape[0], max_idx), fill_value=FILL, dtype=float)
    mapping = dict(zip(relevant_object_ids, np.arange(relevant_object_ids.shape[0])))
    output_arr_2nd_dim = np.array([mapping[v] for v in relevant_dists[1]])
    to_be_added = result[relevant_dists[0], relevant_dists[1]]
    output_arr[relevant_dists[0], output_arr_2nd_dim] = to_be_added
    return output_arr, relevant_object_ids, 0.0


# ---------------------------------------------------------------------------
# the reference's float32 arithmetic, operation by operation (round 6)
# ---------------------------------------------------------------------------
# utils.py:10-11 in float32 is sklearn's normalize (row norms by
# np.einsum('ij,ij->i'), then an in-place division) and a float32 GEMM
# (numpy.matmul -> OpenBLAS sgemm), then 1 - S.  The summation orders below
# restate the third-party code the reference runs on in this container --
# numpy 2.2's einsum sum-of-products loop (SSE baseline: four float32 lanes,
# the four vectors of each 16-element group multiplied and added in reverse
# order, no FMA, lanes summed (0+1)+(2+3)) and OpenBLAS 0.3.29's SkylakeX
# sgemm (a small-matrix kernel when M*N*K <= 96*96*100: sixteen FMA chains
# over k mod 16, summed pairwise -- by halves in the product's corner block
# of the last M mod 4 queries x the last N mod 4 rows; else the blocked
# kernel: one FMA chain per K block of 384, the blocks' sums added) -- found by bitwise search against
# numpy and pinned by tests/test_oracle_blas32.py.  Shapes it does not cover
# (a group of one query or one row -- OpenBLAS forwards those to gemv, whose
# order depends on its thread split -- and groups of at most 3 x 3) return
# None.  The GPU's split mode (x_select_wave_kernel) computes these values.
_BLAS_SMALL_MNK = 96 * 96 * 100
_BLAS_KBLOCK = 384


def _f32(x):
    return np.asarray(x, dtype=np.float32)


def blas32_row_norms(x: np.ndarray) -> np.ndarray:
    """np.einsum('ij,ij->i', x, x) for float32 rows whose length is a
    multiple of 16, in numpy's summation order (see above)."""
    x = np.asarray(x, dtype=np.float32)
    n, d = x.shape
    if d % 16:
        raise ValueError("rows of a multiple of 16 elements")
    acc = np.zeros((4, n), np.float32)
    for g in range(0, d, 16):
        for v in (3, 2, 1, 0):
            blk = x[:, g + 4 * v:g + 4 * v + 4]
            acc += (blk * blk).T            # (float32 product, then float32 add)
    return (acc[0] + acc[1]) + (acc[2] + acc[3])


def blas32_normalize(x: np.ndarray) -> np.ndarray:
    """sklearn normalize(x) in float32, operation by operation."""
    x = np.asarray(x, dtype=np.float32)
    norms = np.sqrt(blas32_row_norms(x))
    norms[norms < 10 * np.finfo(np.float32).eps] = np.float32(1.0)
    return x / norms[:, None]


def _fma_chain(a, b):
    """sum_k a[:, k] * b[:, k] as one FMA chain in ascending k (float32 with
    one rounding per step: the float64 product of two float32 values is
    exact, so float64 add-then-round is the FMA)."""
    acc = np.zeros(a.shape[0], np.float32)
    for k in range(a.shape[1]):
        acc = (acc.astype(np.float64) + a[:, k].astype(np.float64) * b[:, k].astype(np.float64)
               ).astype(np.float32)
    return acc


def blas32_kernel(M: int, N: int, K: int):
    """Which OpenBLAS sgemm path the reference's (M queries x N rows) float32
    product takes: "small", "blocked", or None (gemv / tiny: not restated)."""
    if M <= 1 or N <= 1 or (M <= 3 and N <= 3) or K % 16:
        return None
    return "small" if M * N * K <= _BLAS_SMALL_MNK else "blocked"


def blas32_dot(qn: np.ndarray, yn: np.ndarray, kernel: str, corner=None) -> np.ndarray:
    """Row-wise dot of normalised float32 vectors qn[i] . yn[i] in the order of
    `kernel` (blas32_kernel).  The small kernel sums its sixteen chains
    pairwise ((0+1)+(2+3)...) except in the corner block of the product --
    query i >= 4 floor(M/4) of its group and row j >= 4 floor(N/4) of its
    bucket -- where it sums them by halves ((0+8)+(4+12)...): `corner`, a
    boolean per dot (default none)."""
    qn, yn = _f32(qn), _f32(yn)
    K = qn.shape[1]
    if kernel == "small":
        parts = [_fma_chain(qn[:, l::16], yn[:, l::16]) for l in range(16)]
        pair, half = list(parts), list(parts)
        while len(pair) > 1:
            pair = [pair[2 * i] + pair[2 * i + 1] for i in range(len(pair) // 2)]
            h = len(half) // 2
            half = [half[i] + half[i + h] for i in range(h)]
        return pair[0] if corner is None else np.where(corner, half[0], pair[0])
    tot = None
    for a in range(0, K, _BLAS_KBLOCK):
        c = _fma_chain(qn[:, a:a + _BLAS_KBLOCK], yn[:, a:a + _BLAS_KBLOCK])
        tot = c if tot is None else tot + c
    return tot


def blas32_pairwise_cosine(x, y):
    """pairwise_cosine(x, y) of float32 x [M, d] (a group's queries) and y [N,
    d] (a bucket's rows) from the restated operations; None when the shape's
    kernel is not restated.  Equals pairwise_cosine bit for bit in this
    container (tests/test_oracle_blas32.py)."""
    x, y = _f32(x), _f32(y)
    kern = blas32_kernel(x.shape[0], y.shape[0], x.shape[1])
    if kern is None:
        return None
    xn, yn = blas32_normalize(x), blas32_normalize(y)
    M, N = xn.shape[0], yn.shape[0]
    ii, jj = np.meshgrid(np.arange(M), np.arange(N), indexing="ij")
    corner = ((ii >= M // 4 * 4) & (jj >= N // 4 * 4)).reshape(-1)
    S = blas32_dot(np.repeat(xn, N, axis=0), np.tile(yn, (M, 1)), kern, corner).reshape(M, N)
    return np.float32(1) - S


# ---------------------------------------------------------------------------
# router (model.py)
# ---------------------------------------------------------------------------
def mlp_forward(x: np.ndarray, layers) -> np.ndarray:
    """Linear/ReLU stack, torch layout W[out][in]: y = x W^T + b (fp32)."""
    h = np.asarray(x, dtype=np.float32)
    for i, (w, b) in enumerate(layers):
        h = h @ np.asarray(w, np.float32).T + np.asarray(b, np.float32)
        if i + 1 < len(layers):
            h = np.maximum(h, 0)
    return h.astype(np.float32)


def softmax(logits: np.ndarray) -> np.ndarray:
    m = logits.max(axis=1, keepdims=True)
    e = np.exp(logits - m)
    return (e / e.sum(axis=1, keepdims=True)).astype(np.float32)


def rank_classes(logits: np.ndarray) -> np.ndarray:
    """Classes by descending logit, ties to the lower index (= topk of softmax)."""
    n, c = logits.shape
    idx = np.broadcast_to(np.arange(c), (n, c))
    return np.lexsort((idx, -logits.astype(np.float64)), axis=1).astype(np.int64)


def predict_proba(x, layers):
    """model.py:214-229: (probs sorted desc, classes) over all classes."""
    logits = mlp_forward(x, layers)
    probs = softmax(logits)
    classes = rank_classes(logits)
    return np.take_along_axis(probs, classes, axis=1), classes


def predict(x, layers):
    """model.py:201-212: argmax of the logits (first index on ties)."""
    return np.argmax(mlp_forward(x, layers), axis=1).astype(np.int64)


# ---------------------------------------------------------------------------
# literal restatement of LearnedIndex.search / search_single
# ---------------------------------------------------------------------------
def _stable_argsort_rows(a: np.ndarray) -> np.ndarray:
    # the reference's quicksort on rows of <= 16 values is numpy<=1.24's
    # insertion sort, i.e. stable; longer rows only matter through ties
    return np.argsort(a, kind="stable", axis=-1)


def search_single_direct(labels, ids, data_search, queries_search, pred_categories, k=10,
                         threshold_dist=None):
    """LearnedIndex.py:103-195 with data_navigation = (labels, ids) in row order
    and data_search rows aligned with ids."""
    labels = np.asarray(labels)
    ids = np.asarray(ids)
    nq = queries_search.shape[0]
    nns = np.zeros((nq, k), dtype=np.uint32)
    dists = np.full(shape=(nq, k), fill_value=FILL, dtype=float)
    for cat in np.unique(labels):                          # groupby('category'), ascending
        rows = np.nonzero(labels == cat)[0]                 # g, in row order
        cat_idxs = np.where(pred_categories == cat)[0]      # :144
        bucket_obj_indexes = ids[rows]                      # :145 g.index
        if bucket_obj_indexes.shape[0] != 0 and cat_idxs.shape[0] != 0:
            if threshold_dist is not None:
                seq = pairwise_cosine_threshold(queries_search[cat_idxs], data_search[rows],
                                                threshold_dist, cat_idxs, k)
                if seq[0] is None:
                    continue
                bucket_obj_indexes = bucket_obj_indexes[seq[1]]
                seq = seq[0]
            else:
                seq = pairwise_cosine(queries_search[cat_idxs], data_search[rows])
            ann_relative = _stable_argsort_rows(seq)[:, :k if k < seq.shape[1] else seq.shape[1]]
            if bucket_obj_indexes.shape[0] < k:             # :174-190
                pad_needed = (k - bucket_obj_indexes.shape[0]) // 2 + 1
                bucket_obj_indexes = np.pad(np.array(bucket_obj_indexes), pad_needed, "edge")[:k]
                ann_relative = np.pad(ann_relative[0], pad_needed, "edge")[:k].reshape(1, -1)
                seq = np.pad(seq[0], pad_needed, "edge")[:k].reshape(1, -1)
                _, i = np.unique(seq, return_index=True)
                duplicates_i = np.setdiff1d(np.arange(k), i)
                seq[0][duplicates_i] = FILL
            nns[cat_idxs] = np.array(bucket_obj_indexes)[ann_relative]
            dists[cat_idxs] = np.take_along_axis(seq, ann_relative, axis=1)
    return dists, nns


def search_direct(labels, ids, data_search, queries_search, classes, n_buckets=1, k=10,
                  use_threshold=False):
    """LearnedIndex.py:22-101 given the router's classes (nq, >=R)."""
    anns_final = dists_final = None
    for bucket in range(n_buckets):
        threshold_dist = dists_final.max(axis=1) if (bucket != 0 and use_threshold) else None
        dists, anns = search_single_direct(labels, ids, data_search, queries_search,
                                           classes[:, bucket], threshold_dist=threshold_dist)
        if anns_final is None:
            anns_final, dists_final = anns, dists
        else:
            anns_final = np.hstack((anns_final, anns))
            dists_final = np.hstack((dists_final, dists))
            idx_sorted = dists_final.argsort(kind="stable", axis=1)[:, :k]
            dists_final = np.take_along_axis(dists_final, idx_sorted, axis=1)
            anns_final = np.take_along_axis(anns_final, idx_sorted, axis=1)
            assert anns_final.shape == dists_final.shape == (queries_search.shape[0], k)
    return dists_final, anns_final


# ---------------------------------------------------------------------------
# decomposition: per-(query, probe) lists + replay
# ---------------------------------------------------------------------------
def layout(labels, n_buckets):
    """Bucket-sorted order (stable in row order) and bucket offsets."""
    lab = np.asarray(labels).astype(np.int64)
    order = np.argsort(lab, kind="stable")
    off = np.zeros(n_buckets + 1, np.int64)
    np.cumsum(np.bincount(lab, minlength=n_buckets), out=off[1:])
    return order, off


def bucket_lists(labels, data_search, queries_search, classes, R, k, n_buckets):
    """Exact per-(q, r) top-k inside bucket classes[q, r], ordered by
    (distance, position), padded with (inf, -1).  Distances are computed per
    (r, c) group with the same shapes the reference uses (LearnedIndex.py:166-169),
    in the reference's dtype: float32 for float32 inputs, float64 otherwise
    (sklearn's rule, utils.py:11)."""
    order, off = layout(labels, n_buckets)
    nq = queries_search.shape[0]
    dt = _float_dtype(np.asarray(queries_search), np.asarray(data_search))
    out_d = np.full((nq, R, k), np.inf, dt)
    out_p = np.full((nq, R, k), -1, np.int32)
    for r in range(R):
        col = classes[:, r]
        for c in np.unique(col):
            if c < 0 or c >= n_buckets:
                continue
            a, b = off[c], off[c + 1]
            if a == b:
                continue
            G = np.nonzero(col == c)[0]
            D = pairwise_cosine(queries_search[G], data_search[order[a:b]])
            pos = np.arange(a, b)
            for gi, q in enumerate(G):
                row = D[gi]
                o = np.lexsort((pos, row))[:k]
                out_d[q, r, : o.size] = row[o]
                out_p[q, r, : o.size] = pos[o]
    return out_d, out_p


def _edge_take(a, p, k):
    return np.pad(np.asarray(a), p, "edge")[:k]


def _quirk(row, u_pos, kr):
    ann = np.argsort(np.asarray(row, dtype=np.float64), kind="stable")
    p = (kr - len(u_pos)) // 2 + 1
    ids_p = _edge_take(u_pos, p, kr)
    ann_p = _edge_take(ann, p, kr)
    row_p = _edge_take(np.asarray(row, np.float64), p, kr).copy()
    _, i = np.unique(row_p, return_index=True)
    row_p[np.setdiff1d(np.arange(kr), i)] = FILL
    return row_p[ann_p], ids_p[ann_p]


def replay(classes, lists_d, lists_pos, *, k_round, k_final, bucket_size, pos_to_id,
           use_threshold, thr_round0=None, stats=None):
    """Python twin of lmi_replay (csrc/lmi_replay.cpp): LearnedIndex.py:22-195
    replayed from the per-(query, probe) lists.  `stats` (a dict) counts the
    branches taken: groups, quirk0 (bucket < k), quirk_thr (|U| < k),
    skipped (no object beats the threshold), fillers."""
    st = stats if stats is not None else {}
    for key in ("groups", "quirk0", "quirk_thr", "skipped", "fillers"):
        st.setdefault(key, 0)
    classes = np.asarray(classes)
    if classes.ndim == 1:
        classes = classes[:, None]
    nq, R = classes.shape
    kr = k_round
    lists_d = np.asarray(lists_d).reshape(nq, R, -1)
    lists_pos = np.asarray(lists_pos).reshape(nq, R, -1)
    F_d = F_p = None
    for r in range(R):
        Dd = np.full((nq, kr), FILL)
        Dp = np.full((nq, kr), -1, np.int64)
        thresholded = (r > 0 and use_threshold) or (r == 0 and thr_round0 is not None)
        if thresholded:
            thr = np.asarray(thr_round0, np.float64) if r == 0 else F_d.max(axis=1)
        col = classes[:, r]
        for c in range(len(bucket_size)):
            G = np.nonzero(col == c)[0]
            if G.size == 0 or bucket_size[c] <= 0:
                continue
            st["groups"] += 1
            if thresholded:
                B = {}
                for q in G:
                    sel = []
                    for j in range(min(kr, lists_d.shape[2])):
                        d, p = float(lists_d[q, r, j]), int(lists_pos[q, r, j])
                        if p < 0 or not d < thr[q]:
                            break
                        sel.append((d, p))
                    B[q] = sel
                U = sorted({p for q in G for _, p in B[q]})
                if not U:
                    st["skipped"] += 1
                    continue
                if len(U) >= kr:
                    for q in G:
                        ent = list(B[q])[:kr]
                        mine = {p for _, p in ent}
                        fill = [(FILL, p) for p in U if p not in mine][: kr - len(ent)]
                        st["fillers"] += len(fill)
                        ent += fill
                        Dd[q] = [e[0] for e in ent]
                        Dp[q] = [e[1] for e in ent]
                else:
                    st["quirk_thr"] += 1
                    q0 = G[0]
                    row = np.full(kr, FILL)
                    for d, p in B[q0]:
                        row[U.index(p)] = d
                    dd, pp = _quirk(row, np.asarray(U), kr)
                    Dd[G] = dd
                    Dp[G] = pp
            else:
                n = int(bucket_size[c])
                if n >= kr:
                    Dd[G] = lists_d[G, r, :kr]
                    Dp[G] = lists_pos[G, r, :kr]
                else:
                    st["quirk0"] += 1
                    q0 = G[0]
                    ent = sorted((int(lists_pos[q0, r, j]), float(lists_d[q0, r, j])) for j in range(n))
                    dd, pp = _quirk([e[1] for e in ent], np.asarray([e[0] for e in ent]), kr)
                    Dd[G] = dd
                    Dp[G] = pp
        if r == 0:
            F_d, F_p = Dd, Dp
        else:
            cd = np.hstack((F_d, Dd))
            cp = np.hstack((F_p, Dp))
            o = cd.argsort(kind="stable", axis=1)[:, :k_final]
            F_d = np.take_along_axis(cd, o, axis=1)
            F_p = np.take_along_axis(cp, o, axis=1)
            assert F_d.shape == (nq, k_final)
    anns = np.where(F_p >= 0, np.asarray(pos_to_id)[np.maximum(F_p, 0)], 0).astype(np.uint32)
    return F_d.astype(np.float64), anns


def search_via_lists(labels, ids, data_search, queries_search, classes, n_buckets, R, k=10,
                     use_threshold=False, k_round=10):
    """bucket_lists + replay: must equal search_direct."""
    order, off = layout(labels, n_buckets)
    d, p = bucket_lists(labels, data_search, queries_search, classes, R, k_round, n_buckets)
    return replay(classes[:, :R], d, p, k_round=k_round, k_final=k,
                  bucket_size=np.diff(off), pos_to_id=np.asarray(ids)[order],
                  use_threshold=use_threshold)


# ---------------------------------------------------------------------------
# comparator
# ---------------------------------------------------------------------------
def compare_lists(d_a, p_a, d_b, p_b, *, atol=1e-5, tie=1e-6, stats=None):
    """Tie-aware comparison of per-row sorted lists.

    A row matches when (a) the finite masks agree and |d_a - d_b| <= atol
    elementwise, and (b) every position whose ids differ is explained by a
    tie: list b's id sits elsewhere in list a at a distance within `tie` of
    this position, or — if a does not hold it at all — its distance is within
    `tie` of a's last entry (the k-th place was cut inside a run of ties).
    Returns the number of rows that do not match.  `stats` (a dict) receives
    the counts: rows, mismatched rows, and `tie_rows` = matching rows whose
    ids differ somewhere, i.e. rows that matched only through the tie window
    (`exact_tie_rows`: of those, rows where every differing id sits at
    exactly the same distance in both lists)."""
    d_a = np.asarray(d_a, np.float64)
    k = d_a.shape[-1]
    d_a = d_a.reshape(-1, k)
    d_b = np.asarray(d_b, np.float64).reshape(-1, k)
    p_a = np.asarray(p_a).reshape(-1, k)
    p_b = np.asarray(p_b).reshape(-1, k)
    bad = tie_rows = exact_tie_rows = 0
    for i in range(d_a.shape[0]):
        fa, fb = np.isfinite(d_a[i]), np.isfinite(d_b[i])
        if not np.array_equal(fa, fb) or np.any(np.abs(d_a[i][fa] - d_b[i][fb]) > atol):
            bad += 1
            continue
        diff = np.nonzero(p_a[i] != p_b[i])[0]
        exact = True
        for j in diff:
            where = np.nonzero(p_a[i] == p_b[i][j])[0]
            if where.size:
                gap = abs(d_a[i][where[0]] - d_a[i][j])
            else:
                gap = abs(d_b[i][j] - d_a[i][fa][-1]) if fa.any() else np.inf
            exact = exact and gap == 0
            if not gap <= tie:
                bad += 1
                break
        else:
            if diff.size:
                tie_rows += 1
                exact_tie_rows += 1 if exact else 0
    if stats is not None:
        stats.update(rows=int(d_a.shape[0]), mismatched=int(bad), tie_rows=int(tie_rows),
                     exact_tie_rows=int(exact_tie_rows), tie=tie, atol=atol)
    return bad


# ---------------------------------------------------------------------------
# k-means for the index build (LearnedIndex.py:242-282)
#
# The reference calls faiss.Kmeans(d, k, verbose=True, seed=2023).train(X)
# and labels with kmeans.index.search(X, 1) (LearnedIndex.py:275-282).  faiss
# (1.7.x, pinned by the reference's environment, not vendored and not in this
# image) is restated from its published Clustering::train: subsample to
# k * max_points_per_centroid points, initialise with k random training
# points, niter Lloyd iterations (assign, mean update, split of empty
# clusters).  faiss's own RNG (mt19937 behind faiss::RandomGenerator) is
# replaced by numpy RandomState streams with the same seeds, so sample, init
# and split choices are NOT faiss's: "parity unpinned" against faiss itself.
# The Lloyd arithmetic is pinned against sklearn's KMeans (lloyd, explicit
# init) in tests/test_kmeans.py, and the GPU kernels (csrc/lmi_kmeans.hip)
# are checked bit for bit against the functions below.
# ---------------------------------------------------------------------------
KMEANS_SLICES = 512
KMEANS_EPS = np.float32(1.0 / 1024.0)


def kmeans_assign(x: np.ndarray, cent: np.ndarray):
    """argmin_j Σ_e (x_e - c_je)², fp32, e ascending, each op rounded
    separately (the kernel's exact arithmetic); ties -> lower j (faiss's
    IndexFlatL2 argmin order)."""
    x = np.ascontiguousarray(x, np.float32)
    cent = np.ascontiguousarray(cent, np.float32)
    acc = np.zeros((x.shape[0], cent.shape[0]), np.float32)
    for e in range(x.shape[1]):
        t = x[:, e, None] - cent[None, :, e]
        acc = acc + t * t
    lab = acc.argmin(1).astype(np.int32)
    return lab, acc[np.arange(x.shape[0]), lab]


def kmeans_slices(n: int) -> int:
    return int(max(1, min(KMEANS_SLICES, (n + 127) // 128)))


def kmeans_update(x: np.ndarray, labels: np.ndarray, cent: np.ndarray):
    """Mean of every cluster: fp64 sums per slice in point order, slices added
    in order, rounded once to fp32 (faiss compute_centroids, deterministic
    order of the kernel).  Empty clusters keep their row."""
    n, d = x.shape
    k = cent.shape[0]
    S = kmeans_slices(n)
    tot = np.zeros((k, d), np.float64)
    cnt = np.zeros(k, np.int64)
    for s in range(S):
        a, b = s * n // S, (s + 1) * n // S
        part = np.zeros((k, d), np.float64)
        np.add.at(part, labels[a:b], x[a:b].astype(np.float64))  # sequential, point order
        tot += part
        cnt += np.bincount(labels[a:b], minlength=k)
    out = cent.astype(np.float32).copy()
    nz = cnt > 0
    out[nz] = (tot[nz] / cnt[nz, None]).astype(np.float32)
    return out, cnt


def kmeans_split_empty(cent: np.ndarray, counts: np.ndarray, n: int, rng) -> int:
    """faiss split_clusters: every empty centroid copies a cluster cj picked
    with probability (|cj| - 1)/(n - k) (scanning cj cyclically), both are
    perturbed by ±EPS on alternating dimensions, and cj's count is halved."""
    k = cent.shape[0]
    nsplit = 0
    for ci in range(k):
        if counts[ci] != 0:
            continue
        cj = 0
        while True:
            p = np.float32((counts[cj] - 1.0) / float(np.float32(n - k)))
            r = np.float32(rng.random_sample())
            if r < p:
                break
            cj = (cj + 1) % k
        cent[ci] = cent[cj]
        cent[ci, 0::2] *= np.float32(1) + KMEANS_EPS
        cent[cj, 0::2] *= np.float32(1) - KMEANS_EPS
        cent[ci, 1::2] *= np.float32(1) - KMEANS_EPS
        cent[cj, 1::2] *= np.float32(1) + KMEANS_EPS
        counts[ci] = counts[cj] // 2
        counts[cj] -= counts[ci]
        nsplit += 1
    return nsplit


def kmeans_train_sample(n: int, k: int, seed: int, max_points_per_centroid: int = 256):
    """Rows of X that faiss trains on: all, or a seeded sample of k·mppc."""
    if n > k * max_points_per_centroid:
        return np.random.RandomState(seed).permutation(n)[: k * max_points_per_centroid]
    return np.arange(n)


def kmeans_train(x: np.ndarray, k: int, *, niter: int = 25, seed: int = 1234,
                 max_points_per_centroid: int = 256):
    """faiss Clustering::train restated (see the block comment above);
    returns (centroids [k, d] f32, per-iteration objective list)."""
    x = np.ascontiguousarray(x, np.float32)
    xt = x[kmeans_train_sample(x.shape[0], k, seed, max_points_per_centroid)]
    n = xt.shape[0]
    if n < k:
        raise ValueError(f"{n} training points for {k} centroids")
    cent = xt[np.random.RandomState(seed + 1).permutation(n)[:k]].copy()
    rng = np.random.RandomState(1234)
    obj = []
    for _ in range(niter):
        lab, dist = kmeans_assign(xt, cent)
        obj.append(float(dist.astype(np.float64).sum()))
        cent, cnt = kmeans_update(xt, lab, cent)
        kmeans_split_empty(cent, cnt, n, rng)
    return cent, obj


def search_exact(labels, ids, data_search, queries_search, classes, n_buckets, R, k=10):
    """The `semantics="exact"` option (not a reference behaviour; SURVEY.md
    §8(a) asks for it beside the reference semantics): per query, the exact
    top-k by (distance, bucket-sorted position) over the union of its R probed
    buckets, ids 1-based as DataFrame.index, padded with (10000, 0)."""
    order, _ = layout(labels, n_buckets)
    d, p = bucket_lists(labels, data_search, queries_search, classes, R, k, n_buckets)
    nq = d.shape[0]
    out_d = np.full((nq, k), FILL, np.float64)
    out_a = np.zeros((nq, k), np.uint32)
    for q in range(nq):
        dd, pp = d[q].ravel(), p[q].ravel()
        m = pp >= 0
        dd, pp = dd[m], pp[m]
        o = np.lexsort((pp, dd))[:k]
        out_d[q, : o.size] = dd[o]
        out_a[q, : o.size] = np.asarray(ids)[order[pp[o]]]
    return out_d, out_a
