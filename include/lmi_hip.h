/*
 * lmi_hip.h — C-ABI of liblmi_hip.so, the MI355X (gfx950) implementation of the
 * LMI search hot path of TerkaSlan/sisap23-laion-challenge-learned-index.
 *
 * The reference has no native code and no FFI: its hot path is Python calling
 * torch / sklearn / numpy.  Each entry point below replaces
 * one piece of that Python path; the reference file:line it stands in for is
 * cited per function.  The ctypes binding a maintainer adds on the reference
 * side is in INTEGRATION.md; this repo's own binding is li/_lib.py.
 *
 * Conventions (all entry points):
 *   - plain pointers and sizes only; "device" pointers are HIP device memory
 *     owned by the caller; "host" pointers are ordinary host memory;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *     device entry points are asynchronous on that stream, never allocate and
 *     never synchronise (workspace is passed in), so they can be captured in
 *     a hipGraph;
 *   - return 0 (LMI_OK) or an LMI_E_* code; lmi_last_error() gives text
 *     (thread-local).  No C++ exception crosses the ABI.
 *   - results are deterministic: no float atomics in any reduction; every
 *     top-k list is ordered by (distance, position) ascending, which is the
 *     reference's order on tie-free inputs (LearnedIndex.py:170, :91).
 */
#ifndef LMI_HIP_H
#define LMI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LMI_ABI_VERSION 13

/* ---- status codes ---------------------------------------------------- */
#define LMI_OK 0
#define LMI_E_INVALID 1001     /* bad argument (shape, null pointer, range) */
#define LMI_E_UNSUPPORTED 1002 /* valid request this build does not implement */
#define LMI_E_WORKSPACE 1003   /* workspace too small */
#define LMI_E_HIP 1004         /* a HIP runtime call failed */

/* bits of the device status word written by lmi_bucket_topk */
#define LMI_STATUS_QUERY_NOT_F16 1 /* qmode=LMI_Q_F16 but a query is not fp16-exact */
#define LMI_STATUS_INTERNAL 2      /* a list entry held an out-of-range row (a scan bug): the
                                      entry was dropped instead of read out of bounds */

/* ---- element types / modes ------------------------------------------ */
#define LMI_F32 0
#define LMI_F16 1

#define LMI_ROUTER_TOPR 0   /* softmax + classes sorted by probability (predict_proba) */
#define LMI_ROUTER_ARGMAX 1 /* argmax of logits (predict)                               */

#define LMI_Q_F16 0 /* queries are fp16-representable: exact fp16 MFMA path        */
#define LMI_Q_F32 1 /* general queries: exact-fp32 MFMA path (16x the MFMA time)   */
/* ABI 6, a flag OR-ed into qmode (lmi_bucket_topk / lmi_bucket_topk_f64*, k <=
 * LMI_MAX_K): the lists of probes r >= 1 are needed only below the pair's
 * round-0 k-th distance -- the reference's thresholded rounds compare every
 * later-round object with the running k-th distance, which is never larger
 * than round 0's (LearnedIndex.py:71-75, utils.py:23; the merges only lower
 * it, :86-97) -- so the scan starts every (q, r >= 1) pair with the bound of
 * pair (q, 0) (plus 2 eps in the float64 mode) and its list holds the top-k of
 * the objects at or under that bound.  Only for the replay with thresholds
 * (use_threshold); the lists of r = 0 are unchanged. */
#define LMI_Q_SEED_ROUND0 0x100
/* ABI 7, flags OR-ed into qmode (lmi_bucket_topk / lmi_bucket_topk_f64*, k <=
 * LMI_MAX_K): run only some phases of the call, so that a caller can overlap
 * one batch's plan with another batch's scan (a stream of batches, each with
 * its own workspace, lists and status word).  The phases, in order: PLAN (the
 * queries' fragments and norms, the output prefill, the tile plan, the seed
 * map, the tail split, the bound reset), SCAN (the scan kernel), MERGE (the
 * chunk merge; in lmi_bucket_topk_f64* also the float64 refinement).  No phase
 * flag = all three.  The phase calls of one batch take the same arguments and
 * run in phase order on streams that order them. */
#define LMI_Q_PHASE_PLAN 0x200
#define LMI_Q_PHASE_SCAN 0x400
#define LMI_Q_PHASE_MERGE 0x800
/* ABI 10 (lmi_bucket_topk_f64g only): the float64 refinement as a phase of
 * its own, after the ranks' k-th distances were exchanged. */
#define LMI_Q_PHASE_REFINE 0x1000

#define LMI_MAX_LAYERS 8
#define LMI_MAX_K 16          /* largest k of one scan pass (and of K3 / the float32 ABI 1 lists) */
#define LMI_MAX_K_PASSES 1024 /* lmi_bucket_topk: k > LMI_MAX_K lists (the wide path, below) */
#define LMI_MAX_K_F64 240     /* lmi_bucket_topk_f64: k + 5 guard entries in <= 256-entry lists */

/* ---- router ----------------------------------------------------------- */
/* A torch nn.Sequential of nn.Linear layers with ReLU between consecutive
 * layers (reference model.py:18-83, class Model; the CLI's default 'MLP' is
 * 96->128->ReLU->C, README/north_star's 'MLP-5' is 96->256->128->C). */
typedef struct lmi_mlp_desc {
    int32_t n_layers;                 /* number of nn.Linear layers, 1..LMI_MAX_LAYERS */
    int32_t dims[LMI_MAX_LAYERS + 1]; /* dims[0]=input width ... dims[n_layers]=n_classes */
    const float* W[LMI_MAX_LAYERS];   /* device, torch layout [out][in] row-major (y = x W^T + b) */
    const float* b[LMI_MAX_LAYERS];   /* device, [out] */
} lmi_mlp_desc;

/* Router inference on nq rows of x (device, [nq][dims[0]] f32, row stride ldx).
 * mode LMI_ROUTER_TOPR — replaces NeuralNetwork.predict_proba
 *   (reference model.py:214-229 = softmax(dim=1) then topk(C)):
 *   classes_out (device, [nq][R] int32) = classes by descending probability,
 *   ties by ascending class index; probs_out (device, [nq][R] f32, nullable) =
 *   the matching softmax probabilities.  1 <= R <= n_classes.
 * mode LMI_ROUTER_ARGMAX — replaces NeuralNetwork.predict (model.py:201-212,
 *   used for object labels at LearnedIndex.py:240): R must be 1,
 *   classes_out[q] = argmax of logits (lowest index on ties); probs_out unused. */
int lmi_router(const float* x, int32_t nq, int32_t ldx, const lmi_mlp_desc* mlp,
               int32_t R, int32_t mode, int32_t* classes_out, float* probs_out,
               void* stream);

/* ---- bucket-sorted corpus (one shard) -------------------------------- */
/* Rows of the search corpus (reference: data_search, clip768 'emb',
 * search.py:79-84) ordered by bucket label, stable in row order, i.e. the
 * order in which DataFrame.groupby('category') visits them
 * (LearnedIndex.py:143-145).  A shard of a G-GPU index holds a contiguous
 * slice of every bucket; `gpos` maps a local row to its global position in
 * the unsharded order (the tie-break key; within a bucket it is monotone in
 * the reference's g.index order).  Inside a bucket the rows may be grouped by
 * sub-cluster as long as the rows of each chunk are in ascending gpos. */
typedef struct lmi_index_desc {
    const void* corpus;        /* device, [n_rows][d_pad] of dtype, zero-padded past d */
    int32_t dtype;             /* LMI_F16 (values fp16-exact) or LMI_F32 */
    int32_t d;                 /* logical vector width (768 for clip768) */
    int32_t d_pad;             /* row stride in elements, multiple of 32 */
    int64_t n_rows;            /* rows held by this shard */
    const float* inv_norm;     /* device [n_rows]: 1/||y|| with sklearn's zero rule */
    const int32_t* gpos;       /* device [n_rows]: global position of each row */
    int32_t n_buckets;         /* C (classes of the router) */
    const int64_t* bucket_off; /* device [C+1]: rows of bucket c are [off[c], off[c+1]) */
    int32_t chunk_rows;        /* rows per scan chunk (work unit along the corpus) */
    const int32_t* chunk_first;/* device [C+1]: prefix of ceil(n_c/chunk_rows) (lmi_plan_chunks) */
    int32_t n_chunks;          /* chunk_first[C] */
    int32_t max_chunks;        /* max_c ceil(n_c/chunk_rows) */
    /* ABI 2: optional (NULL = none) device [n_chunks][d_pad] f32, the unit
     * centroid of each chunk.  When a bucket's rows are laid out by
     * sub-cluster (every chunk one sub-cluster; rows inside a chunk still in
     * ascending gpos), the scan visits each (query, probe)'s nearest chunk
     * first, so its pruning bound starts near the final k-th distance.
     * Results do not depend on it. */
    const float* chunk_centroid;
    /* ABI 6: optional (NULL = none) device [n_rows][d_pad] float64: the rows
     * as the caller gave them when they are float64 (a float64 data_search
     * DataFrame).  The scan still reads `corpus` (the rows rounded to
     * float32); the float64 mode (lmi_bucket_topk_f64*) recomputes its band
     * and fallback distances from these rows, i.e. on the values sklearn sees
     * (utils.py:11, :19).  Results of the float32 mode do not depend on it. */
    const double* corpus64;
    /* ABI 9: optional (NULL = none) device [n_rows][d_pad] float32: the rows
     * as the caller gave them when they are float32 but NOT fp16-exact.
     * `corpus` then holds each row L2-normalised and rounded to fp16 (dtype
     * LMI_F16, inv_norm = 1/||that fp16 row||), and the search is exact in two
     * steps (lmi_bucket_topk, _f64, _f64q, k <= LMI_MAX_K; queries as given,
     * float32, rounded inside the call the same way):
     *   1. an fp16 scan on the rounded rows and queries gives each (query,
     *      probe) an upper bound B of its approximate k-th distance d~_k (the
     *      k-th of a per-bucket sample -- each bucket's first chunk_rows rows
     *      -- for k <= 10, the 15th of sampled chunk lists for k <= 15, the
     *      k-th of a whole scan for k = 16); every row's rounded distance
     *      lies within eps_x of its exact one, eps_x = lmi_split_eps(d)
     *      (1.0e-3 at d = 768), so the exact top-k lies within d~_k + 2 eps_x;
     *   2. a collect scan gathers every row under B + 2 eps_x; of those (they
     *      hold the k smallest d~, hence d~_k), the rows within d~_k + 2 eps_x
     *      get their exact distances in float64 from these rows (or from
     *      corpus64 when set, for the float64 mode) and the query, sorted by
     *      (distance, position) -- rounded to float32 first for the float32
     *      mode -- and the first k kept; a pair with more candidates than the
     *      collect buffer holds is scanned whole in float64.
     * Needs d_pad == 768 (the fp16 scan's width).  ABI 11: k <= 10 takes the
     * phase flags (LMI_Q_PHASE_PLAN: the rounded queries and both scans'
     * plans; SCAN: the sample scan, the bound and the collect scan; MERGE:
     * step 3), so a stream of batches runs one batch's re-score beside the
     * next one's scans; other k, no phase flags.
     * ABI 10: the float32 arithmetic re-scores in the reference's own float32
     * operation order -- sklearn's normalize (numpy einsum row norms, a
     * division) and OpenBLAS sgemm's summation order for the (round, bucket)
     * group's shape (oracle blas32_*: numpy 2.2 / OpenBLAS 0.3.29 SkylakeX,
     * the libraries the reference runs on in the build container) -- so its
     * float32 distances are the reference's bit for bit; shapes whose BLAS
     * path is not restated (a group of one query or one row, groups of at
     * most 3 x 3) keep the exact value rounded to float32 (ABI 11: the
     * whole-shard fallback follows the reference's order too). */
    const float* corpus32;
    /* ABI 10: optional (NULL = this shard's own) device [n_buckets] int64: the
     * rows of every bucket in the whole index (a G-GPU index's shards hold
     * slices): the shape of the reference's per-bucket product. */
    const int64_t* bucket_rows;
    /* ABI 11: optional (NULL = normalised per candidate inside the call)
     * device [n_rows][d_pad] float32: corpus32's rows divided by their
     * float32 norms as sklearn's normalize computes them (numpy einsum row
     * norms, zero rule, IEEE division; lmi_split_normalize fills it).  The
     * normalised row depends on the row alone, so the float32 re-score then
     * runs only the product's summation chains per candidate.  Same float32
     * distances, bit for bit, with or without it. */
    const float* corpus32n;
} lmi_index_desc;

/* Host helper: fills chunk_first_out[C+1] from host bucket offsets and returns
 * max chunks per bucket (>= 0) or a negative LMI_E_* code. */
int32_t lmi_plan_chunks(const int64_t* bucket_off_host, int32_t n_buckets,
                        int32_t chunk_rows, int32_t* chunk_first_out);

/* Bytes of workspace lmi_bucket_topk needs for this shard and batch. */
size_t lmi_scan_workspace_bytes(const lmi_index_desc* idx, int32_t nq, int32_t R,
                                int32_t k, int32_t qmode);

/* Per-(query, probe) exact top-k inside the probed bucket — the build contract
 * K2 of SURVEY.md §8(a) A4.  Replaces, for every probe r < R of every query,
 * utils.py:10-11 pairwise_cosine (sklearn normalize + BLAS GEMM), the full-row
 * argsort at LearnedIndex.py:170-172 and the pandas .loc gathers at :152-153,
 * :168.  Distances are 1 - cos(q, y) in fp32.
 *   q        device [nq][ldq] f32, raw query rows (normalised inside, sklearn rule)
 *   classes  device [nq][R] int32 bucket of probe r (router output)
 *   out_d    device [nq][R][k] f32 ascending, +inf past the bucket's size
 *   out_pos  device [nq][R][k] int32 global row positions, -1 past the end
 *   status   device int32, OR-ed with LMI_STATUS_* bits (caller zeroes it)
 * 1 <= k <= LMI_MAX_K_PASSES.  k > LMI_MAX_K (the reference takes any k on its
 * R == 1 path, search.py:134-140 -> LearnedIndex.py:103-111, and in
 * Baseline.py:14-19) returns the first kw = 15 * ceil(k/15) entries of the
 * (distance, position) order.  On the fp16 scan (fp16 corpus, fp16-exact
 * queries, d = 768): a bound scan (every bucket cut into 2 kw/15 lists, each
 * the top-15 of a sample of its rows: the kw-th smallest of those entries
 * bounds the pair's kw-th distance), a collect scan (every row within the
 * bound) and a sort -- two scans whatever k; buckets of fewer than ~2 kw rows
 * are collected whole, pairs whose candidates overflow take lower-bound passes
 * (ceil(k/15) scans, each keeping the next 15 entries after the previous
 * pass's last), as does every pair off the fp16 scan.  Bitwise the same lists
 * either way (LMI_WIDE_PASSES=1: the passes alone).  Same workspace contract
 * (lmi_scan_workspace_bytes). */
int lmi_bucket_topk(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                    const int32_t* classes, int32_t R, int32_t k, int32_t qmode,
                    float* out_d, int32_t* out_pos, int32_t* status,
                    void* workspace, size_t ws_bytes, void* stream);

/* Merge G per-shard lists of the same rows (K3): in
 * device [G][rows][k] (d f32, pos int32, -1 = empty), out device [rows][k] =
 * the k smallest by (d, pos).  Used after the RCCL all-gather of a G-GPU index.
 * 1 <= k <= LMI_MAX_K_PASSES (ABI 6; k > LMI_MAX_K merges by rank: the wide
 * lists of k > 16 at G > 1, search_single(k) / Baseline(k) on the R == 1 path,
 * LearnedIndex.py:103-111, Baseline.py:14-19).  The same range for
 * lmi_merge_topk_f64 and lmi_merge_topk_packed. */
int lmi_merge_topk(const float* d_in, const int32_t* pos_in, int32_t G, int64_t rows,
                   int32_t k, float* out_d, int32_t* out_pos, void* stream);

/* ---- float64 distances (ABI 4) ---------------------------------------- */
/* The reference computes 1 - cosine_similarity in float32 only when BOTH
 * operands are float32; otherwise — the real data: clip768 'emb' is float16 —
 * sklearn promotes to float64 (utils.py:11, :19; check_pairwise_arrays) and
 * the threshold test (utils.py:23) and the merges (LearnedIndex.py:86-97) see
 * float64 values.  lmi_bucket_topk_f64 returns those float64 lists:
 *   - the fp32 scan keeps 15 entries per (query, probe) for k <= 10 (round 5,
 *     fp16 scan: the union of 10-entry lane lists with the filter widened by
 *     2*eps, plus a bound below which no unlisted row lies; otherwise the
 *     top-KL, KL >= k + 5);
 *   - every list entry within 2*eps of the fp32 k-th distance is recomputed
 *     in float64 from the stored row (sklearn normalize + dot; exact fp16
 *     inputs; idx->corpus64 when set), sorted by (d64, position); when no
 *     unlisted row can lie in that band the result is the exact float64
 *     top-k whenever eps bounds the fp32 error |d32 - d64| for every row: the
 *     host passes a bound derived from d_pad and the MFMA accumulation depth
 *     (li.index.refine_eps; 2^-16 for the fp16 path at d 768);
 *   - other pairs are recomputed in float64 over their whole bucket shard
 *     (exact, rare: ties or near-ties of many objects).
 * With LMI_Q_SEED_ROUND0 the lists of rounds r >= 1 are exact below round 0's
 * threshold only (what the thresholded replay reads; k = k_round lists).
 * Same arguments and layout as lmi_bucket_topk; out_d is float64 [nq][R][k]
 * (+inf past the bucket's size), out_pos global positions (-1 past it).
 * 1 <= k <= LMI_MAX_K_F64, d <= 1024; k > 10 lists come from lower-bound
 * passes (as lmi_bucket_topk's) of at least k + 5 entries. */
#define LMI_REFINE_EPS 1.52587890625e-05 /* 2^-16 */
size_t lmi_scan_f64_workspace_bytes(const lmi_index_desc* idx, int32_t nq, int32_t R,
                                    int32_t k, int32_t qmode);
int lmi_bucket_topk_f64(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                        const int32_t* classes, int32_t R, int32_t k, int32_t qmode, double eps,
                        double* out_d, int32_t* out_pos, int32_t* status, void* workspace,
                        size_t ws_bytes, void* stream);
/* ABI 6: as lmi_bucket_topk_f64, with float64 query rows q64 (device,
 * [nq][ldq64], nullable) for the float64 recomputation: the reference's
 * arithmetic on float64 queries (utils.py:11, :19).  q (float32) is what the
 * scan reads -- q64 rounded to float32.  Together with idx->corpus64 this is
 * the float64-input path; eps must then also cover the float32 rounding of
 * the inputs (8u more; li.index.refine_eps). */
int lmi_bucket_topk_f64q(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                         const double* q64, int32_t ldq64, const int32_t* classes, int32_t R,
                         int32_t k, int32_t qmode, double eps, double* out_d, int32_t* out_pos,
                         int32_t* status, void* workspace, size_t ws_bytes, void* stream);
/* ABI 10: lmi_bucket_topk_f64q for a stripe of a G-rank index, with the band
 * decided over every rank's lists (replaces, for the striped
 * float64 search, the per-rank refinement of the same reference lines:
 * utils.py:10-11 in float64 and LearnedIndex.py:170-172).  The float64 top-k
 * of a pair lies in d32 <= T + 2 eps with T the k-th smallest d32 over ALL
 * ranks' rows; T is never above a rank's own k-th, so a rank that knows T
 * refines only its own rows of that merged band (about 1/G of them) instead
 * of the band of its own list.  Phases:
 *   PLAN, SCAN   as lmi_bucket_topk_f64q;
 *   MERGE        the chunk merge, then kth_send (device [nq*R][k] f32) = each
 *                pair's k smallest d32 of this rank (+inf past its list);
 *   (the caller all-gathers kth_send: block g of G at kth_all + g * kth_stride)
 *   REFINE       per pair T from the G blocks, then the refinement of this
 *                rank's listed rows with d32 <= T + 2 eps (and the whole-shard
 *                fallback of a pair whose band may hold unlisted rows): out_d
 *                / out_pos hold this rank's part of the pair's float64 top-k,
 *                ascending by (d64, position), (+inf, -1) past it.
 * No phase flag = all four on one rank (kth_all == kth_send, G == 1).  K3
 * (lmi_merge_topk_f64 / _packed) over the ranks' outputs then gives exactly
 * the one-GPU float64 lists.  Needs the band lists (k <= 10 on the fp16
 * scan): lmi_f64_global_band returns 1 when a call of these arguments has
 * them, 0 otherwise (then lmi_bucket_topk_f64q per rank). */
int lmi_f64_global_band(const lmi_index_desc* idx, int32_t nq, int32_t R, int32_t k, int32_t qmode);
int lmi_bucket_topk_f64g(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                         const double* q64, int32_t ldq64, const int32_t* classes, int32_t R,
                         int32_t k, int32_t qmode, double eps, float* kth_send,
                         const float* kth_all, int32_t G, int64_t kth_stride, double* out_d,
                         int32_t* out_pos, int32_t* status, void* workspace, size_t ws_bytes,
                         void* stream);
/* ABI 9: the split mode's bound eps_x on |d~ - d| (lmi_index_desc.corpus32),
 * for rows of d_pad elements; a host function (≈ 9.9e-4 at d_pad = 768).  In the
 * split mode the eps argument of lmi_bucket_topk_f64* is ignored (this one
 * is used), and so is the fp16 / fp32 class of qmode (the queries are
 * normalised and rounded inside the call). */
double lmi_split_eps(int32_t d_pad);
/* ABI 11: lmi_index_desc.corpus32n from corpus32 (device [n][d_pad] float32
 * in and out, out's padding zeroed; a wave per row, index build, not the hot
 * path).  Replaces, per row, the normalize(Y) of the reference's
 * cosine_distances (utils.py:10-11; sklearn normalize: numpy einsum norms). */
int lmi_split_normalize(const float* rows, int64_t n, int32_t d, int32_t d_pad, float* out,
                        void* stream);
/* Diagnostic (synchronises `stream`): how many (query, probe) pairs of the
 * last lmi_bucket_topk_f64 call on this workspace took the whole-bucket path
 * (the split mode: also of lmi_bucket_topk, whose workspace has the same layout). */
int lmi_refine_fallback_count(const void* workspace, const lmi_index_desc* idx, int32_t nq,
                              int32_t R, int32_t k, int32_t qmode, int32_t* count_out,
                              void* stream);
/* ABI 13, diagnostic (synchronises `stream`): the split mode (k <= 10) collects
 * the rest of every bucket whose sample is at most a quarter of it and takes the
 * sample's rows from the sample scan's own list; how many pairs of the last call
 * on this workspace had a band reaching that list's k-th and were scored over
 * their sample rows and candidates instead (x_fallback_kernel). */
int lmi_split_sample_fallback_count(const void* workspace, const lmi_index_desc* idx, int32_t nq,
                                    int32_t R, int32_t k, int32_t* count_out, void* stream);
/* K3 on float64 lists: order (d64, pos). */
int lmi_merge_topk_f64(const double* d_in, const int32_t* pos_in, int32_t G, int64_t rows,
                       int32_t k, double* out_d, int32_t* out_pos, void* stream);

/* ---- K3 over the all-gathered buffer, in place (ABI 5) ------------------ */
/* A G-GPU search all-gathers one packed int32 buffer per rank instead of
 * separate lists (li/dist.py): rank g's words start at gathered + g *
 * rank_words and hold [distances: rows*k f32, or rows*k f64 as 2 words each]
 * [positions: rows*k int32][the rank's lmi_bucket_topk status word], padded
 * to rank_words (even, >= lmi_packed_rank_words; the buffer 8-byte aligned).
 * lmi_merge_topk_packed merges the G lists as lmi_merge_topk(_f64) does and
 * writes the OR of the G status words to out_status (device int32), so every
 * rank sees every rank's bits; out_d is f32 or f64 [rows][k] by dist_f64.
 * One launch replaces the unpacking copies and the per-rank status ORs. */
int64_t lmi_packed_rank_words(int64_t rows, int32_t k, int32_t dist_f64);
int lmi_merge_topk_packed(const int32_t* gathered, int32_t G, int64_t rank_words, int64_t rows,
                          int32_t k, int32_t dist_f64, void* out_d, int32_t* out_pos,
                          int32_t* out_status, void* stream);

/* ---- host replay of the reference's multi-round merge ----------------- */
/* Reproduces LearnedIndex.search (LearnedIndex.py:22-101) and search_single
 * (:103-195) — thresholds, per-category groups, the <k padding quirk
 * (:174-193), the 10000 fillers (utils.py:35-42) and the stable merge
 * (:86-97) — from the per-(query, probe) lists of lmi_bucket_topk
 * (SURVEY.md §8(a) A5).  All pointers are host memory.
 *   classes   [nq][R] int32;  lists_d / lists_pos [nq][R][k_list] (from device)
 *   k_round   length of one round's result: search_single's k.  search()
 *             never passes its k down (LearnedIndex.py:75-81), so it is 10
 *             there; search.py:134-140 passes k for the R == 1 path.
 *   k_final   search()'s k: columns kept by every merge (LearnedIndex.py:91)
 *   bucket_size [C] int64 objects per category (0 = category absent from
 *               data_navigation, so groupby never visits it)
 *   pos_to_id [n_total] int64  DataFrame index label of each global position
 *   use_threshold  0/1 as the reference's argument (search.py:127 passes True)
 *   thr_round0 [nq] float64 or NULL: search_single's threshold_dist argument
 *             (LearnedIndex.py:110, :149-163) for a direct R == 1 call
 *   dists_out [nq][w] float64, anns_out [nq][w] uint32 with w = k_round if
 *             R == 1 else k_final (*w_out receives w).
 * Returns LMI_E_INVALID where the reference's own assert (LearnedIndex.py:99)
 * would fail (k_final larger than the merged width). */
int lmi_replay(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
               const float* lists_d, const int32_t* lists_pos, int32_t k_round,
               int32_t k_final, const int64_t* bucket_size, int32_t n_buckets,
               const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
               const double* thr_round0, double* dists_out, uint32_t* anns_out,
               int32_t* w_out);
/* ABI 4: the same replay of float64 lists (lmi_bucket_topk_f64). */
int lmi_replay_f64(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                   const double* lists_d, const int32_t* lists_pos, int32_t k_round,
                   int32_t k_final, const int64_t* bucket_size, int32_t n_buckets,
                   const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
                   const double* thr_round0, double* dists_out, uint32_t* anns_out,
                   int32_t* w_out);

/* The same replay on the device (ABI 2): identical results to lmi_replay
 * (checked bit for bit by tests/test_gpu_replay.py), no host round trip.
 * classes, lists_d, lists_pos, bucket_size, pos_to_id, thr_round0 (nullable),
 * dists_out, anns_out are device pointers; status (device int32, caller
 * zeroes it) is OR-ed with nonzero bits on an internal inconsistency (1, 2: a
 * list shorter than its bucket; 4: a position out of range; 8: a round's group
 * never completed in the one-launch replay, which then drains instead of
 * waiting forever).  k_list >= k_round,
 * k_round <= 32, k_final <= 64.  Asynchronous on `stream`; workspace of
 * lmi_replay_device_workspace_bytes bytes. */
size_t lmi_replay_device_workspace_bytes(int32_t nq, int32_t R, int32_t k_list, int32_t k_round,
                                         int32_t k_final, int32_t n_buckets);
int lmi_replay_device(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                      const float* lists_d, const int32_t* lists_pos, int32_t k_round,
                      int32_t k_final, const int64_t* bucket_size, int32_t n_buckets,
                      const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
                      const double* thr_round0, double* dists_out, uint32_t* anns_out,
                      int32_t* status, void* workspace, size_t ws_bytes, void* stream);
/* ABI 4: the same device replay of float64 lists (lmi_bucket_topk_f64). */
int lmi_replay_device_f64(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                          const double* lists_d, const int32_t* lists_pos, int32_t k_round,
                          int32_t k_final, const int64_t* bucket_size, int32_t n_buckets,
                          const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
                          const double* thr_round0, double* dists_out, uint32_t* anns_out,
                          int32_t* status, void* workspace, size_t ws_bytes, void* stream);

/* ABI 9: the device replay in two phases, so that a stream of batches runs the
 * part that depends on the classes only beside the scan:
 *   LMI_REPLAY_PHASE_GROUPS  every round's groups (queries by category, in
 *                            ascending q) and round 0's prologue; zeroes
 *                            *status (the phased call owns the word);
 *   LMI_REPLAY_PHASE_ROUNDS  the rounds and the answer (lists needed).
 * Both = lmi_replay_device / _f64 (the caller zeroes *status then).  Calls of
 * one replay take the same arguments and workspace, GROUPS first (lists_d /
 * lists_pos / pos_to_id / dists_out / anns_out may be NULL in a GROUPS call);
 * lists_f64 selects float64 lists. */
#define LMI_REPLAY_PHASE_GROUPS 1
#define LMI_REPLAY_PHASE_ROUNDS 2
int lmi_replay_device_phase(int32_t phases, int32_t lists_f64, const int32_t* classes, int32_t nq,
                            int32_t R, int32_t k_list, const void* lists_d, const int32_t* lists_pos,
                            int32_t k_round, int32_t k_final, const int64_t* bucket_size,
                            int32_t n_buckets, const int64_t* pos_to_id, int64_t n_total,
                            int32_t use_threshold, const double* thr_round0, double* dists_out,
                            uint32_t* anns_out, int32_t* status, void* workspace, size_t ws_bytes,
                            void* stream);

/* ---- k-means for the index build (ABI 3) -------------- */
/* Replaces faiss.Kmeans(d, k, seed=2023).train(X) and
 * kmeans.index.search(X, 1) (LearnedIndex.py:242-282); the Lloyd loop, the
 * training subsample and the empty-cluster split run on the host
 * (li/kmeans.py).  All pointers are device memory; asynchronous on `stream`.
 *
 * lmi_kmeans_assign: labels_out[i] = argmin_j Σ_e (x[i][e] - cent[j][e])²
 *   (squared L2 in fp32, e ascending, no FMA contraction; ties -> lower j);
 *   dist_out (nullable) receives the minimum.  x [n][d], cent [k][d] f32,
 *   1 <= d <= LMI_KMEANS_MAX_D.
 * lmi_kmeans_update: cent_out[c] = mean of the points labelled c (fp64 sums
 *   in a fixed order, rounded once), counts_out[c] = their number; rows of
 *   empty clusters are left untouched.  A label outside [0, k) ORs 1 into
 *   *status (device int32) and is skipped.  Deterministic. */
#define LMI_KMEANS_MAX_D 128
int lmi_kmeans_assign(const float* x, int64_t n, int32_t d, const float* cent, int32_t k,
                      int32_t* labels_out, float* dist_out, void* stream);
size_t lmi_kmeans_workspace_bytes(int64_t n, int32_t d, int32_t k);
int lmi_kmeans_update(const float* x, int64_t n, int32_t d, const int32_t* labels, int32_t k,
                      float* cent_out, int64_t* counts_out, int32_t* status, void* workspace,
                      size_t ws_bytes, void* stream);

/* ---- kernel timing (measurement only) -------------------------------------- */
/* While enabled, lmi_bucket_topk records a HIP event pair on its stream around
 * its scan kernel (the roofline kernel).  lmi_timing_read waits for the pairs
 * recorded so far, writes up to max_n durations (ms) and clears the record;
 * it returns the number written or a negative LMI_E_* code.  Not for use
 * under graph capture (events recorded into a hipGraph cannot be timed). */
int lmi_timing_enable(int32_t on);
int32_t lmi_timing_read(float* ms_out, int32_t max_n);

/* ---- host utilities (ABI 6) ---------------------------------------------- */
/* 64-bit content hash of n_bytes of HOST memory on `threads` OpenMP threads
 * (<= 0: all), independent of the thread count; not cryptographic.  Keys the
 * drop-in's HBM index cache (li.LearnedIndex): a cached bucket-sorted corpus
 * is served only for byte-identical data_search / labels / ids, where the
 * reference re-gathers every bucket from the DataFrame on every call
 * (LearnedIndex.py:152-153, :168). */
uint64_t lmi_host_hash64(const void* data, uint64_t n_bytes, int32_t threads);

/* ---- staging a host query batch (ABI 8) ------------------------------------ */
/* The reference's queries are host arrays (search.py:49, :85-87); the batch
 * stream (li.stream.StreamedSearch.stage) writes each new batch into pinned
 * staging memory with these, on `threads` OpenMP threads (<= 0: all).
 * lmi_host_stage_f16: n float32 values -> fp16 (IEEE binary16, round to
 * nearest even) in dst; returns 1 when every value round-trips exactly
 * (numpy's array_equal(src.astype(f16).astype(f32), src): the fp16 MFMA
 * scan's precondition), 0 when some value does not (dst then holds rounded
 * values that no fp16-exact path may use), -LMI_E_INVALID on null pointers.
 * lmi_host_copy: a memcpy of n_bytes cut over the threads. */
int32_t lmi_host_stage_f16(const float* src, uint64_t n, uint16_t* dst, int32_t threads);
int lmi_host_copy(void* dst, const void* src, uint64_t n_bytes, int32_t threads);

/* ---- misc --------------------------------------------------------------- */
const char* lmi_last_error(void);
int32_t lmi_abi_version(void);
/* The LMI_* environment switches (diagnostic variants and tuning knobs; results
 * never depend on them) are read once, at the first launch.  Diagnostics that
 * change them inside one process call this to re-read them; not for use while
 * another thread launches.  The scan's workspace layout depends on the tail
 * split knobs (LMI_SCAN_SPLIT, LMI_SCAN_SPLIT_PARTS, LMI_SCAN_NO_PREF): after a
 * reload, size the workspaces again (lmi_scan_workspace_bytes /
 * lmi_scan_f64_workspace_bytes) -- a workspace sized under the old knobs may
 * be refused with LMI_E_WORKSPACE, never overrun. */
int lmi_config_reload(void);
/* The persistent scan's grid (ABI 12): the number of workgroups (one per CU)
 * the scan kernels of lmi_bucket_topk[_f64*] launch from this thread, so a
 * caller can leave CUs to work that runs beside the scan on other streams
 * (li.stream.StreamedSearch: the finish chain of the previous batch).  0: one
 * per CU (or LMI_SCAN_WGS).  Thread-local, read at launch (a captured graph
 * keeps the grid it was captured with); results never depend on it.  Returns
 * the previous setting. */
int32_t lmi_scan_set_workgroups(int32_t wgs);

#ifdef __cplusplus
}
#endif
#endif /* LMI_HIP_H */
