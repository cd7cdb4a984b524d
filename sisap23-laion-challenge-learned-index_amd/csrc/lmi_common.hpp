// Shared helpers of liblmi_hip.so: error plumbing for the C-ABI and the
// (distance, position) key used by every top-k list on the device.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/lmi_hip.h"
#include "lmi_env.hpp"

namespace lmi {

// ---- error plumbing (no exception crosses the C-ABI) -------------------
void set_error(const char* fmt, ...);

#define LMI_CHECK_ARG(cond, ...)              \
    do {                                      \
        if (!(cond)) {                        \
            ::lmi::set_error(__VA_ARGS__);    \
            return LMI_E_INVALID;             \
        }                                     \
    } while (0)

#define LMI_HIP_TRY(expr)                                                        \
    do {                                                                         \
        hipError_t e_ = (expr);                                                  \
        if (e_ != hipSuccess) {                                                  \
            ::lmi::set_error("%s failed: %s", #expr, hipGetErrorString(e_));     \
            return LMI_E_HIP;                                                    \
        }                                                                        \
    } while (0)

#define LMI_TRY(expr)                                                            \
    do {                                                                         \
        const int rc_ = (expr);                                                  \
        if (rc_ != LMI_OK) return rc_;                                           \
    } while (0)

#define LMI_LAUNCH_CHECK(name)                                                   \
    do {                                                                         \
        hipError_t e_ = hipGetLastError();                                       \
        if (e_ != hipSuccess) {                                                  \
            ::lmi::set_error("launch of %s failed: %s", name, hipGetErrorString(e_)); \
            return LMI_E_HIP;                                                    \
        }                                                                        \
    } while (0)

// ---- keys ------------------------------------------------------------------
// A list entry is one u64: high word = order-preserving image of the fp32
// distance, low word = row position.  u64 "<" is then the reference's
// (distance, position) order (LearnedIndex.py:170 argsort of a row whose
// columns are in g.index order; :91 stable merge), and the all-ones key is
// "empty" (sorts after every finite and infinite distance).
constexpr uint64_t kEmptyKey = ~0ull;

__host__ __device__ inline uint32_t f2ord(float f) {
    uint32_t b;
    __builtin_memcpy(&b, &f, 4);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__host__ __device__ inline float ord2f(uint32_t o) {
    uint32_t b = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    float f;
    __builtin_memcpy(&f, &b, 4);
    return f;
}

__host__ __device__ inline uint64_t make_key(float d, uint32_t pos) {
    return (static_cast<uint64_t>(f2ord(d)) << 32) | pos;
}

// Largest distance a candidate may have and still beat `thr` (conservative:
// ord(d) <= hi(thr) is necessary for key < thr).
__device__ inline float key_dist_bound(uint64_t thr) {
    uint32_t hi = static_cast<uint32_t>(thr >> 32);
    if (hi == 0xffffffffu) return __builtin_inff();
    if (hi == 0u) return -__builtin_inff();
    return ord2f(hi);
}

// Insert `x` into the ascending register list L[0..KL), dropping the largest.
// Caller guarantees x < L[KL-1].  Fully unrolled: every index is a constant,
// so the list stays in VGPRs (runtime-indexed arrays go to scratch).
template <int KL>
__device__ inline void list_insert(uint64_t (&L)[KL], uint64_t x) {
#pragma unroll
    for (int i = KL - 1; i > 0; --i) {
        const uint64_t prev = L[i - 1];
        const uint64_t cur = L[i];
        L[i] = (x < prev) ? prev : ((x < cur) ? x : cur);
    }
    L[0] = (x < L[0]) ? x : L[0];
}

// list_insert that carries a payload word beside every key (the local row of
// an entry whose key holds its global position)
template <int KL>
__device__ inline void list_insert_pair(uint64_t (&L)[KL], int32_t (&W)[KL], uint64_t x,
                                        int32_t w) {
#pragma unroll
    for (int i = KL - 1; i > 0; --i) {
        const bool take_prev = x < L[i - 1];
        const bool take_x = !take_prev && x < L[i];
        W[i] = take_prev ? W[i - 1] : (take_x ? w : W[i]);
        L[i] = take_prev ? L[i - 1] : (take_x ? x : L[i]);
    }
    if (x < L[0]) {
        L[0] = x;
        W[0] = w;
    }
}

template <int KL>
__device__ inline void list_clear(uint64_t (&L)[KL]) {
#pragma unroll
    for (int i = 0; i < KL; ++i) L[i] = kEmptyKey;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }


// ---- internal entry points shared between translation units -------------
// phases of bucket_topk_impl (LMI_Q_PHASE_* of the ABI, shifted to bits 0..2)
constexpr int kPhasePlan = 1, kPhaseScan = 2, kPhaseMerge = 4, kPhaseAll = 7;
// LMI_Q_PHASE_* bits of a qmode -> kPhase* (none set = all); strips them from qmode
inline int take_phases(int32_t& qmode) {
    const int p = (qmode >> 9) & 7;
    qmode &= ~(7 << 9);
    return p ? p : kPhaseAll;
}
// K2 up to the merged per-pair lists (lmi_scan.hip): lmi_bucket_topk with an
// optional third output, the shard-local row of every entry (-1 = empty).
// lo_g (nullable, device [nq*R]): keep only objects after the (distance,
// global position) key of their pair (the passes of k > 16); ldo: entries per
// pair in the outputs (default k); prefill: write (+inf, -1) over all R*ldo
// entries first (the first pass).  seed_r0: LMI_Q_SEED_ROUND0 (pairs r >= 1
// start from the bound of pair (q, 0), + seed_margin in distance).
// out_bound (nullable, [nq*R] float; k <= 15 on scan v3, kl = 15): the float64
// mode's band lists -- the scan's filter widened by seed_margin (2 eps), every
// pair's first 15 entries, and out_bound[pair] a distance such that each row
// of the shard the list does not hold failed the widened filter or has
// d32 >= it (chunk_merge_band_kernel); kth_out (nullable, with out_bound):
// each pair's first kth_k list distances also written to kth_out[pair * kth_k]
// (the float64 global band's kth_send, ABI 10).
// The scans of the wide path (k > 16, bucket_topk_wide): mode 1 writes every
// (pair, chunk part) list as that part's own top-15 (no global bound); mode 2
// collects every row within the pair's bound bound_ord[pair id] (a distance
// ordinal; 0 = none) into cand[grouped pair * cap + i] (ccount: slots taken).
struct WideScan {
    int mode;
    const uint32_t* bound_ord;
    uint64_t* cand;
    uint32_t* ccount;
    int32_t cap;
    uint32_t* bins;  // mode 1: [P][nbins], all ones at the start (Scan2Args::bins)
    int32_t nbins;
    const int32_t* sub_rows;  // mode 1: Scan2Args::sub_rows / sub_take
    const int32_t* sub_take;
    // mode 2: a pair whose (odd) bucket b has rows skipped in front of it
    // (bucket b - 1 of the descriptor not empty: the split mode's sample,
    // x_collect_desc) starts with its app_k (distance, row) entries app_d /
    // app_row [pair id][app_k] as candidates (-1 rows skipped); null: none
    const float* app_d;
    const int32_t* app_row;
    int32_t app_k;
};
int bucket_topk_impl(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                     const int32_t* classes, int32_t R, int32_t k, int32_t qmode, float* out_d,
                     int32_t* out_pos, int32_t* out_row, int32_t* status, void* workspace,
                     size_t ws_bytes, hipStream_t s, const unsigned long long* lo_g = nullptr,
                     int32_t ldo = 0, bool prefill = true, bool seed_r0 = false,
                     float seed_margin = 0.0f, int phases = kPhaseAll,
                     const WideScan* wide = nullptr, float* out_bound = nullptr,
                     float* kth_out = nullptr, int32_t kth_k = 0);
// scan v3 serves this index and query class (the float64 mode's band lists)
bool band_capable(const lmi_index_desc* idx, int qmode);
size_t scan_workspace_bytes(const lmi_index_desc* idx, int32_t nq, int32_t R, int32_t k,
                            int32_t qmode, bool lo = false);
// k > LMI_MAX_K: passes_of() passes of kp-entry lists; bucket_topk_passes fills
// [nq*R][ldo] lists (ldo >= passes * kp) with (d32, global position[, local row]).
int passes_of(const lmi_index_desc* idx, int qmode, int k, int* kp_out);
size_t passes_ws_bytes(const lmi_index_desc* idx, int nq, int R, int k, int qmode);
int bucket_topk_passes(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                       const int32_t* classes, int32_t R, int32_t k, int32_t qmode, float* out_d,
                       int32_t* out_pos, int32_t* out_row, int32_t ldo, int32_t* status,
                       void* workspace, size_t ws_bytes, hipStream_t s);
// k > LMI_MAX_K, the same lists as bucket_topk_passes from two scans (scan v3):
// chunk lists -> per-pair bound (the kw-th smallest of the pair's chunk-list
// distances, kw = passes * kp) -> collect the rows within it -> sort; pairs
// without a bound (too few chunk-list entries) or whose candidates overflow
// go through bucket_topk_passes restricted to them.  Off scan v3 (or under
// LMI_WIDE_PASSES) it is bucket_topk_passes.
size_t wide_ws_bytes(const lmi_index_desc* idx, int nq, int R, int k, int qmode, int ldo);
int bucket_topk_wide(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                     const int32_t* classes, int32_t R, int32_t k, int32_t qmode, float* out_d,
                     int32_t* out_pos, int32_t* out_row, int32_t ldo, int32_t* status,
                     void* workspace, size_t ws_bytes, hipStream_t s);
// The split mode's exact step (lmi_refine.hip; ABI 9, idx->corpus32): per
// grouped pair of the collect scan, the exact distances of its candidates,
// sorted, the first k; overflowed pairs scanned whole.
struct XArgs {
    const float* rows32;   // [n_rows][d_pad] the caller's float32 rows
    const double* rows64;  // [n_rows][d_pad] float64 rows (idx->corpus64) or null
    int32_t d, d_pad;
    const int32_t* gpos;
    const int64_t* bucket_off;
    int64_t n_rows;
    const float* q;        // [nq][ldq] float32 queries
    int32_t ldq;
    const double* q64;     // float64 queries or null
    int32_t ldq64;
    const int32_t* classes;
    int32_t nq, R, k;
    const int32_t* pair_q;       // grouped pair -> pair id (the collect scan's plan)
    const int32_t* pair_bucket;  // grouped pair -> bucket (-1: none)
    const uint64_t* cand;        // [grouped pair][cap] (ord(d~) << 32 | row)
    const uint32_t* ccount;
    int32_t cap;
    void* out_d;                 // [nq*R][k] float (out_f64 = 0) or double
    int32_t out_f64;
    int32_t* out_pos;
    int32_t* failed;
    int32_t* n_failed;
    int32_t* status;
    // > 0: the candidates are every row under a sampled bound + two_eps; only
    // those within the k-th smallest d~ + two_eps are re-scored
    double two_eps;
    const int32_t* fix;  // [nq*R] pairs without a sampled bound (whole shard), or null
    // ABI 10, the float32 output only: the reference's float32 operation order
    // (oracle blas32_*; lmi_index_desc.corpus32): qn32 [nq][d_pad] the queries
    // normalised as sklearn does in float32 (null: the exact value rounded),
    // grp [R][C] queries of each (round, bucket) group, nrows_c [C] rows of
    // each bucket in the whole index (null: this shard's)
    const float* qn32;
    const int32_t* grp;
    const int64_t* nrows_c;
    int32_t C;
    // (the small kernel's corner block: tailq[pair] = the query is among the
    // last M mod 4 of its group; goff [C+1] the buckets' global offsets)
    const uint8_t* tailq;
    const int64_t* goff;
    const int32_t* plan_counts;  // [C] pairs per bucket (the collect scan's plan)
    // ABI 11: rows32 normalised as sklearn does in float32 (idx->corpus32n) or
    // null (then normalised per candidate)
    const float* rows32n;
    // the grouped pairs x_select_wave_kernel leaves to x_select_kernel (more
    // candidates, overflowed, unbounded), appended by the wave kernel, and
    // their count (null: x_select_kernel walks every grouped pair)
    int32_t* wgl;
    int32_t* n_wgl;
    // the collect scan skipped each split bucket's sample rows (x_collect_desc):
    // soff [2C+1] (bucket c's sample rows [soff[2c], soff[2c+1]), empty where the
    // bucket was collected whole) and skth [nq*R][k] the sample's own lists (the
    // pair's k-th at k - 1); a pair whose band reaches its sample's k-th goes to
    // sfailed (grouped pair ids, count n_sfailed) and x_fallback_kernel scores
    // its sample rows and its candidates exactly.  null: none skipped.  plan_cm:
    // plan_counts has plan_cm entries per bucket, the pairs of bucket c at
    // plan_cm c + plan_cm - 1
    const int64_t* soff;
    const float* skth;
    int32_t* sfailed;
    int32_t* n_sfailed;
    double* spd;     // the sliced sfailed pairs' slice lists (x_fallback_slice_kernel)
    int32_t* spg;
    int32_t plan_cm;
};
// the sliced sample fallback (x_fallback_slice_kernel): the first
// kXSlicedPairs sfailed pairs, kXSlices slices each (XArgs::spd / spg hold
// kXSlicedPairs x kXSlices x k entries)
constexpr int kXSlices = 32;
constexpr int kXSlicedPairs = 256;
int launch_x_refine(const XArgs& a, int64_t P, hipStream_t s);
double split_eps(int d_pad);
size_t x_ws_bytes(const lmi_index_desc* idx, int nq, int R, int k);
size_t x_nfailed_offset(const lmi_index_desc* idx, int nq, int R, int k);
int bucket_topk_x(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq, const double* q64,
                  int32_t ldq64, const int32_t* classes, int32_t R, int32_t k, void* out_d, int out_f64,
                  int32_t* out_pos, int32_t* status, void* workspace, size_t ws_bytes, hipStream_t s,
                  int phases = kPhaseAll);

// n_words 32-bit words of `value` from p (4-byte aligned) on stream s, by a
// kernel (lmi_merge.hip): workspace initialisation stays a kernel node when a
// caller captures the launch sequence in a HIP graph (no memset nodes).
int fill_u32(void* p, uint32_t value, size_t n_words, hipStream_t s);

}  // namespace lmi
