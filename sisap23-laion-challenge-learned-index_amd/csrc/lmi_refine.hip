// K2 in float64 — the reference's distance arithmetic on fp16 data (gfx950).
//
// sklearn's cosine_similarity runs in float32 only when both operands are
// float32; the real clip768 'emb' is float16, so the reference computes
// d = 1 - <x/|x|, y/|y|> in float64 (utils.py:11, :19 via
// check_pairwise_arrays/_return_float_dtype) and thresholds and merges float64
// values (utils.py:23, LearnedIndex.py:86-97).  The fp32 scan (lmi_scan.hip)
// cannot order two objects whose float64 distances differ by less than its
// rounding, so for that case K2 runs in two steps:
//
//   1. the fp32 MFMA scan keeps per (query, probe) the top-KL (KL > k) by the
//      fp32 distance d32 (bucket_topk_impl, with local rows);
//   2. refine_kernel, one wave per (query, probe): with eps >= |d32 - d64|
//      for every row, every object of the float64 top-k has
//      d32 <= d32[k-1] + 2 eps.  If fewer than KL list entries lie in that
//      band, the list holds all of them (a row outside the list has
//      d32 >= d32[KL-1]); their float64 distances are recomputed from the
//      stored rows (exact fp16 values), sorted by (d64, global position) and
//      the first k written.  Otherwise the pair is queued for
//   3. fallback_kernel, one workgroup per queued pair: float64 distances of
//      every row of its bucket shard, top-k by (d64, position).
//
// The float64 arithmetic follows sklearn.normalize + GEMM: |q| = sqrt(sum q^2)
// with the `norm < 10 eps -> 1` rule, q^ = q/|q|, d = 1 - (sum q^_e y_e)/|y|.
// It differs from the reference's BLAS dgemm only in summation order (a few
// ulp of 1.0), so ids agree except where the reference's own float64 values
// tie to that level.
#include "lmi_common.hpp"

#include <algorithm>
#include <mutex>

namespace lmi {
namespace {

constexpr int kRefT = 256;     // refine: 4 waves, one pair each
constexpr int kFbT = 1024;     // fallback: 16 waves on one pair
constexpr int kFbRows = 4;     // rows per wave in flight (fallback)
constexpr double kEps64 = 2.220446049250313e-16;

struct RefineArgs {
    const void* corpus;
    int32_t dtype;  // LMI_F16 / LMI_F32
    int32_t d, d_pad;
    const int32_t* gpos;
    const int64_t* bucket_off;
    int64_t n_rows;
    const float* q;
    int32_t ldq;
    const double* corpus64;  // float64 rows (idx->corpus64) or null
    const double* q64;       // float64 queries or null
    int32_t ldq64;
    const int32_t* classes;
    int32_t nq, R, kl, k;
    double eps;
    const float* ld;       // [nq][R][kl] d32 ascending
    const int32_t* lrow;   // [nq][R][kl] local rows (-1 empty)
    const int32_t* lpos;   // [nq][R][kl] global positions
    const float* lbound;   // [nq*R] band lists: bound of the unlisted rows (null: plain lists)
    int32_t seeded;        // LMI_Q_SEED_ROUND0 (band lists: rounds r >= 1 need rows under round 0's bound only)
    double* out_d;         // [nq][R][k]
    int32_t* out_pos;
    int32_t* failed;       // [nq*R] queued pairs
    int32_t* n_failed;
    int32_t* status;
    double* pd;            // sliced fallback partial lists [kFbSlicedPairs][kFbSlices][k] (null: off)
    int32_t* pg;
    // ABI 10 (band lists, a stripe of a G-rank index): the k smallest d32 of
    // every rank's band list of every pair, gathered: block g at kth_all +
    // g * kth_stride, [nq*R][k] ascending (+inf past the list); the band is
    // then decided by the pair's k-th over all ranks (null: its own list's)
    const float* kth_all;
    int32_t kth_G;
    int64_t kth_stride;
    const float* kth_g;  // [nq*R] that k-th per pair (band_kth_kernel), read by refine_kernel
};

// The k-th smallest of the G ascending lists of k values of every pair (the
// multiset union: equal values on different lists each count; +inf when the
// lists hold fewer than k finite values), before the refine: segments of W =
// the power of two >= G lanes, 64 / W pairs a wave, lane g of a segment
// holding list g in registers; k steps of a segment minimum, the winning lane
// (lowest on ties) shifting its list.  (In the refine itself, one wave per
// pair ran these k steps once or twice -- the seeded rounds read pair (q, 0)'s
// too -- beside the list and the query: a per-pair fixed cost of the refine
// at G = 8, where most pairs have no band row on a stripe.)
__global__ __launch_bounds__(256) void band_kth_kernel(const float* __restrict__ kth_all, int32_t G,
                                                       int64_t stride, int64_t P, int32_t k, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    int W = 1;
    while (W < G) W <<= 1;
    const int per = 64 / W, seg = lane / W, g = lane - seg * W;
    const int64_t p = ((int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * per + seg;
    const bool live = p < P && g < G;
    float v[LMI_MAX_K];
    const float* L = kth_all + (size_t)(live ? g : 0) * stride + (size_t)(live ? p : 0) * k;
#pragma unroll
    for (int i = 0; i < LMI_MAX_K; ++i) v[i] = (live && i < k) ? L[i] : __builtin_inff();
    const uint64_t segmask = (W == 64 ? ~0ull : ((1ull << W) - 1ull)) << (seg * W);
    float m = __builtin_inff();
    for (int step = 0; step < k; ++step) {
        float mn = v[0];
        for (int off = W >> 1; off > 0; off >>= 1) mn = fminf(mn, __shfl_xor(mn, off));
        m = mn;
        const uint64_t b = __ballot(v[0] == mn) & segmask;
        if (b != 0ull && lane == (int)__builtin_ctzll(b)) {
#pragma unroll
            for (int i = 0; i + 1 < LMI_MAX_K; ++i) v[i] = v[i + 1];
            v[LMI_MAX_K - 1] = __builtin_inff();
        }
    }
    if (p < P && g == 0) out[p] = m;
}

__device__ inline double wave_sum_d(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// the 4-element pieces of a row a lane owns: piece l + 64 i (i < nps)
template <typename TC>
__device__ inline void load_piece(const TC* row, int piece, int d, double (&v)[4]) {
    const int e0 = 4 * piece;
    if constexpr (sizeof(TC) == 2) {
        if (e0 + 4 <= d) {
            const uint2 raw = *reinterpret_cast<const uint2*>(row + e0);
            _Float16 h[4];
            __builtin_memcpy(h, &raw, 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (double)h[j];
            return;
        }
    } else if constexpr (sizeof(TC) == 8) {
        if (e0 + 4 <= d) {
            const double2 a = *reinterpret_cast<const double2*>(row + e0);
            const double2 b = *reinterpret_cast<const double2*>(row + e0 + 2);
            v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
            return;
        }
    } else {
        if (e0 + 4 <= d) {
            const float4 f = *reinterpret_cast<const float4*>(row + e0);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (e0 + j < d) ? (double)row[e0 + j] : 0.0;
}

constexpr int kMaxPieces = 4;  // d <= 1024 (4 pieces of 4 per lane)

// q^ for this lane's pieces (sklearn normalize of the query row, float64)
template <typename TQ, int NP = kMaxPieces>
__device__ inline void query_hat(const TQ* qrow, int d, int nps, double (&qh)[NP][4]) {
    const int lane = threadIdx.x & 63;
    double ss = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 4 * (lane + 64 * i) + j;
            const double v = (i < nps && e < d) ? (double)qrow[e] : 0.0;
            qh[i][j] = v;
            ss = fma(v, v, ss);
        }
    }
    double n = sqrt(wave_sum_d(ss));
    if (n < 10.0 * kEps64) n = 1.0;  // sklearn _handle_zeros_in_scale
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) qh[i][j] = qh[i][j] / n;
}

// 1 - <q^, y/|y|> of one stored row, float64 (every lane gets the value)
template <typename TC, int NP = kMaxPieces>
__device__ inline double row_dist64(const TC* row, int d, int nps, const double (&qh)[NP][4]) {
    const int lane = threadIdx.x & 63;
    double dot = 0.0, ss = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        if (i < nps) {
            double v[4];
            load_piece<TC>(row, lane + 64 * i, d, v);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                dot = fma(qh[i][j], v[j], dot);
                ss = fma(v[j], v[j], ss);
            }
        }
    }
    dot = wave_sum_d(dot);
    double n = sqrt(wave_sum_d(ss));
    if (n < 10.0 * kEps64) n = 1.0;
    return 1.0 - dot / n;
}

// row_dist64 of up to kB fp16 rows at once (d % 4 == 0): every row's pieces
// are loaded before any is used, so a wave waits one memory latency per kB
// rows instead of one per row, and the 2 kB wave reductions interleave; each
// row's value is computed in exactly row_dist64's order (the same bits)
// (NPS: pieces per lane known at compile time, 3 for d in (512, 768])
constexpr int kB = 4;
template <int NPS, int KB = kB>
__device__ inline void rows_dist64_f16(const _Float16* base, size_t d_pad, const int32_t (&r)[KB], int d,
                                       int nps, const double (&qh)[NPS][4], double (&out)[KB]) {
    const int lane = threadIdx.x & 63;
    uint2 raw[KB][NPS];
#pragma unroll
    for (int b = 0; b < KB; ++b)
#pragma unroll
        for (int i = 0; i < NPS; ++i) {
            const int e0 = 4 * (lane + 64 * i);
            raw[b][i] = (r[b] >= 0 && i < nps && e0 + 4 <= d)
                            ? *reinterpret_cast<const uint2*>(base + (size_t)r[b] * d_pad + e0)
                            : make_uint2(0u, 0u);
        }
    double dot[KB], ss[KB];
#pragma unroll
    for (int b = 0; b < KB; ++b) {
        dot[b] = 0.0;
        ss[b] = 0.0;
#pragma unroll
        for (int i = 0; i < NPS; ++i) {
            if (i < nps) {
                _Float16 h[4];
                __builtin_memcpy(h, &raw[b][i], 8);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double v = (double)h[j];
                    dot[b] = fma(qh[i][j], v, dot[b]);
                    ss[b] = fma(v, v, ss[b]);
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            dot[b] += __shfl_xor(dot[b], off);
            ss[b] += __shfl_xor(ss[b], off);
        }
#pragma unroll
    for (int b = 0; b < KB; ++b) {
        double n = sqrt(ss[b]);
        if (n < 10.0 * kEps64) n = 1.0;
        out[b] = 1.0 - dot[b] / n;
    }
}

__device__ inline bool lt_dp(double a, int32_t pa, double b, int32_t pb) {
    return a < b || (a == b && pa < pb);
}

constexpr int kSlots = 4;  // list entries per lane: lists of <= 256 entries

// the slot-`s` value of lane `l` of a wave-uniform (s, l)
template <typename T, int NS>
__device__ inline T shfl_slot(const T (&v)[NS], int j) {
    const int s = j >> 6, l = j & 63;
    T x = v[0];
#pragma unroll
    for (int i = 1; i < NS; ++i) x = s == i ? v[i] : x;
    return __shfl(x, l);
}

// the rows the float64 distances are computed from (the stored fp16 / f32
// rows, or the caller's float64 rows) and the query rows (float32 or float64)
template <typename TC>
__device__ inline const TC* rows_of(const RefineArgs& a) {
    if constexpr (sizeof(TC) == 8) return a.corpus64;
    else return reinterpret_cast<const TC*>(a.corpus);
}
template <typename TQ>
__device__ inline const TQ* query_of(const RefineArgs& a, int64_t q) {
    if constexpr (sizeof(TQ) == 8) return a.q64 + (size_t)q * a.ldq64;
    else return a.q + (size_t)q * a.ldq;
}

// NP: pieces of 4 per lane held for the query (3: d <= 768; 4: d <= 1024)
template <typename TC, typename TQ, int NP, int KB = kB, int NSL = kSlots>
__global__ __launch_bounds__(kRefT) __attribute__((amdgpu_waves_per_eu(KB >= 4 ? 5 : (KB == 2 ? 6 : 7) + (NSL == 1 ? 1 : 0))))
void refine_kernel(RefineArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * (kRefT / 64) + (threadIdx.x >> 6);
    const int64_t P = (int64_t)a.nq * a.R;
    if (p >= P) return;
    const int kl = a.kl, k = a.k;
    const size_t li = (size_t)p * kl;
    // lane l, slot s holds list entry 64 s + l
    float dj[NSL];
    int32_t rj[NSL], gj[NSL];
    int n_valid = 0;
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
        const int e = 64 * s + lane;
        const bool has = e < kl;
        dj[s] = has ? a.ld[li + e] : __builtin_inff();
        rj[s] = has ? a.lrow[li + e] : -1;
        gj[s] = has ? a.lpos[li + e] : -1;
        n_valid += __popcll(__ballot(rj[s] >= 0));
    }
    // ABI 10: the k-th over every rank's list -- never above this rank's own
    // -- decides the band, so each rank refines only its rows of the merged
    // pair's band; computed before the query's registers are live
    float tg = 0.0f, tg0 = 0.0f;
    if (a.lbound && a.kth_all) {
        tg = a.kth_g[p];
        if (a.seeded && p % a.R != 0) tg0 = a.kth_g[p - p % a.R];
    }
    const int nps = (a.d + 255) / 256;
    double* od = a.out_d + (size_t)p * k;
    int32_t* op = a.out_pos + (size_t)p * k;
    int m;
    if (a.lbound) {
        // band lists: an unlisted row failed the scan's filter (d32 past the
        // pair's k-th + 2 eps) or has d32 >= lbound (+inf: no row was
        // dropped); the list holds the band unless lbound lies in it
        double t = n_valid >= k ? (double)a.ld[li + k - 1] + 2.0 * a.eps : __builtin_inf();
        if (a.kth_all)
            t = tg == __builtin_inff() ? __builtin_inf() : (double)tg + 2.0 * a.eps;
        // (LMI_Q_SEED_ROUND0, rounds r >= 1: the thresholded replay reads only
        // entries with d64 below round 0's final threshold D0 <= d32 10th of
        // pair (q, 0) + eps, i.e. rows with d32 < that + 2 eps; the list must
        // hold those alone -- the seed's own premise)
        double lim = t;
        if (a.seeded && p % a.R != 0) {
            const float t0 = a.kth_all ? tg0 : a.ld[(size_t)(p - p % a.R) * kl + k - 1];
            lim = fmin(lim, (double)t0 + 2.0 * a.eps);
        }
        const float ub = a.lbound[p];
        if (ub != __builtin_inff() && (double)ub <= lim) {
            if (lane == 0) a.failed[atomicAdd(a.n_failed, 1)] = (int32_t)p;
            return;
        }
        m = 0;
#pragma unroll
        for (int s = 0; s < NSL; ++s)
            m += __popcll(__ballot(64 * s + lane < kl && rj[s] >= 0 && (double)dj[s] <= t));
    } else if (n_valid < kl) {
        m = n_valid;  // the shard's whole bucket is listed
    } else {
        const double t = (double)a.ld[li + k - 1] + 2.0 * a.eps;
        m = 0;
#pragma unroll
        for (int s = 0; s < NSL; ++s)
            m += __popcll(__ballot(64 * s + lane < kl && (double)dj[s] <= t));
        if (m >= kl) {  // the band may continue past the list: exact fallback
            if (lane == 0) a.failed[atomicAdd(a.n_failed, 1)] = (int32_t)p;
            return;
        }
    }
    if (m == 0) {
        // (no listed row in the band: the global band of a stripe holding
        // none of the pair's merged band -- most pairs of most stripes at
        // G = 8 -- needs no query; the list is all padding)
        for (int j = lane; j < k; j += 64) {
            od[j] = __builtin_inf();
            op[j] = -1;
        }
        return;
    }
    // (the query, once the pair has rows to refine)
    double qh[NP][4];
    query_hat<TQ, NP>(query_of<TQ>(a, p / a.R), a.d, nps, qh);
#pragma unroll
    for (int s = 0; s < NSL; ++s)
        if (rj[s] >= (int64_t)a.n_rows) atomicOr(a.status, LMI_STATUS_INTERNAL);
    double mine[NSL];
#pragma unroll
    for (int s = 0; s < NSL; ++s) mine[s] = __builtin_inf();
    auto keep = [&](int j, double dv) {
        if (lane == (j & 63)) {
            const int s = j >> 6;
#pragma unroll
            for (int i = 0; i < NSL; ++i) mine[i] = s == i ? dv : mine[i];
        }
    };
    if constexpr (sizeof(TC) == 2) {
        if (a.d % 4 == 0) {
            // (the stored fp16 rows: KB at a time)
            for (int j0 = 0; j0 < m; j0 += KB) {
                int32_t r[KB];
#pragma unroll
                for (int b = 0; b < KB; ++b) {
                    const int32_t x = j0 + b < m ? shfl_slot(rj, j0 + b) : -1;
                    r[b] = (x < 0 || x >= a.n_rows) ? -1 : x;
                }
                double dv[KB];
                rows_dist64_f16<NP, KB>(rows_of<TC>(a), (size_t)a.d_pad, r, a.d, nps, qh, dv);
#pragma unroll
                for (int b = 0; b < KB; ++b)
                    if (r[b] >= 0) keep(j0 + b, dv[b]);
            }
            goto ranked;
        }
    }
    for (int j = 0; j < m; ++j) {
        const int32_t r = shfl_slot(rj, j);
        if (r < 0 || r >= a.n_rows) continue;
        const TC* row = rows_of<TC>(a) + (size_t)r * a.d_pad;
        keep(j, row_dist64<TC, NP>(row, a.d, nps, qh));
    }
ranked:
    // rank of every refined entry among the m by (d64, position)
    int rank[NSL] = {};
    for (int i = 0; i < m; ++i) {
        const double di = shfl_slot(mine, i);
        const int32_t gi = shfl_slot(gj, i);
#pragma unroll
        for (int s = 0; s < NSL; ++s)
            rank[s] += (64 * s + lane != i && lt_dp(di, gi, mine[s], gj[s])) ? 1 : 0;
    }
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
        if (64 * s + lane < m && rank[s] < k) {
            od[rank[s]] = mine[s];
            op[rank[s]] = gj[s];
        }
    }
    for (int j = m + lane; j < k; j += 64) {
        od[j] = __builtin_inf();
        op[j] = -1;
    }
}

// One workgroup per queued pair: float64 distance of every row of its bucket
// shard (a wave per row, kFbRows rows in flight); lane 0 of every wave keeps
// the wave's top-k in LDS, thread 0 merges the waves' lists.
constexpr int kFbK = 256;
// The sliced fallback (k <= kFbSliceK): each of the first kFbSlicedPairs
// failed pairs' bucket shard is cut into kFbSlices row slices, every (pair,
// slice) a 256-thread workgroup item of a fixed grid (a pair's rows run on
// kFbSlices CUs instead of one), each writing its slice's top-k; then one
// merge per pair.
constexpr int kFbSliceK = 16;
constexpr int kFbSlices = 32;
constexpr int kFbSlicedPairs = 512;
constexpr int kFbSliceT = 256;
// one wave on sliced failed pair f: its kFbSlices slice lists (k each, by
// (d64, position)) merged to the first k (wave 0 of fallback_kernel's
// workgroups, after fallback_slice_kernel: one launch fewer on the path)
__device__ void fallback_merge_pair(const RefineArgs& a, int f) {
    const int k = a.k;
    const int lane = threadIdx.x & 63;
    {
        const int64_t p = a.failed[f];
        const double* pd = a.pd + (size_t)f * kFbSlices * kFbSliceK;
        const int32_t* pg = a.pg + (size_t)f * kFbSlices * kFbSliceK;
        // lane s < kFbSlices walks slice s; each round the wave's minimum head
        // is taken (position breaks distance ties, like every merge here)
        int h = 0;
        double* od = a.out_d + (size_t)p * k;
        int32_t* op = a.out_pos + (size_t)p * k;
        for (int j = 0; j < k; ++j) {
            const bool has = lane < kFbSlices && h < k;
            const double x = has ? pd[lane * kFbSliceK + h] : __builtin_inf();
            const int32_t g = has ? pg[lane * kFbSliceK + h] : INT32_MAX;
            double bx = x;
            int32_t bg = g;
            int bl = lane;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const double ox = __shfl_xor(bx, off);
                const int32_t og = __shfl_xor(bg, off);
                const int ol = __shfl_xor(bl, off);
                if (lt_dp(ox, og, bx, bg) || (ox == bx && og == bg && ol < bl)) {
                    bx = ox;
                    bg = og;
                    bl = ol;
                }
            }
            if (lane == bl) ++h;
            if (lane == 0) {
                const bool empty = bg == INT32_MAX;
                od[j] = empty ? __builtin_inf() : bx;
                op[j] = empty ? -1 : bg;
            }
        }
    }
}

template <typename TC, typename TQ>
__global__ __launch_bounds__(kFbT) void fallback_kernel(RefineArgs a) {
    __shared__ double sd[kFbT / 64][kFbK];
    __shared__ int32_t sp[kFbT / 64][kFbK];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nf = *a.n_failed;
    const int k = a.k;
    const int nps = (a.d + 255) / 256;
    // (the first kFbSlicedPairs failed pairs of k <= kFbSliceK take the
    // sliced path: fallback_slice_kernel, then their merge in wave 0 here)
    const int f0 = a.pd ? kFbSlicedPairs : 0;
    if (a.pd && w == 0)
        for (int f = blockIdx.x; f < min(nf, kFbSlicedPairs); f += gridDim.x) fallback_merge_pair(a, f);
    for (int f = f0 + blockIdx.x; f < nf; f += gridDim.x) {
        const int64_t p = a.failed[f];
        const int c = a.classes[p];  // classes is [nq][R]: pair p = q*R + r
        const int64_t b0 = a.bucket_off[c], b1 = a.bucket_off[c + 1];
        double qh[kMaxPieces][4];
        query_hat(query_of<TQ>(a, p / a.R), a.d, nps, qh);
        double* L = sd[w];
        int32_t* G = sp[w];
        if (lane == 0)
            for (int i = 0; i < k; ++i) {
                L[i] = __builtin_inf();
                G[i] = INT32_MAX;
            }
        for (int64_t r0 = b0 + (int64_t)w * kFbRows; r0 < b1; r0 += (int64_t)(kFbT / 64) * kFbRows) {
            double dv[kFbRows];
#pragma unroll
            for (int u = 0; u < kFbRows; ++u) {
                const int64_t r = r0 + u;
                const TC* row = rows_of<TC>(a) + (size_t)(r < b1 ? r : b0) * a.d_pad;
                dv[u] = row_dist64<TC>(row, a.d, nps, qh);
            }
            if (lane == 0) {
#pragma unroll
                for (int u = 0; u < kFbRows; ++u) {
                    const int64_t r = r0 + u;
                    if (r >= b1) break;
                    const double x = dv[u];
                    const int32_t g = a.gpos[r];
                    if (!lt_dp(x, g, L[k - 1], G[k - 1])) continue;
                    // insertion into the ascending list of k entries
                    int i = k - 1;
                    while (i > 0 && lt_dp(x, g, L[i - 1], G[i - 1])) {
                        L[i] = L[i - 1];
                        G[i] = G[i - 1];
                        --i;
                    }
                    L[i] = x;
                    G[i] = g;
                }
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int head[kFbT / 64] = {};
            double* od = a.out_d + (size_t)p * k;
            int32_t* op = a.out_pos + (size_t)p * k;
            for (int j = 0; j < k; ++j) {
                int best = -1;
                for (int v = 0; v < kFbT / 64; ++v) {
                    if (head[v] >= k) continue;
                    if (best < 0 || lt_dp(sd[v][head[v]], sp[v][head[v]], sd[best][head[best]],
                                          sp[best][head[best]]))
                        best = v;
                }
                const double x = sd[best][head[best]];
                const int32_t g = sp[best][head[best]];
                ++head[best];
                const bool empty = g == INT32_MAX;
                od[j] = empty ? __builtin_inf() : x;
                op[j] = empty ? -1 : g;
            }
        }
        __syncthreads();
    }
}

template <typename TC, typename TQ>
__global__ __launch_bounds__(kFbSliceT) void fallback_slice_kernel(RefineArgs a) {
    __shared__ double sd[kFbSliceT / 64][kFbSliceK];
    __shared__ int32_t sp[kFbSliceT / 64][kFbSliceK];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nf = min(*a.n_failed, kFbSlicedPairs);
    const int k = a.k;
    const int nps = (a.d + 255) / 256;
    for (int item = blockIdx.x; item < nf * kFbSlices; item += gridDim.x) {
        const int f = item / kFbSlices, sl = item - f * kFbSlices;
        const int64_t p = a.failed[f];
        const int c = a.classes[p];
        const int64_t b0 = a.bucket_off[c], n = a.bucket_off[c + 1] - b0;
        const int64_t r_lo = b0 + n * sl / kFbSlices, r_hi = b0 + n * (sl + 1) / kFbSlices;
        double qh[3][4];
        query_hat<TQ, 3>(query_of<TQ>(a, p / a.R), a.d, nps, qh);
        double* L = sd[w];
        int32_t* G = sp[w];
        if (lane == 0)
            for (int i = 0; i < k; ++i) {
                L[i] = __builtin_inf();
                G[i] = INT32_MAX;
            }
        for (int64_t r0 = r_lo + (int64_t)w * kB; r0 < r_hi; r0 += (int64_t)(kFbSliceT / 64) * kB) {
            int32_t r[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) r[b] = r0 + b < r_hi ? (int32_t)(r0 + b) : -1;
            double dv[kB];
            bool done = false;
            if constexpr (sizeof(TC) == 2) {
                // (the fp16 rows' loads of kB rows in flight together)
                if (a.d % 4 == 0) {
                    rows_dist64_f16<3>(rows_of<TC>(a), (size_t)a.d_pad, r, a.d, nps, qh, dv);
                    done = true;
                }
            }
            if (!done) {
#pragma unroll
                for (int b = 0; b < kB; ++b)
                    dv[b] = row_dist64<TC, 3>(rows_of<TC>(a) + (size_t)(r[b] >= 0 ? r[b] : r_lo) * a.d_pad, a.d, nps,
                                              qh);
            }
            if (lane == 0) {
#pragma unroll
                for (int b = 0; b < kB; ++b) {
                    if (r[b] < 0) break;
                    const double x = dv[b];
                    const int32_t g = a.gpos[r[b]];
                    if (!lt_dp(x, g, L[k - 1], G[k - 1])) continue;
                    int i = k - 1;
                    while (i > 0 && lt_dp(x, g, L[i - 1], G[i - 1])) {
                        L[i] = L[i - 1];
                        G[i] = G[i - 1];
                        --i;
                    }
                    L[i] = x;
                    G[i] = g;
                }
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int head[kFbSliceT / 64] = {};
            double* od = a.pd + ((size_t)f * kFbSlices + sl) * kFbSliceK;
            int32_t* og = a.pg + ((size_t)f * kFbSlices + sl) * kFbSliceK;
            for (int j = 0; j < k; ++j) {
                int best = 0;
                for (int v = 1; v < kFbSliceT / 64; ++v)
                    if (lt_dp(sd[v][head[v]], sp[v][head[v]], sd[best][head[best]], sp[best][head[best]])) best = v;
                od[j] = sd[best][head[best]];
                og[j] = sp[best][head[best]];
                if (head[best] < k - 1) ++head[best];
                else sd[best][head[best]] = __builtin_inf(), sp[best][head[best]] = INT32_MAX;
            }
        }
        __syncthreads();
    }
}

struct RefineWs {
    size_t scan, ld, lrow, lpos, lbound, failed, nfailed, pd, pg, kth_g, total;
    int kl;       // scan list length refined (>= k + 5, or 15 for k <= 10)
    int passes;   // 0: one scan of kl entries, else lower-bound passes
};

RefineWs refine_ws(const lmi_index_desc* idx, int nq, int R, int k, int qmode) {
    RefineWs w{};
    if (k + 5 <= 15) {
        w.kl = 15;
        w.passes = 0;
    } else {
        int kp;
        w.passes = passes_of(idx, qmode, k + 5, &kp);
        w.kl = w.passes * kp;
    }
    const size_t P = (size_t)nq * R;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t at = off;
        off = align_up(off + bytes, 256);
        return at;
    };
    w.ld = take(P * w.kl * 4);
    w.lrow = take(P * w.kl * 4);
    w.lpos = take(P * w.kl * 4);
    w.lbound = take(P * 4);
    w.failed = take(P * 4);
    w.nfailed = take(256);
    w.pd = take((size_t)kFbSlicedPairs * kFbSlices * kFbSliceK * 8);
    w.pg = take((size_t)kFbSlicedPairs * kFbSlices * kFbSliceK * 4);
    w.kth_g = take(P * 4);
    w.scan = take(w.passes ? wide_ws_bytes(idx, nq, R, k + 5, qmode, w.kl)
                           : scan_workspace_bytes(idx, nq, R, w.kl, qmode));
    w.total = off;
    return w;
}

int num_cus_ref() {
    static int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) v = 256;
        return v > 0 ? v : 256;
    }();
    return n;
}

}  // namespace
}  // namespace lmi

// ---------------------------------------------------------------------------
// The split mode (ABI 9, idx->corpus32): a float32 corpus that is not
// fp16-exact.  lmi_scan.hip's bucket_topk_x runs the fp16 scan on the
// normalised, rounded rows and queries and then a collect scan of every row
// within d~_k + 2 eps_x of each pair (its candidates); here the candidates'
// exact distances are computed in float64 from the caller's rows and query,
// sorted, and the first k written (x_select_kernel); a pair whose candidates
// overflowed the collect buffer is scanned whole (x_fallback_kernel).
// ---------------------------------------------------------------------------
namespace lmi {
namespace {

constexpr double kEps32 = 1.1920928955078125e-07;

// 1 - <q^, y/|y|> of kB rows of float32 or float64 values at once (every row's
// pieces loaded before any is used), in row_dist64's order; sklearn's zero
// rule with the eps of the output dtype
template <typename TC, int NPS, int KB = kB>
__device__ inline void rows_dist64_x(const TC* base, size_t d_pad, const int32_t (&r)[KB], int d, int nps,
                                     const double (&qh)[NPS][4], double zero_eps, double (&out)[KB]) {
    const int lane = threadIdx.x & 63;
    double dot[KB], ss[KB];
    if constexpr (sizeof(TC) == 4) {
        // float32 rows stay float32 until used (half the registers of doubles)
        float v[KB][NPS][4];
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int i = 0; i < NPS; ++i) {
                const int e0 = 4 * (lane + 64 * i);
                const TC* row = base + (size_t)(r[b] >= 0 ? r[b] : 0) * d_pad;
                if (r[b] >= 0 && i < nps && e0 + 4 <= d) {
                    const float4 f = *reinterpret_cast<const float4*>(row + e0);
                    v[b][i][0] = f.x; v[b][i][1] = f.y; v[b][i][2] = f.z; v[b][i][3] = f.w;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[b][i][j] = (r[b] >= 0 && i < nps && e0 + j < d) ? row[e0 + j] : 0.0f;
                }
            }
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            dot[b] = 0.0;
            ss[b] = 0.0;
#pragma unroll
            for (int i = 0; i < NPS; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double x = (double)v[b][i][j];
                    dot[b] = fma(qh[i][j], x, dot[b]);
                    ss[b] = fma(x, x, ss[b]);
                }
        }
    } else {
        double v[KB][NPS][4];
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int i = 0; i < NPS; ++i) {
                if (r[b] >= 0 && i < nps) {
                    load_piece<TC>(base + (size_t)r[b] * d_pad, lane + 64 * i, d, v[b][i]);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[b][i][j] = 0.0;
                }
            }
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            dot[b] = 0.0;
            ss[b] = 0.0;
#pragma unroll
            for (int i = 0; i < NPS; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    dot[b] = fma(qh[i][j], v[b][i][j], dot[b]);
                    ss[b] = fma(v[b][i][j], v[b][i][j], ss[b]);
                }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            dot[b] += __shfl_xor(dot[b], off);
            ss[b] += __shfl_xor(ss[b], off);
        }
#pragma unroll
    for (int b = 0; b < KB; ++b) {
        double n = sqrt(ss[b]);
        if (n < 10.0 * zero_eps) n = 1.0;
        out[b] = 1.0 - dot[b] / n;
    }
}

// q^ with the zero rule of the output dtype (query_hat is float64's)
template <typename TQ, int NP>
__device__ inline void query_hat_x(const TQ* qrow, int d, int nps, double zero_eps, double (&qh)[NP][4]) {
    const int lane = threadIdx.x & 63;
    double ss = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 4 * (lane + 64 * i) + j;
            const double v = (i < nps && e < d) ? (double)qrow[e] : 0.0;
            qh[i][j] = v;
            ss = fma(v, v, ss);
        }
    double n = sqrt(wave_sum_d(ss));
    if (n < 10.0 * zero_eps) n = 1.0;
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) qh[i][j] = qh[i][j] / n;
}

// ---- the reference's float32 operation order (ABI 10; oracle blas32_*) ------
// utils.py:10-11 in float32 = sklearn normalize (np.einsum('ij,ij->i') row
// norms, then a division) + numpy.matmul (OpenBLAS sgemm) + 1 - S.  The
// orders are numpy 2.2's einsum loop (four lanes, each 16-element group's
// vectors in reverse order, product then add) and OpenBLAS 0.3.29's SkylakeX
// sgemm: the small-matrix kernel (sixteen FMA chains over k mod 16, summed
// pairwise) when M*N*K <= 96*96*100, else one FMA chain per 384-wide K block,
// the blocks added.  M = the (round, bucket) group's queries, N = the bucket's
// rows (tests/test_oracle_blas32.py pins the restatement to numpy bit for bit).
constexpr int kBlasSmallMNK = 96 * 96 * 100;
constexpr int kBlasKBlock = 384;
constexpr float kEps32f = 1.1920928955078125e-07f;
constexpr int LMI_MAX_R = 16;  // rounds the tail flags rank at once

// 0: not restated (the exact value rounded), 1: small kernel, 2: blocked
__device__ inline int blas32_kernel_of(const XArgs& a, int64_t p) {
    if (!a.qn32 || (a.d & 15)) return 0;
    const int c = a.classes[p];
    if (c < 0 || c >= a.C) return 0;
    const int64_t M = a.grp[(size_t)(p % a.R) * a.C + c];
    const int64_t N = a.goff[c + 1] - a.goff[c];
    if (M <= 1 || N <= 1 || (M <= 3 && N <= 3)) return 0;
    return M * N * (int64_t)a.d <= kBlasSmallMNK ? 1 : 2;
}
// the small kernel sums its chains by halves, not pairwise, in the product's
// corner block: the last M mod 4 queries of the group x the last N mod 4
// rows of the bucket (oracle blas32_dot)
__device__ inline bool blas32_corner(const XArgs& a, int64_t p, int32_t row) {
    if (!a.tailq[p]) return false;
    const int c = a.classes[p];
    const int64_t N = a.goff[c + 1] - a.goff[c];
    return (int64_t)a.gpos[row] - a.goff[c] >= N / 4 * 4;
}

// (each function turns FMA contraction off in its own scope: every product
// and sum is rounded where the reference rounds it)
// x / n correctly rounded from rn = RN(1 / n) (Markstein: one residual FMA and
// one correction; the same value as the IEEE division numpy's divps gives)
__device__ inline float div_rn(float x, float n, float rn) {
#pragma clang fp contract(off)
    const float q0 = x * rn;
    const float e = __builtin_fmaf(-q0, n, x);
    return __builtin_fmaf(e, rn, q0);
}

// 1 - <qn, y / |y|> in the reference's float32 order (kern from
// blas32_kernel_of; qn normalised by x_qn32_kernel), a quad of lanes per
// candidate (every lane of the quad returns it).  NORMED: y is the row
// already normalised (lmi_index_desc.corpus32n: the row's own norm and
// division, done once at build), else lane w = lane & 3 runs the einsum's
// chain w (the values 16 g + 4 v + w, v = 3 .. 0) and every value is divided
// here.  Small kernel: lane w runs the chains 4 v + w (v = 0 .. 3) -- the
// quad's four lanes read four consecutive values, so each wave instruction
// touches 16 cache lines, not 64 as a lane per row did.  Blocked kernel: lane
// w runs the chain of K block w (d <= 4 * 384), the blocks then added in order.
template <bool NORMED>
__device__ inline float blas32_dist_quad(const float* y, const float* qn, int d, int kern, bool corner) {
#pragma clang fp contract(off)
    const int w = threadIdx.x & 3;
    const int qb = (threadIdx.x & 63) & ~3;
    float n = 1.0f, rn = 1.0f;
    if constexpr (!NORMED) {
        float a = 0.0f;
        for (int g0 = 0; g0 < d; g0 += 64) {
            float x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = y[g0 + 4 * i + w];
#pragma unroll
            for (int gg = 0; gg < 4; ++gg)
#pragma unroll
                for (int v = 3; v >= 0; --v) a = a + x[4 * gg + v] * x[4 * gg + v];
        }
        const float s01 = __shfl(a, qb) + __shfl(a, qb + 1), s23 = __shfl(a, qb + 2) + __shfl(a, qb + 3);
        n = __builtin_sqrtf(s01 + s23);
        if (n < 10.0f * kEps32f) n = 1.0f;
        rn = 1.0f / n;
    }
    float s;
    if (kern == 1) {
        float c[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // chains 4 v + w
        for (int g0 = 0; g0 < d; g0 += 64) {
            float x[16], q[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                x[i] = y[g0 + 4 * i + w];
                q[i] = qn[g0 + 4 * i + w];
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if constexpr (NORMED) c[i & 3] = __builtin_fmaf(q[i], x[i], c[i & 3]);
                else c[i & 3] = __builtin_fmaf(q[i], div_rn(x[i], n, rn), c[i & 3]);
            }
        }
        // chain l = 4 v + w sits in lane w as c[v]: all sixteen to every lane
        float t[16];
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int ww = 0; ww < 4; ++ww) t[4 * v + ww] = __shfl(c[v], qb + ww);
        if (corner) {
#pragma unroll
            for (int h = 8; h >= 1; h >>= 1)
#pragma unroll
                for (int i = 0; i < h; ++i) t[i] = t[i] + t[i + h];
        } else {
#pragma unroll
            for (int h = 8; h >= 1; h >>= 1)
#pragma unroll
                for (int i = 0; i < h; ++i) t[i] = t[2 * i] + t[2 * i + 1];
        }
        s = t[0];
    } else {
        float c = 0.0f;
        const int b0 = w * kBlasKBlock;
        const int b1 = b0 + kBlasKBlock < d ? b0 + kBlasKBlock : d;
        for (int e0 = b0; e0 < b1; e0 += 64) {
            // (a 64-value step passes b1 only inside d_pad's zero padding:
            // d_pad = 768 and d a multiple of 16 in the split mode)
            float4 x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = *reinterpret_cast<const float4*>(y + e0 + 4 * i);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float4 q = *reinterpret_cast<const float4*>(qn + e0 + 4 * i);
                if constexpr (NORMED) {
                    c = __builtin_fmaf(q.x, x[i].x, c);
                    c = __builtin_fmaf(q.y, x[i].y, c);
                    c = __builtin_fmaf(q.z, x[i].z, c);
                    c = __builtin_fmaf(q.w, x[i].w, c);
                } else {
                    c = __builtin_fmaf(q.x, div_rn(x[i].x, n, rn), c);
                    c = __builtin_fmaf(q.y, div_rn(x[i].y, n, rn), c);
                    c = __builtin_fmaf(q.z, div_rn(x[i].z, n, rn), c);
                    c = __builtin_fmaf(q.w, div_rn(x[i].w, n, rn), c);
                }
            }
        }
        const int nb = (d + kBlasKBlock - 1) / kBlasKBlock;
        s = __shfl(c, qb);
        for (int b = 1; b < nb; ++b) s = s + __shfl(c, qb + b);
    }
    return 1.0f - s;
}

// Lanes per candidate of the float32 re-score (wave-uniform: kern is the
// pair's): the blocked kernel on normalised rows takes one lane per K block
// (d <= 768: 1 or 2 lanes), everything else a quad (blas32_dist_quad)
__device__ inline int blas32_lanes(const XArgs& a, int kern) {
    return (kern == 2 && a.rows32n) ? (a.d + kBlasKBlock - 1) / kBlasKBlock : 4;
}

// The float32 distance of local row x in the reference's order by its group
// of L = blas32_lanes lanes (every lane of the group returns it; ok is the
// group's).  L < 4: lane b of the group runs the chain of K block b over the
// normalised row, the blocks then added in order.
// NORM: a.rows32n is set (a compile-time split: each form keeps only its own
// registers).
template <bool NORM>
__device__ inline float blas32_dist_group(const XArgs& a, int64_t p, const float* qn, int64_t x, bool ok,
                                          int kern, int L) {
#pragma clang fp contract(off)
    if (!ok) return __builtin_inff();
    if (!NORM || L == 4) {
        const bool cr = kern == 1 && blas32_corner(a, p, (int32_t)x);
        return blas32_dist_quad<NORM>((NORM ? a.rows32n : a.rows32) + (size_t)x * a.d_pad, qn, a.d, kern, cr);
    }
    // the query's two K blocks through the scalar cache (qn is the pair's:
    // wave-uniform; the constant address space lets the loads be scalar) and
    // each lane's block picked per element; d_pad = 768 in the split mode, so
    // block 1's 384 values are inside the query's row even when L == 1, and a
    // step past d reads the zero padding (adding exact zeros)
    typedef float v4f __attribute__((ext_vector_type(4)));
    using cv4f = __attribute__((address_space(4))) const v4f;
    const cv4f* q0 = (cv4f*)(qn);
    const cv4f* q1 = (cv4f*)(qn + kBlasKBlock);
    const bool hi = (threadIdx.x & (L - 1)) != 0;
    const float* y = a.rows32n + (size_t)x * a.d_pad + (hi ? kBlasKBlock : 0);
    float c = 0.0f;
    for (int e0 = 0; e0 < kBlasKBlock; e0 += 64) {
        float4 v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = *reinterpret_cast<const float4*>(y + e0 + 4 * i);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const v4f qa = q0[e0 / 4 + i], qb = q1[e0 / 4 + i];
            c = __builtin_fmaf(hi ? qb.x : qa.x, v[i].x, c);
            c = __builtin_fmaf(hi ? qb.y : qa.y, v[i].y, c);
            c = __builtin_fmaf(hi ? qb.z : qa.z, v[i].z, c);
            c = __builtin_fmaf(hi ? qb.w : qa.w, v[i].w, c);
        }
    }
    const int base = (threadIdx.x & 63) & ~(L - 1);
    float s = __shfl(c, base);
    for (int b = 1; b < L; ++b) s = s + __shfl(c, base + b);
    return 1.0f - s;
}

// The queries normalised as sklearn does in float32, a wave per query: the
// lanes square their values (rounded) into LDS, four lanes run the einsum's
// four chains, and every lane divides its values by the norm
__global__ __launch_bounds__(256) void x_qn32_kernel(const float* __restrict__ q, int32_t ldq, int32_t nq, int32_t d,
                                                     int32_t d_pad, float* __restrict__ out) {
#pragma clang fp contract(off)
    __shared__ float sq[4][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = blockIdx.x * 4 + w;
    if (i >= nq || (d & 15) || d > 1024) return;  // ((d & 15): not restated, blas32_kernel_of returns 0)
    const float* row = q + (size_t)i * ldq;
    float* o = out + (size_t)i * d_pad;
    for (int e = lane; e < d; e += 64) {
        const float x = row[e];
        sq[w][e] = x * x;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float acc = 0.0f;
    if (lane < 4)
        for (int g = 0; g < d; g += 16)
#pragma unroll
            for (int v = 3; v >= 0; --v) acc = acc + sq[w][g + 4 * v + lane];
    const float s01 = __shfl(acc, 0) + __shfl(acc, 1), s23 = __shfl(acc, 2) + __shfl(acc, 3);
    float n = __builtin_sqrtf(s01 + s23);
    if (n < 10.0f * kEps32f) n = 1.0f;
    for (int e = lane; e < d_pad; e += 64) o[e] = e < d ? row[e] / n : 0.0f;
}

// queries of every (round, bucket) group (grp zeroed by the caller)
__global__ __launch_bounds__(256) void x_groups_kernel(const int32_t* __restrict__ classes, int64_t P, int32_t R,
                                                       int32_t C, int32_t* __restrict__ grp) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    const int c = classes[p];
    if (c >= 0 && c < C) atomicAdd(&grp[(size_t)(p % R) * C + c], 1);
}

// tailq[pair (q, r)] = q is among the last M mod 4 queries of its group
// (its rank in the group, ascending q, is >= 4 floor(M / 4)), a wave per
// bucket over the collect scan's plan (the bucket's pairs in ascending pair
// id, so every round's pairs in ascending q: ranks by ballots, 64 pairs at a
// time); and the buckets' global offsets (block 0, lane 0)
__global__ __launch_bounds__(64) void x_tail_kernel(const int32_t* __restrict__ pair_q,
                                                    const int32_t* __restrict__ counts, int32_t cm, int32_t R, int32_t C,
                                                    const int32_t* __restrict__ grp,
                                                    const int64_t* __restrict__ nrows_c,
                                                    const int64_t* __restrict__ bucket_off, uint8_t* __restrict__ tailq,
                                                    int64_t* __restrict__ goff) {
    const int lane = threadIdx.x, c = blockIdx.x;
    if (c == 0 && lane == 0) {
        int64_t acc = 0;
        for (int b = 0; b < C; ++b) {
            goff[b] = acc;
            acc += nrows_c ? nrows_c[b] : bucket_off[b + 1] - bucket_off[b];
        }
        goff[C] = acc;
    }
    // (the plan's bucket of c: cm c + cm - 1, cm buckets per class)
    const int cb = cm * c + cm - 1;
    int s = 0;
    for (int b = lane; b < cb; b += 64) s += counts[b];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    const int e = s + counts[cb];
    const uint64_t below = (1ull << lane) - 1ull;
    int base[LMI_MAX_R];
#pragma unroll
    for (int r = 0; r < LMI_MAX_R; ++r) base[r] = 0;
    for (int i0 = s; i0 < e; i0 += 64) {
        const int i = i0 + lane;
        const int p = i < e ? pair_q[i] : -1;
        const int rp = p >= 0 ? p % R : -1;
        int rank = 0;
#pragma unroll
        for (int r = 0; r < LMI_MAX_R; ++r) {
            if (r < R) {
                const uint64_t m = __ballot(rp == r);
                if (rp == r) rank = base[r] + __popcll(m & below);
                base[r] += __popcll(m);
            }
        }
        if (p >= 0) tailq[p] = rank >= (grp[(size_t)rp * C + c] & ~3) ? 1 : 0;
    }
}

template <bool OUT64>
__device__ inline double out_value(double x) {
    if constexpr (OUT64) return x;
    else return (double)(float)x;  // the float32 mode orders its own (rounded) values
}

template <typename TC, typename TQ>
__device__ inline const TC* x_rows(const XArgs& a) {
    if constexpr (sizeof(TC) == 8) return a.rows64;
    else return a.rows32;
}
template <typename TQ>
__device__ inline const TQ* x_query(const XArgs& a, int64_t q) {
    if constexpr (sizeof(TQ) == 8) return a.q64 + (size_t)q * a.ldq64;
    else return a.q + (size_t)q * a.ldq;
}

template <bool OUT64>
__device__ inline void x_store(const XArgs& a, size_t o, double v, int32_t pos) {
    if constexpr (OUT64) reinterpret_cast<double*>(a.out_d)[o] = v;
    else reinterpret_cast<float*>(a.out_d)[o] = (float)v;
    a.out_pos[o] = pos;
}

constexpr int kXT = 256;  // x_select: 4 waves on one pair
constexpr int kXW = 256;  // x_select_wave: the candidates a wave takes (4 per lane)

// the grouped pairs x_select_wave_kernel answers (a wave each): band
// candidates (every row under a sampled bound + 2 eps), at most kXW of them;
// x_select_kernel takes the rest (more candidates, whole-scan candidates) and
// queues the overflowed and unbounded pairs for the fallback
__device__ inline bool x_wave_pair(const XArgs& a, uint32_t n, int p) {
    return a.two_eps > 0.0 && n <= (uint32_t)kXW && n <= (uint32_t)a.cap && !(a.fix && a.fix[p]);
}

// the collect scan skipped the pair's sample rows (XArgs::soff) and its band
// (d~ <= t) reaches the sample's own k-th: an unlisted sample row may lie in
// it, so the pair is scored over its sample rows (x_fallback_kernel)
__device__ inline bool x_band_past_sample(const XArgs& a, int p, double t) {
    if (!a.soff) return false;
    const int c = a.classes[p];
    if (c < 0 || c >= a.C || !(a.soff[2 * c] < a.soff[2 * c + 1])) return false;
    return (double)a.skth[(size_t)p * a.k + a.k - 1] <= t;
}

// A workgroup on one grouped pair of the collect scan: the exact distance of
// every candidate (a wave per kB rows), a bitonic sort of (distance, row) in
// LDS -- rows ascend with global position inside a bucket shard, so this is
// the reference's (distance, g.index) order -- and the first k written.
template <typename TC, typename TQ, bool OUT64>
__device__ inline void x_select_pair(const XArgs& a, const int pp, double* sd, int32_t* sr, uint32_t& s_nr) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (a.pair_bucket[pp] < 0) return;
    const int p = a.pair_q[pp];
    const int64_t P = (int64_t)a.nq * a.R;
    if (p < 0 || p >= P) return;
    const uint32_t n = a.ccount[pp];
    if (x_wave_pair(a, n, p)) return;  // (x_select_wave_kernel's)
    // the collect buffer overflowed, or the pair had no sampled bound: the whole shard
    if (n > (uint32_t)a.cap || (a.fix && a.fix[p])) {
        if (tid == 0) a.failed[atomicAdd(a.n_failed, 1)] = p;
        return;
    }
    const uint64_t* src = a.cand + (size_t)pp * a.cap;
    const bool band = a.two_eps > 0.0;
    uint32_t nr = n;  // candidates re-scored
    if (band) {
        // every row under a sampled bound + 2 eps: sort the (d~, row) keys,
        // keep the rows within the k-th smallest d~ + 2 eps (the candidates
        // hold the k smallest d~, so that is the pair's own k-th)
        uint64_t* keys = reinterpret_cast<uint64_t*>(sd);
        uint32_t m = 1;
        while (m < n) m <<= 1;
        for (uint32_t i = tid; i < m; i += kXT) keys[i] = i < n ? src[i] : kEmptyKey;
        if (tid == 0) s_nr = 0u;
        __syncthreads();
        for (uint32_t k2 = 2; k2 <= m; k2 <<= 1) {
            for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < m; i += kXT) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const uint64_t x = keys[i], y = keys[l];
                        if ((x > y) == ((i & k2) == 0)) {
                            keys[i] = y;
                            keys[l] = x;
                        }
                    }
                }
                __syncthreads();
            }
        }
        const double t = n >= (uint32_t)a.k ? (double)ord2f((uint32_t)(keys[a.k - 1] >> 32)) + a.two_eps
                                            : __builtin_inf();
        if (x_band_past_sample(a, p, t)) {
            if (tid == 0) a.sfailed[atomicAdd(a.n_sfailed, 1)] = pp;
            return;
        }
        uint32_t c = 0;
        for (uint32_t i = tid; i < n; i += kXT) c += (double)ord2f((uint32_t)(keys[i] >> 32)) <= t ? 1u : 0u;
        atomicAdd(&s_nr, c);
        __syncthreads();
        nr = s_nr;  // (a prefix of the sorted keys)
        for (uint32_t i = tid; i < nr; i += kXT) sr[i] = (int32_t)(uint32_t)keys[i];
        __syncthreads();
    }
    const int kern = OUT64 ? 0 : blas32_kernel_of(a, p);
    if (kern != 0) {
        // the reference's float32 order: a group of L lanes per candidate
        const float* qn = a.qn32 + (size_t)(p / a.R) * a.d_pad;
        const int L = blas32_lanes(a, kern);
        for (uint32_t j0 = 0; j0 < nr; j0 += kXT / L) {
            const uint32_t j = j0 + tid / L;
            const int64_t x = j < nr ? (band ? (int64_t)sr[j] : (int64_t)(uint32_t)src[j]) : -1;
            const bool ok = x >= 0 && x < a.n_rows;
            const float v = a.rows32n ? blas32_dist_group<true>(a, p, qn, x, ok, kern, L)
                                       : blas32_dist_group<false>(a, p, qn, x, ok, kern, L);
            __syncthreads();  // (every group read its row index before any is overwritten)
            if (j < nr && (tid & (L - 1)) == 0) {
                if (!ok) atomicOr(a.status, LMI_STATUS_INTERNAL);
                sd[j] = ok ? (double)v : __builtin_inf();
                sr[j] = ok ? (int32_t)x : INT32_MAX;
            }
        }
    }
    const double zero_eps = OUT64 ? kEps64 : kEps32;
    const int nps = (a.d + 255) / 256;
    double qh[3][4];
    if (kern == 0) query_hat_x<TQ, 3>(x_query<TQ>(a, p / a.R), a.d, nps, zero_eps, qh);
    for (uint32_t j0 = (uint32_t)w * kB; kern == 0 && j0 < nr; j0 += (kXT / 64) * kB) {
        int32_t r[kB];
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            const int64_t x = j0 + b < nr ? (band ? (int64_t)sr[j0 + b] : (int64_t)(uint32_t)src[j0 + b]) : -1;
            r[b] = (x < 0 || x >= a.n_rows) ? -1 : (int32_t)x;
            if (j0 + b < nr && r[b] < 0 && lane == 0) atomicOr(a.status, LMI_STATUS_INTERNAL);
        }
        double dv[kB];
        rows_dist64_x<TC, 3>(x_rows<TC, TQ>(a), (size_t)a.d_pad, r, a.d, nps, qh, zero_eps, dv);
        if (lane == 0) {
#pragma unroll
            for (int b = 0; b < kB; ++b)
                if (j0 + b < nr) {
                    sd[j0 + b] = r[b] >= 0 ? out_value<OUT64>(dv[b]) : __builtin_inf();
                    sr[j0 + b] = r[b] >= 0 ? r[b] : INT32_MAX;
                }
        }
    }
    uint32_t m = 1;
    while (m < nr) m <<= 1;
    for (uint32_t i = nr + tid; i < m; i += kXT) {
        sd[i] = __builtin_inf();
        sr[i] = INT32_MAX;
    }
    __syncthreads();
    for (uint32_t k2 = 2; k2 <= m; k2 <<= 1) {
        for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
            for (uint32_t i = tid; i < m; i += kXT) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const double xd = sd[i], yd = sd[l];
                    const int32_t xr = sr[i], yr = sr[l];
                    const bool up = (i & k2) == 0;
                    const bool gt = xd > yd || (xd == yd && xr > yr);
                    if (gt == up) {
                        sd[i] = yd;
                        sd[l] = xd;
                        sr[i] = yr;
                        sr[l] = xr;
                    }
                }
            }
            __syncthreads();
        }
    }
    const size_t o = (size_t)p * a.k;
    for (int i = tid; i < a.k; i += kXT) {
        const bool has = i < (int)nr && sr[i] != INT32_MAX;
        x_store<OUT64>(a, o + i, has ? sd[i] : __builtin_inf(), has ? a.gpos[sr[i]] : -1);
    }
}

// (a grid of a few workgroups per CU walks the grouped pairs: most of them
// are the wave kernel's, and an early exit costs a loop step, not a
// workgroup launch at this kernel's register count)
template <typename TC, typename TQ, bool OUT64>
__global__ __launch_bounds__(kXT) void x_select_kernel(XArgs a) {
    extern __shared__ double x_lds[];
    __shared__ uint32_t s_nr;
    const int P = a.nq * a.R;
    // (after x_select_wave_kernel: only the pairs it listed -- a walk over
    // every grouped pair cost ~0.36 ms a batch of dependent loads to skip them)
    const int n = a.wgl ? *a.n_wgl : P;
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        x_select_pair<TC, TQ, OUT64>(a, a.wgl ? a.wgl[i] : i, x_lds, reinterpret_cast<int32_t*>(x_lds + a.cap), s_nr);
        __syncthreads();  // (the pair's LDS lists are read before the next pair's fill)
    }
}

__device__ inline uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off);
        v = o < v ? o : v;
    }
    return v;
}

// A wave per grouped pair with at most kXW band candidates (x_wave_pair): the
// same answer as x_select_kernel without its two LDS sorts and barriers.  The
// lanes hold the (d~, row) keys (4 each); the k-th smallest is found by k
// wave minima, the keys within it + 2 eps are compacted into the wave's LDS
// row list (any order), re-scored kB at a time, and the first k by (exact
// distance, row) are taken by k wave minima -- the (distance, g.index) order,
// rows ascending with global position inside a bucket shard.
template <typename TC, typename TQ, bool OUT64, int KB = kB, bool NORM = false>
// (the float32 output runs the reference's float32 order, blas32_dist_group;
// NORM: over the normalised rows, a.rows32n; 4 waves per SIMD leave it the
// registers of its 64-value load blocks)
__global__ __launch_bounds__(kXT) __attribute__((amdgpu_waves_per_eu(sizeof(TC) == 8 ? 1 : !OUT64 ? 4 : KB >= 4 ? 4 : KB == 2 ? 5 : 7))) void x_select_wave_kernel(XArgs a, int32_t n_pairs) {
    __shared__ int32_t s_rows[kXT / 64][kXW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int pp = __builtin_amdgcn_readfirstlane(blockIdx.x * (kXT / 64) + w);
    if (pp >= n_pairs || a.pair_bucket[pp] < 0) return;
    const int p = a.pair_q[pp];
    const int64_t P = (int64_t)a.nq * a.R;
    if (p < 0 || p >= P) return;
    const uint32_t n = a.ccount[pp];
    if (!x_wave_pair(a, n, p)) {
        // (x_select_kernel's: it walks this list instead of every pair)
        if (a.wgl && lane == 0) a.wgl[atomicAdd(a.n_wgl, 1)] = pp;
        return;
    }
    const uint64_t* src = a.cand + (size_t)pp * a.cap;
    uint64_t key[4], work[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint32_t i = 64u * s + lane;
        key[s] = i < n ? src[i] : kEmptyKey;
        work[s] = key[s];
    }
    const int k = a.k;
    // the k-th smallest key (keys are distinct: one per row)
    uint64_t kth = kEmptyKey;
    for (int r = 0; r < k; ++r) {
        const uint64_t m = wave_min_u64(std::min(std::min(work[0], work[1]), std::min(work[2], work[3])));
        kth = m;
        if (m == kEmptyKey) break;
#pragma unroll
        for (int s = 0; s < 4; ++s) work[s] = work[s] == m ? kEmptyKey : work[s];
    }
    const double t = (n >= (uint32_t)k && kth != kEmptyKey)
                         ? (double)ord2f((uint32_t)(kth >> 32)) + a.two_eps : __builtin_inf();
    if (x_band_past_sample(a, p, t)) {
        if (lane == 0) a.sfailed[atomicAdd(a.n_sfailed, 1)] = pp;
        return;
    }
    int32_t* rows = s_rows[w];
    int nr = 0;
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const bool sel = key[s] != kEmptyKey && (double)ord2f((uint32_t)(key[s] >> 32)) <= t;
        const uint64_t b = __ballot(sel);
        if (sel) rows[nr + __popcll(b & lt)] = (int32_t)(uint32_t)key[s];
        nr += __popcll(b);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // entry j (< nr) is kept by lane j % 64, slot j / 64
    double mine[4];
    int32_t mrow[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        mine[s] = __builtin_inf();
        mrow[s] = INT32_MAX;
    }
    const int kern = OUT64 ? 0 : blas32_kernel_of(a, p);
    if (kern != 0) {
        // the reference's float32 order: a group of L lanes per candidate,
        // 64 / L at a time; entry j's value moves to its keeper, lane j % 64
        const float* qn = a.qn32 + (size_t)(p / a.R) * a.d_pad;
        const int L = blas32_lanes(a, kern), per = 64 / L;
        for (int j0 = 0; j0 < nr; j0 += per) {
            const int jq = j0 + lane / L;
            int64_t x = jq < nr ? (int64_t)rows[jq] : -1;
            const bool ok = x >= 0 && x < a.n_rows;
            if (jq < nr && !ok && (lane & (L - 1)) == 0) atomicOr(a.status, LMI_STATUS_INTERNAL);
            const float v = blas32_dist_group<NORM>(a, p, qn, x, ok, kern, L);
            // (lanes j0 % 64 .. + per - 1 keep entries j0 .. j0 + per - 1, slot j0 / 64)
            const int t = lane - (j0 & 63);
            const float mv = __shfl(v, L * (t & (per - 1)));
            const int32_t mx = __shfl(ok ? (int32_t)x : INT32_MAX, L * (t & (per - 1)));
            if (t >= 0 && t < per && j0 + t < nr) {
                const int sl = j0 >> 6;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    mine[s] = s == sl ? (double)mv : mine[s];
                    mrow[s] = s == sl ? mx : mrow[s];
                }
            }
        }
    }
    // (the query's float64 hat only where it is used: the float32 order's
    // chains keep those registers)
    const double zero_eps = OUT64 ? kEps64 : kEps32;
    const int nps = (a.d + 255) / 256;
    double qh[3][4];
    if (kern == 0) query_hat_x<TQ, 3>(x_query<TQ>(a, p / a.R), a.d, nps, zero_eps, qh);
    for (int j0 = 0; kern == 0 && j0 < nr; j0 += KB) {
        int32_t r[KB];
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int64_t x = j0 + b < nr ? (int64_t)rows[j0 + b] : -1;
            r[b] = (x < 0 || x >= a.n_rows) ? -1 : (int32_t)x;
            if (j0 + b < nr && r[b] < 0 && lane == 0) atomicOr(a.status, LMI_STATUS_INTERNAL);
        }
        double dv[KB];
        rows_dist64_x<TC, 3, KB>(x_rows<TC, TQ>(a), (size_t)a.d_pad, r, a.d, nps, qh, zero_eps, dv);
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int j = j0 + b;
            if (j < nr && r[b] >= 0 && lane == (j & 63)) {
                const int sl = j >> 6;
                const double v = out_value<OUT64>(dv[b]);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    mine[s] = s == sl ? v : mine[s];
                    mrow[s] = s == sl ? r[b] : mrow[s];
                }
            }
        }
    }
    const size_t o = (size_t)p * k;
    for (int i = 0; i < k; ++i) {
        double bd = mine[0];
        int32_t br = mrow[0];
#pragma unroll
        for (int s = 1; s < 4; ++s)
            if (lt_dp(mine[s], mrow[s], bd, br)) {
                bd = mine[s];
                br = mrow[s];
            }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const double od = __shfl_xor(bd, off);
            const int32_t orw = __shfl_xor(br, off);
            if (lt_dp(od, orw, bd, br)) {
                bd = od;
                br = orw;
            }
        }
        const bool empty = br == INT32_MAX;
        if (lane == 0) x_store<OUT64>(a, o + i, empty ? __builtin_inf() : bd, empty ? -1 : a.gpos[br]);
        if (!empty) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
                if (mrow[s] == br) {
                    mine[s] = __builtin_inf();
                    mrow[s] = INT32_MAX;
                }
        }
    }
}

// The exact distances of a pair's rows vrow(j), j = j_lo .. j_hi - 1 (-1:
// none) by the NW waves of a workgroup (a wave per kB rows; the float32 output
// in the reference's order, a group of lanes per row, where blas32_kernel_of
// restates it); lane 0 of wave w keeps the wave's top-k by (distance, row) in
// L[w] / G[w].
template <typename TC, typename TQ, bool OUT64, int NW, typename VR>
__device__ inline void x_rows_topk(const XArgs& a, int64_t p, const VR& vrow, int64_t j_lo, int64_t j_hi,
                                   double (*L)[LMI_MAX_K], int32_t (*G)[LMI_MAX_K]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = a.k;
    const int nps = (a.d + 255) / 256;
    const double zero_eps = OUT64 ? kEps64 : kEps32;
    double* Lw = L[w];
    int32_t* Gw = G[w];
    if (lane == 0)
        for (int i = 0; i < k; ++i) {
            Lw[i] = __builtin_inf();
            Gw[i] = INT32_MAX;
        }
    auto keep = [&](double xv, int32_t rr) {
        if (!lt_dp(xv, rr, Lw[k - 1], Gw[k - 1])) return;
        int i = k - 1;
        while (i > 0 && lt_dp(xv, rr, Lw[i - 1], Gw[i - 1])) {
            Lw[i] = Lw[i - 1];
            Gw[i] = Gw[i - 1];
            --i;
        }
        Lw[i] = xv;
        Gw[i] = rr;
    };
    const int kern = OUT64 ? 0 : blas32_kernel_of(a, p);
    // the reference's float32 order: a group of nl lanes per row, 64 / nl rows
    // a wave
    const int nl = kern != 0 ? blas32_lanes(a, kern) : 4, per = 64 / nl;
    const float* qn = kern != 0 ? a.qn32 + (size_t)(p / a.R) * a.d_pad : nullptr;
    for (int64_t j0 = j_lo + (int64_t)w * per; kern != 0 && j0 < j_hi; j0 += (int64_t)NW * per) {
        const int64_t jx = j0 + lane / nl;
        const int64_t x = jx < j_hi ? vrow(jx) : -1;
        const bool ok = x >= 0 && x < a.n_rows;
        const float v = a.rows32n ? blas32_dist_group<true>(a, p, qn, ok ? x : 0, ok, kern, nl)
                                   : blas32_dist_group<false>(a, p, qn, ok ? x : 0, ok, kern, nl);
        for (int j = 0; j < per; ++j) {
            const float vj = __shfl(v, nl * j);
            const int32_t rr = __shfl(ok ? (int32_t)x : -1, nl * j);
            if (lane == 0 && rr >= 0) keep((double)vj, rr);
        }
    }
    double qh[3][4];
    if (kern == 0) query_hat_x<TQ, 3>(x_query<TQ>(a, p / a.R), a.d, nps, zero_eps, qh);
    for (int64_t j0 = j_lo + (int64_t)w * kB; kern == 0 && j0 < j_hi; j0 += (int64_t)NW * kB) {
        int32_t r[kB];
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            const int64_t x = j0 + b < j_hi ? vrow(j0 + b) : -1;
            r[b] = (x >= 0 && x < a.n_rows) ? (int32_t)x : -1;
        }
        double dv[kB];
        rows_dist64_x<TC, 3>(x_rows<TC, TQ>(a), (size_t)a.d_pad, r, a.d, nps, qh, zero_eps, dv);
        if (lane == 0) {
#pragma unroll
            for (int b = 0; b < kB; ++b)
                if (r[b] >= 0) keep(out_value<OUT64>(dv[b]), r[b]);
        }
    }
}

// thread 0: the first k of the NW waves' lists (ascending, (inf, INT32_MAX)
// padded) by (distance, row), handed to put(j, distance, row)
template <int NW, typename PUT>
__device__ inline void x_merge_waves(int k, double (*L)[LMI_MAX_K], int32_t (*G)[LMI_MAX_K], const PUT& put) {
    int head[NW] = {};
    for (int j = 0; j < k; ++j) {
        int best = -1;
        for (int v = 0; v < NW; ++v) {
            if (head[v] >= k) continue;
            if (best < 0 || lt_dp(L[v][head[v]], G[v][head[v]], L[best][head[best]], G[best][head[best]])) best = v;
        }
        put(j, L[best][head[best]], G[best][head[best]]);
        ++head[best];
    }
}

// A pair of sfailed (its band reached its skipped sample's k-th): its rows are
// the sample's [soff[2c], soff[2c+1]) and then its collected candidates
// outside it -- a superset of the pair's answer, each row once.
struct XSampleRows {
    int64_t b0, b1, nv;
    const uint64_t* cnd;
    __device__ int64_t operator()(int64_t j) const {
        if (j >= nv) return -1;
        if (j < b1 - b0) return b0 + j;
        const int64_t x = (int64_t)(uint32_t)cnd[j - (b1 - b0)];
        return (x >= b0 && x < b1) ? -1 : x;
    }
};
__device__ inline XSampleRows x_sample_rows(const XArgs& a, int pp, int64_t p) {
    const int c = a.classes[p];
    XSampleRows v;
    v.b0 = a.soff[2 * c];
    v.b1 = a.soff[2 * c + 1];
    v.cnd = a.cand + (size_t)pp * a.cap;
    v.nv = (v.b1 - v.b0) + (int64_t)min(a.ccount[pp], (uint32_t)a.cap);
    return v;
}
struct XBucketRows {
    int64_t b0, b1;
    __device__ int64_t operator()(int64_t j) const { return b0 + j < b1 ? b0 + j : -1; }
};

// The first kXSlicedPairs sfailed pairs: each pair's rows cut into kXSlices
// slices, every (pair, slice) a workgroup item (a pair's ~n_c / 16 sample rows
// on kXSlices CUs instead of one: ~1 ms a batch with one such pair before),
// each writing its slice's top-k to spd / spg; x_fallback_kernel merges them.
constexpr int kXSliceT = 256;  // (kXSlices, kXSlicedPairs: lmi_common.hpp)
template <typename TC, typename TQ, bool OUT64>
__global__ __launch_bounds__(kXSliceT) void x_fallback_slice_kernel(XArgs a) {
    __shared__ double sd[kXSliceT / 64][LMI_MAX_K];
    __shared__ int32_t sr[kXSliceT / 64][LMI_MAX_K];
    const int ns = min(*a.n_sfailed, kXSlicedPairs);
    for (int item = blockIdx.x; item < ns * kXSlices; item += gridDim.x) {
        const int f = item / kXSlices, sl = item - f * kXSlices;
        const int pp = a.sfailed[f];
        const int64_t p = a.pair_q[pp];
        const XSampleRows v = x_sample_rows(a, pp, p);
        x_rows_topk<TC, TQ, OUT64, kXSliceT / 64>(a, p, v, v.nv * sl / kXSlices, v.nv * (sl + 1) / kXSlices, sd, sr);
        __syncthreads();
        if (threadIdx.x == 0) {
            double* od = a.spd + ((size_t)f * kXSlices + sl) * a.k;
            int32_t* og = a.spg + ((size_t)f * kXSlices + sl) * a.k;
            x_merge_waves<kXSliceT / 64>(a.k, sd, sr, [&](int j, double x, int32_t r) {
                od[j] = x;
                og[j] = r;
            });
        }
        __syncthreads();
    }
}

// one wave on sliced sfailed pair f: its kXSlices slice lists merged to the
// first k (lane s walks slice s; position breaks distance ties)
template <bool OUT64>
__device__ inline void x_merge_slices(const XArgs& a, int f) {
    const int k = a.k, lane = threadIdx.x & 63;
    const int64_t p = a.pair_q[a.sfailed[f]];
    const double* pd = a.spd + (size_t)f * kXSlices * k;
    const int32_t* pg = a.spg + (size_t)f * kXSlices * k;
    int h = 0;
    for (int j = 0; j < k; ++j) {
        const bool has = lane < kXSlices && h < k;
        double bx = has ? pd[lane * k + h] : __builtin_inf();
        int32_t bg = has ? pg[lane * k + h] : INT32_MAX;
        int bl = lane;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const double ox = __shfl_xor(bx, off);
            const int32_t og = __shfl_xor(bg, off);
            const int ol = __shfl_xor(bl, off);
            if (lt_dp(ox, og, bx, bg) || (ox == bx && og == bg && ol < bl)) {
                bx = ox;
                bg = og;
                bl = ol;
            }
        }
        if (lane == bl) ++h;
        const bool empty = bg == INT32_MAX;
        if (lane == 0) x_store<OUT64>(a, (size_t)p * k + j, empty ? __builtin_inf() : bx, empty ? -1 : a.gpos[bg]);
    }
}

// One workgroup per overflowed pair: the exact distance of every row of its
// bucket shard (x_rows_topk over 16 waves), thread 0 merges the waves' lists;
// then the sfailed pairs past the sliced ones, over their sample rows and
// candidates.  Wave 0 first merges the sliced sfailed pairs' slice lists.
template <typename TC, typename TQ, bool OUT64>
__global__ __launch_bounds__(kFbT) void x_fallback_kernel(XArgs a) {
    __shared__ double sd[kFbT / 64][LMI_MAX_K];
    __shared__ int32_t sr[kFbT / 64][LMI_MAX_K];
    const int w = threadIdx.x >> 6;
    const int nf = *a.n_failed;
    const int ns = a.n_sfailed ? *a.n_sfailed : 0;
    const int nsl = min(ns, kXSlicedPairs);
    const int k = a.k;
    if (w == 0)
        for (int f = blockIdx.x; f < nsl; f += gridDim.x) x_merge_slices<OUT64>(a, f);
    for (int f = blockIdx.x; f < nf + (ns - nsl); f += gridDim.x) {
        const bool whole = f < nf;
        const int pp = whole ? -1 : a.sfailed[nsl + f - nf];
        const int64_t p = whole ? a.failed[f] : a.pair_q[pp];
        if (whole) {
            const int c = a.classes[p];  // classes [nq][R]: pair p = q*R + r
            const XBucketRows v{a.bucket_off[c], a.bucket_off[c + 1]};
            x_rows_topk<TC, TQ, OUT64, kFbT / 64>(a, p, v, 0, v.b1 - v.b0, sd, sr);
        } else {
            const XSampleRows v = x_sample_rows(a, pp, p);
            x_rows_topk<TC, TQ, OUT64, kFbT / 64>(a, p, v, 0, v.nv, sd, sr);
        }
        __syncthreads();
        if (threadIdx.x == 0)
            x_merge_waves<kFbT / 64>(k, sd, sr, [&](int j, double x, int32_t rr) {
                const bool empty = rr == INT32_MAX;
                x_store<OUT64>(a, (size_t)p * k + j, empty ? __builtin_inf() : x, empty ? -1 : a.gpos[rr]);
            });
        __syncthreads();
    }
}

template <typename TC, typename TQ, bool OUT64>
int launch_x3(const XArgs& a, int64_t P, hipStream_t s) {
    const size_t lds = (size_t)a.cap * (sizeof(double) + sizeof(int32_t));
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [] {
        attr_err = hipFuncSetAttribute((const void*)x_select_kernel<TC, TQ, OUT64>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    });
    LMI_HIP_TRY(attr_err);
    if (a.two_eps > 0.0) {
        const dim3 wg((unsigned)((P + kXT / 64 - 1) / (kXT / 64)));
        // (float32 rows: LMI_XSEL_KB rows in flight per wave; float64 rows: 4)
        int kb = sizeof(TC) == 4 ? env_config().xsel_kb : 4;
        if constexpr (!OUT64 && sizeof(TC) == 4) {
            if (a.rows32n) {  // (the float32 order over the normalised rows)
                if (kb == 1)
                    hipLaunchKernelGGL((x_select_wave_kernel<TC, TQ, OUT64, 1, true>), wg, dim3(kXT), 0, s, a, (int32_t)P);
                else if (kb == 2)
                    hipLaunchKernelGGL((x_select_wave_kernel<TC, TQ, OUT64, 2, true>), wg, dim3(kXT), 0, s, a, (int32_t)P);
                else
                    hipLaunchKernelGGL((x_select_wave_kernel<TC, TQ, OUT64, 4, true>), wg, dim3(kXT), 0, s, a, (int32_t)P);
                kb = -1;
            }
        }
        if constexpr (sizeof(TC) == 4) {
            if (kb == 1)
                hipLaunchKernelGGL((x_select_wave_kernel<TC, TQ, OUT64, 1>), wg, dim3(kXT), 0, s, a, (int32_t)P);
            else if (kb == 2)
                hipLaunchKernelGGL((x_select_wave_kernel<TC, TQ, OUT64, 2>), wg, dim3(kXT), 0, s, a, (int32_t)P);
        }
        if (kb != 1 && kb != 2 && kb != -1)
            hipLaunchKernelGGL((x_select_wave_kernel<TC, TQ, OUT64, 4>), wg, dim3(kXT), 0, s, a, (int32_t)P);
        LMI_LAUNCH_CHECK("x_select_wave_kernel");
    }
    const unsigned sg = (unsigned)std::max<int64_t>(1, std::min<int64_t>(P, 4 * num_cus_ref()));
    hipLaunchKernelGGL((x_select_kernel<TC, TQ, OUT64>), dim3(sg), dim3(kXT), lds, s, a);
    LMI_LAUNCH_CHECK("x_select_kernel");
    if (a.n_sfailed) {
        // (the sfailed pairs' slices: no work unless a pair's band reached its
        // skipped sample's k-th)
        const unsigned xg = (unsigned)std::max<int64_t>(1, std::min<int64_t>(P * kXSlices, 4 * num_cus_ref()));
        hipLaunchKernelGGL((x_fallback_slice_kernel<TC, TQ, OUT64>), dim3(xg), dim3(kXSliceT), 0, s, a);
        LMI_LAUNCH_CHECK("x_fallback_slice_kernel");
    }
    const unsigned fg = (unsigned)std::max<int64_t>(1, std::min<int64_t>(P, num_cus_ref()));
    hipLaunchKernelGGL((x_fallback_kernel<TC, TQ, OUT64>), dim3(fg), dim3(kFbT), 0, s, a);
    LMI_LAUNCH_CHECK("x_fallback_kernel");
    return LMI_OK;
}
}  // namespace

int launch_x_refine(const XArgs& a, int64_t P, hipStream_t s) {
    if (a.d > 3 * 256) {
        set_error("split mode: d=%d > 768", a.d);
        return LMI_E_UNSUPPORTED;
    }
    if (a.out_f64) {
        if (a.rows64) return a.q64 ? launch_x3<double, double, true>(a, P, s) : launch_x3<double, float, true>(a, P, s);
        return a.q64 ? launch_x3<float, double, true>(a, P, s) : launch_x3<float, float, true>(a, P, s);
    }
    if (a.qn32) {
        // the reference's float32 order: the queries normalised as sklearn
        // does, the (round, bucket) group sizes (XArgs; oracle blas32_*)
        hipLaunchKernelGGL(x_qn32_kernel, dim3((unsigned)((a.nq + 3) / 4)), dim3(256), 0, s, a.q, a.ldq, a.nq,
                           a.d, a.d_pad, const_cast<float*>(a.qn32));
        LMI_LAUNCH_CHECK("x_qn32_kernel");
        LMI_TRY(fill_u32(const_cast<int32_t*>(a.grp), 0u, (size_t)a.R * a.C, s));
        hipLaunchKernelGGL(x_groups_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, a.classes, P, a.R,
                           a.C, const_cast<int32_t*>(a.grp));
        LMI_LAUNCH_CHECK("x_groups_kernel");
        LMI_CHECK_ARG(a.R <= LMI_MAX_R, "R=%d > %d", a.R, LMI_MAX_R);
        hipLaunchKernelGGL(x_tail_kernel, dim3((unsigned)a.C), dim3(64), 0, s, a.pair_q, a.plan_counts,
                           std::max(1, a.plan_cm), a.R, a.C,
                           a.grp, a.nrows_c, a.bucket_off, const_cast<uint8_t*>(a.tailq), const_cast<int64_t*>(a.goff));
        LMI_LAUNCH_CHECK("x_tail_kernel");
    }
    return launch_x3<float, float, false>(a, P, s);
}
}  // namespace lmi

extern "C" size_t lmi_scan_f64_workspace_bytes(const lmi_index_desc* idx, int32_t nq, int32_t R,
                                               int32_t k, int32_t qmode) {
    qmode &= ~LMI_Q_SEED_ROUND0;
    lmi::take_phases(qmode);
    if (!idx || nq < 0 || R < 1 || k < 1 || k > LMI_MAX_K_F64) return 0;
    if (idx->corpus32) return k <= LMI_MAX_K ? lmi::x_ws_bytes(idx, nq, R, k) : 0;
    return lmi::refine_ws(idx, nq, R, k, qmode).total;
}

namespace lmi {
namespace {
template <typename TC, typename TQ>
void launch_refine(const RefineArgs& a, dim3 grid, dim3 fgrid, hipStream_t s) {
    // (d <= 768: three pieces per lane, the registers of the fourth freed)
    bool done = false;
    if constexpr (sizeof(TC) == 2) {
        // (fp16 rows, d <= 768, lists of <= 64 entries: one list slot per
        // lane, the registers of three freed for more waves per SIMD, and KB
        // rows in flight per wave, LMI_REFINE_KB)
        const int kb = env_config().refine_kb;
        if (a.d <= 3 * 256 && a.kl <= 64) {
            done = true;
            if (kb == 1)
                hipLaunchKernelGGL((refine_kernel<TC, TQ, 3, 1, 1>), grid, dim3(kRefT), 0, s, a);
            else if (kb == 4)
                hipLaunchKernelGGL((refine_kernel<TC, TQ, 3, 4, 1>), grid, dim3(kRefT), 0, s, a);
            else
                hipLaunchKernelGGL((refine_kernel<TC, TQ, 3, 2, 1>), grid, dim3(kRefT), 0, s, a);
        }
    }
    if (!done && a.d <= 3 * 256)
        hipLaunchKernelGGL((refine_kernel<TC, TQ, 3>), grid, dim3(kRefT), 0, s, a);
    else if (!done)
        hipLaunchKernelGGL((refine_kernel<TC, TQ, kMaxPieces>), grid, dim3(kRefT), 0, s, a);
    // one workgroup per queued pair (the grid strides over the queue; the
    // queue length is read on the device, usually 0); k <= kFbSliceK: the
    // first kFbSlicedPairs pairs in row slices over many workgroups instead
    if (a.pd) {
        hipLaunchKernelGGL((fallback_slice_kernel<TC, TQ>), dim3(2 * (unsigned)num_cus_ref()), dim3(kFbSliceT), 0,
                           s, a);
    }
    hipLaunchKernelGGL((fallback_kernel<TC, TQ>), fgrid, dim3(kFbT), 0, s, a);
}
template <typename TC>
void launch_refine_q(const RefineArgs& a, dim3 grid, dim3 fgrid, hipStream_t s) {
    if (a.q64) launch_refine<TC, double>(a, grid, fgrid, s);
    else launch_refine<TC, float>(a, grid, fgrid, s);
}
}  // namespace
}  // namespace lmi

extern "C" int lmi_bucket_topk_f64(const lmi_index_desc* idx, const float* q, int32_t nq,
                                   int32_t ldq, const int32_t* classes, int32_t R, int32_t k,
                                   int32_t qmode, double eps, double* out_d, int32_t* out_pos,
                                   int32_t* status, void* workspace, size_t ws_bytes,
                                   void* stream) {
    return lmi_bucket_topk_f64q(idx, q, nq, ldq, nullptr, 0, classes, R, k, qmode, eps, out_d,
                                out_pos, status, workspace, ws_bytes, stream);
}

namespace lmi {
namespace {

// lmi_bucket_topk_f64q, and with `global` (ABI 10, lmi_bucket_topk_f64g) the
// band decided over every rank's lists: the MERGE phase writes each pair's k
// smallest d32 to kth_send (chunk_merge_band_kernel, beside the lists), the
// REFINE phase reads the gathered kth_all
int bucket_topk_f64_impl(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                         const double* q64, int32_t ldq64, const int32_t* classes, int32_t R,
                         int32_t k, int32_t qmode, double eps, double* out_d, int32_t* out_pos,
                         int32_t* status, void* workspace, size_t ws_bytes, void* stream,
                         bool global, float* kth_send, const float* kth_all, int32_t kth_G,
                         int64_t kth_stride) {
    const bool seed = (qmode & LMI_Q_SEED_ROUND0) != 0;
    qmode &= ~LMI_Q_SEED_ROUND0;
    int phases;
    bool do_refine;
    if (global) {
        // PLAN / SCAN / MERGE (the chunk merge, writing kth_send) and REFINE;
        // none = all four (one rank: kth_all == kth_send)
        const bool ref = (qmode & LMI_Q_PHASE_REFINE) != 0;
        qmode &= ~LMI_Q_PHASE_REFINE;
        const bool any = ((qmode >> 9) & 7) != 0;
        phases = take_phases(qmode);
        if (!any && ref) phases = 0;
        do_refine = ref || !any;
        LMI_CHECK_ARG(any || ref || (kth_all == kth_send && kth_G == 1),
                      "one call of every phase needs kth_all == kth_send and G == 1");
        LMI_CHECK_ARG(!(phases & kPhaseMerge) || kth_send, "the MERGE phase needs kth_send");
        LMI_CHECK_ARG(!do_refine || (kth_all && kth_G >= 1 && kth_G <= 64 && kth_stride >= (int64_t)nq * R * k),
                      "the REFINE phase needs kth_all, 1 <= G <= 64, stride >= nq*R*k");
    } else {
        phases = take_phases(qmode);
        do_refine = (phases & kPhaseMerge) != 0;
    }
    LMI_CHECK_ARG(idx != nullptr, "null index");
    LMI_CHECK_ARG(k >= 1 && k <= LMI_MAX_K_F64, "k=%d outside [1, %d]", k, LMI_MAX_K_F64);
    LMI_CHECK_ARG(nq >= 0 && R >= 1 && (int64_t)nq * R < INT32_MAX, "bad nq/R");
    LMI_CHECK_ARG(idx->d >= 1 && idx->d <= 4 * 256, "d=%d outside [1, 1024] for float64 refinement",
                  idx->d);
    LMI_CHECK_ARG(eps >= 0.0 && eps < 1.0, "eps must lie in [0, 1)");
    if (nq == 0) return LMI_OK;
    LMI_CHECK_ARG(q && classes && out_d && out_pos && status && workspace, "null pointer");
    LMI_CHECK_ARG(q64 == nullptr || ldq64 >= idx->d, "ldq64 < d");
    if (idx->corpus32) {  // (phases: k <= 10, ABI 11; not the global band's REFINE)
        LMI_CHECK_ARG(!global, "the global band needs an index without corpus32");
        return bucket_topk_x(idx, q, nq, ldq, q64, ldq64, classes, R, k, out_d, 1, out_pos, status,
                             workspace, ws_bytes, reinterpret_cast<hipStream_t>(stream), phases);
    }
    const RefineWs w = refine_ws(idx, nq, R, k, qmode);
    if (ws_bytes < w.total) {
        set_error("workspace %zu B < required %zu B", ws_bytes, w.total);
        return LMI_E_WORKSPACE;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    const int kl = w.kl;
    RefineArgs a{};
    a.corpus = idx->corpus;
    a.dtype = idx->dtype;
    a.d = idx->d;
    a.d_pad = idx->d_pad;
    a.gpos = idx->gpos;
    a.bucket_off = idx->bucket_off;
    a.n_rows = idx->n_rows;
    a.q = q;
    a.ldq = ldq;
    a.corpus64 = idx->corpus64;
    a.q64 = q64;
    a.ldq64 = ldq64;
    a.classes = classes;
    a.nq = nq;
    a.R = R;
    a.kl = kl;
    a.k = k;
    a.eps = eps;
    a.ld = (const float*)(ws + w.ld);
    a.lrow = (const int32_t*)(ws + w.lrow);
    a.lpos = (const int32_t*)(ws + w.lpos);
    // k <= 10 on scan v3: the band lists (10-entry lane lists, the filter
    // widened by 2 eps, 15 entries + a bound per pair) instead of 15-entry
    // lane lists
    const bool band = !w.passes && band_capable(idx, qmode);
    a.lbound = band ? (const float*)(ws + w.lbound) : nullptr;
    a.seeded = seed ? 1 : 0;
    a.out_d = out_d;
    a.out_pos = out_pos;
    a.failed = (int32_t*)(ws + w.failed);
    a.n_failed = (int32_t*)(ws + w.nfailed);
    a.status = status;
    const bool sliced = k <= kFbSliceK && idx->d <= 3 * 256;  // (the slices hold 3 pieces of a query per lane)
    a.pd = sliced ? (double*)(ws + w.pd) : nullptr;
    a.pg = sliced ? (int32_t*)(ws + w.pg) : nullptr;
    if (w.passes && phases != kPhaseAll) {
        set_error("phase flags need k + 5 <= %d (one scan pass)", LMI_MAX_K);
        return LMI_E_UNSUPPORTED;
    }
    if (global && !band) {
        set_error("the global band needs the band lists (k <= 10 on the fp16 scan; "
                  "lmi_f64_global_band)");
        return LMI_E_UNSUPPORTED;
    }
    if (global) {
        a.kth_all = kth_all;
        a.kth_G = kth_G;
        a.kth_stride = kth_stride;
    }
    if (phases & kPhasePlan) LMI_TRY(fill_u32(ws + w.nfailed, 0u, 1, s));
    int rc = phases == 0 ? LMI_OK : w.passes
        ? bucket_topk_wide(idx, q, nq, ldq, classes, R, k + 5, qmode, (float*)(ws + w.ld),
                             (int32_t*)(ws + w.lpos), (int32_t*)(ws + w.lrow), kl, status,
                             ws + w.scan, w.total - w.scan, s)
        : bucket_topk_impl(idx, q, nq, ldq, classes, R, kl, qmode, (float*)(ws + w.ld),
                           (int32_t*)(ws + w.lpos), (int32_t*)(ws + w.lrow), status,
                           ws + w.scan, w.total - w.scan, s, nullptr, 0, true, seed,
                           (float)(2.0 * eps), phases, nullptr, band ? (float*)(ws + w.lbound) : nullptr,
                           global ? kth_send : nullptr, k);
    if (rc != LMI_OK) return rc;
    const int64_t P = (int64_t)nq * R;
    if (!do_refine) return LMI_OK;
    if (global && P > 0) {
        int W = 1;
        while (W < kth_G) W <<= 1;
        const int64_t pairs_per_block = 4 * (64 / W);
        a.kth_g = (const float*)(ws + w.kth_g);
        hipLaunchKernelGGL(band_kth_kernel, dim3((unsigned)((P + pairs_per_block - 1) / pairs_per_block)), dim3(256), 0,
                           s, kth_all, kth_G, kth_stride, P, k, (float*)(ws + w.kth_g));
        LMI_LAUNCH_CHECK("band_kth_kernel");
    }
    const dim3 grid((unsigned)((P + kRefT / 64 - 1) / (kRefT / 64)));
    const dim3 fgrid((unsigned)std::max<int64_t>(1, std::min<int64_t>(P, num_cus_ref())));
    if (idx->corpus64)
        launch_refine_q<double>(a, grid, fgrid, s);
    else if (idx->dtype == LMI_F16)
        launch_refine_q<_Float16>(a, grid, fgrid, s);
    else
        launch_refine_q<float>(a, grid, fgrid, s);
    LMI_LAUNCH_CHECK("refine_kernel / fallback_kernel");
    return LMI_OK;
}
}  // namespace
}  // namespace lmi

extern "C" int lmi_bucket_topk_f64q(const lmi_index_desc* idx, const float* q, int32_t nq,
                                    int32_t ldq, const double* q64, int32_t ldq64,
                                    const int32_t* classes, int32_t R, int32_t k, int32_t qmode,
                                    double eps, double* out_d, int32_t* out_pos, int32_t* status,
                                    void* workspace, size_t ws_bytes, void* stream) {
    return lmi::bucket_topk_f64_impl(idx, q, nq, ldq, q64, ldq64, classes, R, k, qmode, eps, out_d,
                                     out_pos, status, workspace, ws_bytes, stream, false, nullptr,
                                     nullptr, 0, 0);
}

extern "C" int lmi_f64_global_band(const lmi_index_desc* idx, int32_t nq, int32_t R, int32_t k,
                                   int32_t qmode) {
    using namespace lmi;
    qmode &= ~(LMI_Q_SEED_ROUND0 | LMI_Q_PHASE_REFINE);
    take_phases(qmode);
    if (!idx || idx->corpus32 || nq < 0 || R < 1 || k < 1 || k > LMI_MAX_K_F64) return 0;
    return (!refine_ws(idx, nq, R, k, qmode).passes && band_capable(idx, qmode)) ? 1 : 0;
}

extern "C" int lmi_bucket_topk_f64g(const lmi_index_desc* idx, const float* q, int32_t nq,
                                    int32_t ldq, const double* q64, int32_t ldq64,
                                    const int32_t* classes, int32_t R, int32_t k, int32_t qmode,
                                    double eps, float* kth_send, const float* kth_all, int32_t G,
                                    int64_t kth_stride, double* out_d, int32_t* out_pos,
                                    int32_t* status, void* workspace, size_t ws_bytes, void* stream) {
    LMI_CHECK_ARG(idx != nullptr && !idx->corpus32, "the global band needs an index without corpus32");
    return lmi::bucket_topk_f64_impl(idx, q, nq, ldq, q64, ldq64, classes, R, k, qmode, eps, out_d,
                                     out_pos, status, workspace, ws_bytes, stream, true, kth_send,
                                     kth_all, G, kth_stride);
}

extern "C" int lmi_refine_fallback_count(const void* workspace, const lmi_index_desc* idx,
                                         int32_t nq, int32_t R, int32_t k, int32_t qmode,
                                         int32_t* count_out, void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(workspace && idx && count_out, "null pointer");
    qmode &= ~LMI_Q_SEED_ROUND0;
    take_phases(qmode);
    const size_t at = idx->corpus32 ? x_nfailed_offset(idx, nq, R, k) : refine_ws(idx, nq, R, k, qmode).nfailed;
    LMI_HIP_TRY(hipMemcpyAsync(count_out, (const unsigned char*)workspace + at, 4,
                               hipMemcpyDeviceToHost, reinterpret_cast<hipStream_t>(stream)));
    LMI_HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    return LMI_OK;
}

extern "C" int lmi_split_sample_fallback_count(const void* workspace, const lmi_index_desc* idx, int32_t nq,
                                               int32_t R, int32_t k, int32_t* count_out, void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(workspace && idx && count_out, "null pointer");
    LMI_CHECK_ARG(idx->corpus32 != nullptr, "not a split-mode index (corpus32)");
    LMI_CHECK_ARG(nq >= 0 && R >= 1 && k >= 1 && k <= LMI_MAX_K, "bad nq/R/k");
    const size_t at = x_nfailed_offset(idx, nq, R, k) + 8 * sizeof(int32_t);
    LMI_HIP_TRY(hipMemcpyAsync(count_out, (const unsigned char*)workspace + at, 4,
                               hipMemcpyDeviceToHost, reinterpret_cast<hipStream_t>(stream)));
    LMI_HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    return LMI_OK;
}

extern "C" int lmi_split_normalize(const float* rows, int64_t n, int32_t d, int32_t d_pad, float* out,
                                   void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(n >= 0 && (n == 0 || (rows && out)), "null pointer");
    LMI_CHECK_ARG(d > 0 && d <= 1024 && (d & 15) == 0 && d_pad >= d,
                  "split normalise: d=%d d_pad=%d (d a multiple of 16, at most 1024)", d, d_pad);
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    constexpr int64_t kStep = int64_t(1) << 28;  // rows per launch (int32 row ids inside)
    for (int64_t a = 0; a < n; a += kStep) {
        const int32_t m = (int32_t)std::min<int64_t>(kStep, n - a);
        hipLaunchKernelGGL(x_qn32_kernel, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, s, rows + (size_t)a * d_pad,
                           d_pad, m, d, d_pad, out + (size_t)a * d_pad);
        LMI_LAUNCH_CHECK("x_qn32_kernel");
    }
    return LMI_OK;
}
