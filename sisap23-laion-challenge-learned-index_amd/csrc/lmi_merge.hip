// K3 — merge of per-shard top-k lists after the RCCL all-gather (gfx950).
//
// No reference counterpart: the reference is single-process.  A G-GPU index
// stripes every bucket over the ranks; the per-(query,
// probe) top-k of the whole bucket is the top-k of the union of the per-shard
// top-k lists, so rank outputs are all-gathered and merged here by the same
// (distance, global position) key the scan uses — the result is bitwise
// identical for any G.
#include "lmi_common.hpp"

#include <algorithm>

namespace lmi {
namespace {

constexpr int kThreads = 256;

// Rank g's lists start at d_in + g * gs_d and pos_in + g * gs_p (elements):
// [G][rows][k] arrays (gs = rows * k), or the all-gathered packed buffer of
// lmi_merge_topk_packed read in place.  With st_in, thread 0 also writes the
// OR of the G status words (rank g's at st_in + g * gs_st) to st_out.
__device__ inline void or_status(const int32_t* st_in, int64_t gs_st, int32_t G,
                                 int32_t* st_out) {
    if (st_in == nullptr || blockIdx.x != 0 || threadIdx.x != 0) return;
    int32_t v = 0;
    for (int g = 0; g < G; ++g) v |= st_in[(size_t)g * gs_st];
    *st_out = v;
}

template <int KL>
__global__ __launch_bounds__(kThreads) void merge_kernel(const float* __restrict__ d_in,
                                                         const int32_t* __restrict__ pos_in,
                                                         int32_t G, int64_t rows, int32_t k,
                                                         int64_t gs_d, int64_t gs_p,
                                                         const int32_t* __restrict__ st_in,
                                                         int64_t gs_st, int32_t* __restrict__ st_out,
                                                         float* __restrict__ out_d,
                                                         int32_t* __restrict__ out_pos) {
    or_status(st_in, gs_st, G, st_out);
    const int64_t row = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (row >= rows) return;
    uint64_t M[KL];
    list_clear<KL>(M);
    for (int g = 0; g < G; ++g) {
        const float* dg = d_in + (size_t)g * gs_d + (size_t)row * k;
        const int32_t* pg = pos_in + (size_t)g * gs_p + (size_t)row * k;
        for (int i = 0; i < k; ++i) {
            const int32_t p = pg[i];
            const uint64_t key = (p < 0) ? kEmptyKey : make_key(dg[i], (uint32_t)p);
            if (key >= M[KL - 1]) break;  // each input list is ascending
            list_insert<KL>(M, key);
        }
    }
#pragma unroll
    for (int i = 0; i < KL; ++i) {
        if (i < k) {
            const bool empty = M[i] == kEmptyKey;
            out_d[row * k + i] = empty ? __builtin_inff() : ord2f((uint32_t)(M[i] >> 32));
            out_pos[row * k + i] = empty ? -1 : (int32_t)(uint32_t)M[i];
        }
    }
}

// float64 lists (lmi_bucket_topk_f64): the same merge on (d64, position)
template <int KL>
__global__ __launch_bounds__(kThreads) void merge_f64_kernel(const double* __restrict__ d_in,
                                                             const int32_t* __restrict__ pos_in,
                                                             int32_t G, int64_t rows, int32_t k,
                                                             int64_t gs_d, int64_t gs_p,
                                                             const int32_t* __restrict__ st_in,
                                                             int64_t gs_st,
                                                             int32_t* __restrict__ st_out,
                                                             double* __restrict__ out_d,
                                                             int32_t* __restrict__ out_pos) {
    or_status(st_in, gs_st, G, st_out);
    const int64_t row = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (row >= rows) return;
    double M[KL];
    uint32_t Q[KL];  // positions as unsigned: -1 (empty) sorts last
#pragma unroll
    for (int i = 0; i < KL; ++i) {
        M[i] = __builtin_inf();
        Q[i] = 0xffffffffu;
    }
    auto lt = [](double a, uint32_t pa, double b, uint32_t pb) {
        return a < b || (a == b && pa < pb);
    };
    for (int g = 0; g < G; ++g) {
        const double* dg = d_in + (size_t)g * gs_d + (size_t)row * k;
        const int32_t* pg = pos_in + (size_t)g * gs_p + (size_t)row * k;
        for (int i = 0; i < k; ++i) {
            const int32_t p = pg[i];
            if (p < 0) break;  // each input list is ascending, empties last
            const double x = dg[i];
            const uint32_t u = (uint32_t)p;
            if (!lt(x, u, M[KL - 1], Q[KL - 1])) break;
#pragma unroll
            for (int j = KL - 1; j > 0; --j) {
                const bool take_prev = lt(x, u, M[j - 1], Q[j - 1]);
                const bool take_x = !take_prev && lt(x, u, M[j], Q[j]);
                M[j] = take_prev ? M[j - 1] : (take_x ? x : M[j]);
                Q[j] = take_prev ? Q[j - 1] : (take_x ? u : Q[j]);
            }
            if (lt(x, u, M[0], Q[0])) {
                M[0] = x;
                Q[0] = u;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < KL; ++i) {
        if (i < k) {
            const bool empty = Q[i] == 0xffffffffu;
            out_d[row * k + i] = empty ? __builtin_inf() : M[i];
            out_pos[row * k + i] = empty ? -1 : (int32_t)Q[i];
        }
    }
}

// k > LMI_MAX_K (the wide lists of the lower-bound passes, up to
// LMI_MAX_K_PASSES entries; k > 16 at G > 1 and the exact semantics over R
// wide lists): merge by rank, one thread per INPUT entry (g, row, i).  Its
// rank in the row's merged order is i plus, for every other list g', the
// number of entries of g' that come before it (a binary search: lists ascend
// by (distance, position); keys repeat only for empty slots (+inf, -1), and
// those order by list index g); entries of rank < k land at out[row][rank].
// The ranks of a row are a permutation of [0, G k), so out[row][0..k) is
// written exactly once.  Deterministic, no atomics.
template <typename T>
__device__ inline bool key_lt(T a, uint32_t pa, T b, uint32_t pb) {
    return a < b || (a == b && pa < pb);
}
template <typename T>
__global__ __launch_bounds__(kThreads) void merge_wide_kernel(const T* __restrict__ d_in,
                                                              const int32_t* __restrict__ pos_in,
                                                              int32_t G, int64_t rows, int32_t k,
                                                              int64_t gs_d, int64_t gs_p,
                                                              const int32_t* __restrict__ st_in,
                                                              int64_t gs_st, int32_t* __restrict__ st_out,
                                                              T* __restrict__ out_d,
                                                              int32_t* __restrict__ out_pos) {
    or_status(st_in, gs_st, G, st_out);
    const int64_t per_g = rows * k;
    const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (e >= per_g * G) return;
    const int g = (int)(e / per_g);
    const int64_t rem = e - (int64_t)g * per_g;
    const int64_t row = rem / k;
    const int i = (int)(rem - row * k);
    const int32_t p = pos_in[(size_t)g * gs_p + rem];
    const uint32_t u = (uint32_t)p;  // -1 (empty) sorts last
    const T x = p < 0 ? (T)__builtin_inf() : d_in[(size_t)g * gs_d + rem];
    int64_t rank = i;
    for (int g2 = 0; g2 < G; ++g2) {
        if (g2 == g) continue;
        const T* dl = d_in + (size_t)g2 * gs_d + (size_t)row * k;
        const int32_t* pl = pos_in + (size_t)g2 * gs_p + (size_t)row * k;
        // first j whose entry does not come before (x, u, g)
        int lo = 0, hi = k;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const int32_t pm = pl[mid];
            const uint32_t um = (uint32_t)pm;
            const T xm = pm < 0 ? (T)__builtin_inf() : dl[mid];
            const bool before = key_lt<T>(xm, um, x, u) || (xm == x && um == u && g2 < g);
            if (before) lo = mid + 1;
            else hi = mid;
        }
        rank += lo;
    }
    if (rank < k) {
        out_d[(size_t)row * k + rank] = x;
        out_pos[(size_t)row * k + rank] = p < 0 ? -1 : p;
    }
}

}  // namespace
}  // namespace lmi

namespace lmi {
namespace {
int launch_merge(const void* d_in, const int32_t* pos_in, int32_t G, int64_t rows, int32_t k,
                 bool f64, int64_t gs_d, int64_t gs_p, const int32_t* st_in, int64_t gs_st,
                 int32_t* st_out, void* out_d, int32_t* out_pos, hipStream_t s) {
    if (k > LMI_MAX_K) {
        const int64_t n = (int64_t)G * rows * k;
        const dim3 wgrid((unsigned)std::max<int64_t>(1, (n + kThreads - 1) / kThreads));
        if (f64)
            hipLaunchKernelGGL(merge_wide_kernel<double>, wgrid, dim3(kThreads), 0, s,
                               (const double*)d_in, pos_in, G, rows, k, gs_d, gs_p, st_in, gs_st,
                               st_out, (double*)out_d, out_pos);
        else
            hipLaunchKernelGGL(merge_wide_kernel<float>, wgrid, dim3(kThreads), 0, s,
                               (const float*)d_in, pos_in, G, rows, k, gs_d, gs_p, st_in, gs_st,
                               st_out, (float*)out_d, out_pos);
        LMI_LAUNCH_CHECK("merge_wide_kernel");
        return LMI_OK;
    }
    const dim3 grid((unsigned)std::max<int64_t>(1, (rows + kThreads - 1) / kThreads));
    if (f64) {
        auto* kp = k <= 10 ? merge_f64_kernel<10> : merge_f64_kernel<16>;
        hipLaunchKernelGGL(kp, grid, dim3(kThreads), 0, s, (const double*)d_in, pos_in, G, rows, k,
                           gs_d, gs_p, st_in, gs_st, st_out, (double*)out_d, out_pos);
        LMI_LAUNCH_CHECK("merge_f64_kernel");
    } else {
        auto* kp = k <= 10 ? merge_kernel<10> : merge_kernel<16>;
        hipLaunchKernelGGL(kp, grid, dim3(kThreads), 0, s, (const float*)d_in, pos_in, G, rows, k,
                           gs_d, gs_p, st_in, gs_st, st_out, (float*)out_d, out_pos);
        LMI_LAUNCH_CHECK("merge_kernel");
    }
    return LMI_OK;
}
}  // namespace
}  // namespace lmi

extern "C" int lmi_merge_topk_f64(const double* d_in, const int32_t* pos_in, int32_t G,
                                  int64_t rows, int32_t k, double* out_d, int32_t* out_pos,
                                  void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(G >= 1 && rows >= 0, "bad G/rows");
    LMI_CHECK_ARG(k >= 1 && k <= LMI_MAX_K_PASSES, "k=%d outside [1, %d]", k, LMI_MAX_K_PASSES);
    if (rows == 0) return LMI_OK;
    LMI_CHECK_ARG(d_in && pos_in && out_d && out_pos, "null pointer");
    return launch_merge(d_in, pos_in, G, rows, k, true, rows * k, rows * k, nullptr, 0, nullptr,
                        out_d, out_pos, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int lmi_merge_topk(const float* d_in, const int32_t* pos_in, int32_t G, int64_t rows,
                              int32_t k, float* out_d, int32_t* out_pos, void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(G >= 1 && rows >= 0, "bad G/rows");
    LMI_CHECK_ARG(k >= 1 && k <= LMI_MAX_K_PASSES, "k=%d outside [1, %d]", k, LMI_MAX_K_PASSES);
    if (rows == 0) return LMI_OK;
    LMI_CHECK_ARG(d_in && pos_in && out_d && out_pos, "null pointer");
    return launch_merge(d_in, pos_in, G, rows, k, false, rows * k, rows * k, nullptr, 0, nullptr,
                        out_d, out_pos, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int64_t lmi_packed_rank_words(int64_t rows, int32_t k, int32_t dist_f64) {
    const int64_t n = rows * k * (dist_f64 ? 3 : 2) + 1;
    return (n + 1) & ~(int64_t)1;
}

extern "C" int lmi_merge_topk_packed(const int32_t* gathered, int32_t G, int64_t rank_words,
                                     int64_t rows, int32_t k, int32_t dist_f64, void* out_d,
                                     int32_t* out_pos, int32_t* out_status, void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(G >= 1 && rows >= 0, "bad G/rows");
    LMI_CHECK_ARG(k >= 1 && k <= LMI_MAX_K_PASSES, "k=%d outside [1, %d]", k, LMI_MAX_K_PASSES);
    LMI_CHECK_ARG(rank_words >= lmi_packed_rank_words(rows, k, dist_f64) && rank_words % 2 == 0,
                  "rank_words %lld < lmi_packed_rank_words() or odd", (long long)rank_words);
    LMI_CHECK_ARG(gathered && out_status && (rows == 0 || (out_d && out_pos)), "null pointer");
    LMI_CHECK_ARG(((uintptr_t)gathered & 7) == 0, "gathered buffer not 8-byte aligned");
    const int64_t nd = rows * k * (dist_f64 ? 2 : 1);  // distance words per rank
    return launch_merge(gathered, gathered + nd, G, rows, k, dist_f64 != 0,
                        dist_f64 ? rank_words / 2 : rank_words, rank_words,
                        gathered + nd + rows * k, rank_words, out_status, out_d, out_pos,
                        reinterpret_cast<hipStream_t>(stream));
}

namespace lmi {
namespace {
__global__ void fill_u32_kernel(uint32_t* __restrict__ p, uint32_t value, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = value;
}
}  // namespace

int fill_u32(void* p, uint32_t value, size_t n_words, hipStream_t s) {
    if (n_words == 0) return LMI_OK;
    const size_t blocks = std::min<size_t>((n_words + 255) / 256, 4096);
    hipLaunchKernelGGL(fill_u32_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<uint32_t*>(p), value, n_words);
    LMI_LAUNCH_CHECK("fill_u32_kernel");
    return LMI_OK;
}
}  // namespace lmi
