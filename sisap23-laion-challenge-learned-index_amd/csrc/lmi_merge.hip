// K3 — merge of per-shard top-k lists after the RCCL all-gather (gfx950).
//
// No reference counterpart: the reference is single-process.  A G-GPU index
// stripes every bucket over the ranks; the per-(query,
// probe) top-k of the whole bucket is the top-k of the union of the per-shard
// top-k lists, so rank outputs are all-gathered and merged here by the same
// (distance, global position) key the scan uses — the result is bitwise
// identical for any G.
#include "lmi_common.hpp"

namespace lmi {
namespace {

constexpr int kThreads = 256;

template <int KL>
__global__ __launch_bounds__(kThreads) void merge_kernel(const float* __restrict__ d_in,
                                                         const int32_t* __restrict__ pos_in,
                                                         int32_t G, int64_t rows, int32_t k,
                                                         float* __restrict__ out_d,
                                                         int32_t* __restrict__ out_pos) {
    const int64_t row = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (row >= rows) return;
    uint64_t M[KL];
    list_clear<KL>(M);
    for (int g = 0; g < G; ++g) {
        const size_t base = ((size_t)g * rows + row) * k;
        for (int i = 0; i < k; ++i) {
            const int32_t p = pos_in[base + i];
            const uint64_t key = (p < 0) ? kEmptyKey : make_key(d_in[base + i], (uint32_t)p);
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
                                                             double* __restrict__ out_d,
                                                             int32_t* __restrict__ out_pos) {
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
        const size_t base = ((size_t)g * rows + row) * k;
        for (int i = 0; i < k; ++i) {
            const int32_t p = pos_in[base + i];
            if (p < 0) break;  // each input list is ascending, empties last
            const double x = d_in[base + i];
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

}  // namespace
}  // namespace lmi

extern "C" int lmi_merge_topk_f64(const double* d_in, const int32_t* pos_in, int32_t G,
                                  int64_t rows, int32_t k, double* out_d, int32_t* out_pos,
                                  void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(G >= 1 && rows >= 0, "bad G/rows");
    LMI_CHECK_ARG(k >= 1 && k <= LMI_MAX_K, "k=%d outside [1, %d]", k, LMI_MAX_K);
    if (rows == 0) return LMI_OK;
    LMI_CHECK_ARG(d_in && pos_in && out_d && out_pos, "null pointer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((rows + kThreads - 1) / kThreads));
    if (k <= 10)
        hipLaunchKernelGGL(merge_f64_kernel<10>, grid, dim3(kThreads), 0, s, d_in, pos_in, G, rows,
                           k, out_d, out_pos);
    else
        hipLaunchKernelGGL(merge_f64_kernel<16>, grid, dim3(kThreads), 0, s, d_in, pos_in, G, rows,
                           k, out_d, out_pos);
    LMI_LAUNCH_CHECK("merge_f64_kernel");
    return LMI_OK;
}

extern "C" int lmi_merge_topk(const float* d_in, const int32_t* pos_in, int32_t G, int64_t rows,
                              int32_t k, float* out_d, int32_t* out_pos, void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(G >= 1 && rows >= 0, "bad G/rows");
    LMI_CHECK_ARG(k >= 1 && k <= LMI_MAX_K, "k=%d outside [1, %d]", k, LMI_MAX_K);
    if (rows == 0) return LMI_OK;
    LMI_CHECK_ARG(d_in && pos_in && out_d && out_pos, "null pointer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((rows + kThreads - 1) / kThreads));
    if (k <= 10)
        hipLaunchKernelGGL(merge_kernel<10>, grid, dim3(kThreads), 0, s, d_in, pos_in, G, rows, k,
                           out_d, out_pos);
    else
        hipLaunchKernelGGL(merge_kernel<16>, grid, dim3(kThreads), 0, s, d_in, pos_in, G, rows, k,
                           out_d, out_pos);
    LMI_LAUNCH_CHECK("merge_kernel");
    return LMI_OK;
}
