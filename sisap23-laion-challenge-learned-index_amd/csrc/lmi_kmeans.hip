// K5 — k-means for the index build, gfx950.
//
// The reference clusters the pca96 navigation data with faiss.Kmeans
// (LearnedIndex.py:242-282: seed 2023, faiss' defaults niter = 25 and
// max_points_per_centroid = 256) and labels every object with
// `kmeans.index.search(X, 1)` (:282).  Those labels train the router.
// faiss is not in this image; this file is the device half of a
// Lloyd iteration whose host loop is li/kmeans.py:
//
//   kmeans_assign_kernel  nearest centroid of every point (squared L2,
//                         ties -> lower centroid index, as faiss' argmin)
//   kmeans_accum_kernel   per-slice fp64 sums and counts in a fixed order
//   kmeans_reduce_kernel  slices summed in slice order -> new centroids
//
// Everything is deterministic and reproduced bit for bit by
// oracle/lmi_oracle.py (kmeans_assign / kmeans_update):
// - distance = Σ_e (x_e - c_e)² accumulated over e in ascending order with
//   separately rounded fp32 subtract / multiply / add (no FMA contraction);
//   the padding columns add exact zeros;
// - sums: slice s owns points [s·n/S, (s+1)·n/S) and adds them in point
//   order into its own fp64 partial (no atomics); the reduce adds the S
//   partials in slice order and rounds sum/count to fp32 once.
//
// The assignment is VALU-bound (3 fp32 ops per point·centroid·dim, 96·122
// per point at the reference shape) with centroids broadcast from LDS and a
// point's row held in registers; HBM traffic is one read of X.
#include "lmi_common.hpp"

namespace lmi {
namespace {

constexpr int kThreads = 256;
constexpr int kCentLds = 16384;  // floats of the LDS centroid tile (64 KiB)
constexpr int kSlices = 512;     // fixed partition of the points for the sums (<= 512 slices of >= 128 points)

// #pragma clang fp contract(off) keeps a*b+c as two rounded operations
template <int DP>
__global__ __launch_bounds__(kThreads) void kmeans_assign_kernel(
    const float* __restrict__ x, int64_t n, int32_t d, const float* __restrict__ cent, int32_t k,
    int32_t* __restrict__ labels, float* __restrict__ dist) {
#pragma clang fp contract(off)
    __shared__ float4 cs[kCentLds / 4];
    constexpr int KT = kCentLds / DP;  // centroids per LDS tile
    const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const bool live = p < n;
    float xr[DP];
    const float* xp = x + (live ? p : 0) * (int64_t)d;
#pragma unroll
    for (int e = 0; e < DP; ++e) xr[e] = (live && e < d) ? xp[e] : 0.0f;
    float best = __builtin_inff();
    int bi = 0;
    for (int t0 = 0; t0 < k; t0 += KT) {
        const int nt = min(KT, k - t0);
        __syncthreads();
        for (int i = threadIdx.x; i < nt * DP; i += kThreads) {
            const int j = i / DP, e = i - j * DP;
            reinterpret_cast<float*>(cs)[i] = (e < d) ? cent[(int64_t)(t0 + j) * d + e] : 0.0f;
        }
        __syncthreads();
        for (int j = 0; j < nt; ++j) {
            const float4* cj = cs + j * (DP / 4);
            float acc = 0.0f;
#pragma unroll
            for (int e4 = 0; e4 < DP / 4; ++e4) {
                const float4 c = cj[e4];  // one broadcast LDS read for the wave
                float t;
                t = xr[4 * e4 + 0] - c.x; acc = acc + t * t;
                t = xr[4 * e4 + 1] - c.y; acc = acc + t * t;
                t = xr[4 * e4 + 2] - c.z; acc = acc + t * t;
                t = xr[4 * e4 + 3] - c.w; acc = acc + t * t;
            }
            if (acc < best) {  // strict: the first minimum wins
                best = acc;
                bi = t0 + j;
            }
        }
    }
    if (live) {
        labels[p] = bi;
        if (dist) dist[p] = best;
    }
}

// One workgroup per slice; thread e owns column e of the slice's partial.
__global__ __launch_bounds__(kThreads) void kmeans_accum_kernel(
    const float* __restrict__ x, int64_t n, int32_t d, const int32_t* __restrict__ labels, int32_t k,
    int32_t S, double* __restrict__ part, int64_t* __restrict__ pcount, int32_t* __restrict__ status) {
    const int s = blockIdx.x;
    const int64_t a = (int64_t)s * n / S, b = (int64_t)(s + 1) * n / S;
    double* ps = part + (size_t)s * k * d;
    int64_t* pc = pcount + (size_t)s * k;
    for (int64_t p0 = a; p0 < b; p0 += 64) {
        const int m = (b - p0 < 64) ? (int)(b - p0) : 64;
        for (int i = 0; i < m; ++i) {
            const int c = labels[p0 + i];  // uniform across the workgroup
            if (c < 0 || c >= k) {
                if (threadIdx.x == 0) atomicOr(status, 1);
                continue;
            }
            for (int e = threadIdx.x; e < d; e += kThreads)
                ps[(size_t)c * d + e] += (double)x[(p0 + i) * d + e];
            if (threadIdx.x == 0) pc[c] += 1;
        }
    }
}

__global__ __launch_bounds__(kThreads) void kmeans_reduce_kernel(
    const double* __restrict__ part, const int64_t* __restrict__ pcount, int32_t S, int32_t k,
    int32_t d, float* __restrict__ cent, int64_t* __restrict__ counts) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= (int64_t)k * d) return;
    const int c = (int)(i / d);
    double sum = 0.0;
    int64_t cnt = 0;
    for (int s = 0; s < S; ++s) {
        sum += part[(size_t)s * k * d + i];
        cnt += pcount[(size_t)s * k + c];
    }
    if (cnt > 0) cent[i] = (float)(sum / (double)cnt);
    if (i - (int64_t)c * d == 0 && counts) counts[c] = cnt;
}

int slices_for(int64_t n) {
    const int64_t s = (n + 127) / 128;
    return (int)(s < 1 ? 1 : (s > kSlices ? kSlices : s));
}

}  // namespace
}  // namespace lmi

extern "C" int lmi_kmeans_assign(const float* x, int64_t n, int32_t d, const float* cent, int32_t k,
                                 int32_t* labels_out, float* dist_out, void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(n >= 0, "n=%lld < 0", (long long)n);
    LMI_CHECK_ARG(d >= 1 && d <= LMI_KMEANS_MAX_D, "d=%d outside [1, %d]", d, LMI_KMEANS_MAX_D);
    LMI_CHECK_ARG(k >= 1, "k=%d < 1", k);
    if (n == 0) return LMI_OK;
    LMI_CHECK_ARG(x && cent && labels_out, "null pointer");
    LMI_CHECK_ARG(n <= (int64_t)INT32_MAX * kThreads, "n too large");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((n + kThreads - 1) / kThreads));
    if (d <= 32)
        hipLaunchKernelGGL(kmeans_assign_kernel<32>, grid, dim3(kThreads), 0, s, x, n, d, cent, k,
                           labels_out, dist_out);
    else if (d <= 64)
        hipLaunchKernelGGL(kmeans_assign_kernel<64>, grid, dim3(kThreads), 0, s, x, n, d, cent, k,
                           labels_out, dist_out);
    else if (d <= 96)
        hipLaunchKernelGGL(kmeans_assign_kernel<96>, grid, dim3(kThreads), 0, s, x, n, d, cent, k,
                           labels_out, dist_out);
    else
        hipLaunchKernelGGL(kmeans_assign_kernel<128>, grid, dim3(kThreads), 0, s, x, n, d, cent, k,
                           labels_out, dist_out);
    LMI_LAUNCH_CHECK("kmeans_assign_kernel");
    return LMI_OK;
}

extern "C" size_t lmi_kmeans_workspace_bytes(int64_t n, int32_t d, int32_t k) {
    if (n < 0 || d < 1 || k < 1) return 0;
    const size_t S = (size_t)lmi::slices_for(n);
    return lmi::align_up(S * k * d * sizeof(double), 256) + S * k * sizeof(int64_t);
}

extern "C" int lmi_kmeans_update(const float* x, int64_t n, int32_t d, const int32_t* labels,
                                 int32_t k, float* cent_out, int64_t* counts_out, int32_t* status,
                                 void* workspace, size_t ws_bytes, void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(n >= 0 && d >= 1 && k >= 1, "bad n/d/k");
    LMI_CHECK_ARG(cent_out && counts_out && status, "null pointer");
    LMI_CHECK_ARG(n == 0 || (x && labels), "null pointer");
    const size_t need = lmi_kmeans_workspace_bytes(n, d, k);
    if (ws_bytes < need || !workspace) {
        set_error("workspace %zu < %zu bytes", ws_bytes, need);
        return LMI_E_WORKSPACE;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int S = slices_for(n);
    double* part = reinterpret_cast<double*>(workspace);
    int64_t* pcount = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(workspace) +
                                                 align_up((size_t)S * k * d * sizeof(double), 256));
    LMI_HIP_TRY(hipMemsetAsync(workspace, 0, need, s));
    if (n > 0) {
        hipLaunchKernelGGL(kmeans_accum_kernel, dim3(S), dim3(kThreads), 0, s, x, n, d, labels, k, S,
                           part, pcount, status);
        LMI_LAUNCH_CHECK("kmeans_accum_kernel");
    }
    const int64_t kd = (int64_t)k * d;
    hipLaunchKernelGGL(kmeans_reduce_kernel, dim3((unsigned)((kd + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, s, part, pcount, S, k, d, cent_out, counts_out);
    LMI_LAUNCH_CHECK("kmeans_reduce_kernel");
    return LMI_OK;
}
