// K1 — router inference (MLP bucket classifier) on gfx950.
//
// Replaces NeuralNetwork.predict_proba (reference search/li/model.py:214-229:
// Linear/ReLU stack, softmax(dim=1), topk over all classes) and
// NeuralNetwork.predict (model.py:201-212: argmax of the logits, used for the
// object labels at LearnedIndex.py:240).
//
// One workgroup (4 waves) owns a tile of TQ query rows.  The activations of
// the tile live in LDS (two ping-pong buffers, one row per query, padded to an
// odd-ish stride so per-lane row reads are conflict-free); every lane owns one
// query and a group of output neurons; weight rows are read straight from
// global memory (they are tiny: 112 KB for 'MLP', 294 KB for 'MLP-5', and are
// shared by all workgroups through L2).  Each output is the fp32 FMA chain
// b[o] + sum_i h[i] * W[o][i] in ascending i, i.e. torch's Linear up to
// summation order.  The last layer's logits stay in LDS and are reduced to the
// top-R classes (descending logit, ties to the lower class index) and their
// softmax probabilities, or to the argmax.
#include "lmi_common.hpp"

namespace lmi {
namespace {

struct RouterArgs {
    const float* x;
    int32_t nq, ldx;
    int32_t n_layers;
    int32_t dims[LMI_MAX_LAYERS + 1];
    const float* W[LMI_MAX_LAYERS];
    const float* b[LMI_MAX_LAYERS];
    int32_t stride;  // LDS row stride in floats
    int32_t R, mode;
    int32_t* classes;
    float* probs;
};

constexpr int kThreads = 256;
constexpr int kOB = 4;  // outputs per lane per pass (register blocking)

// (logit a, class ia) ranks before (logit b, class ib)?
__device__ inline bool better(float a, int ia, float b, int ib) {
    return a > b || (a == b && ia < ib);
}

template <int TQ>
__global__ __launch_bounds__(kThreads) void router_kernel(RouterArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int G = 64 / TQ;    // query groups per wave
    constexpr int NG = 4 * G;     // output groups per workgroup
    const int S = a.stride;
    float* H[2] = {smem, smem + TQ * S};
    float* stat = smem + 2 * TQ * S;  // [TQ][2]: max, sum

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int ql = lane % TQ;
    const int grp = wave * G + lane / TQ;
    const int q0 = blockIdx.x * TQ;

    // Stage the query tile.
    const int din0 = a.dims[0];
    for (int e = tid; e < TQ * din0; e += kThreads) {
        const int r = e / din0, c = e - r * din0;
        const int q = q0 + r;
        H[0][r * S + c] = (q < a.nq) ? a.x[(size_t)q * a.ldx + c] : 0.0f;
    }
    __syncthreads();

    int cur = 0;
    for (int l = 0; l < a.n_layers; ++l) {
        const int din = a.dims[l], dout = a.dims[l + 1];
        const float* __restrict__ W = a.W[l];
        const float* __restrict__ bias = a.b[l];
        const float* hin = H[cur] + ql * S;
        float* hout = H[cur ^ 1] + ql * S;
        const bool relu = (l + 1 < a.n_layers);
        for (int o0 = grp * kOB; o0 < dout; o0 += NG * kOB) {
            float acc[kOB];
            const float* wr[kOB];
#pragma unroll
            for (int j = 0; j < kOB; ++j) {
                const int o = min(o0 + j, dout - 1);
                acc[j] = bias[o];
                wr[j] = W + (size_t)o * din;
            }
            for (int i = 0; i < din; ++i) {
                const float h = hin[i];
#pragma unroll
                for (int j = 0; j < kOB; ++j) acc[j] = fmaf(h, wr[j][i], acc[j]);
            }
#pragma unroll
            for (int j = 0; j < kOB; ++j) {
                if (o0 + j < dout) hout[o0 + j] = relu ? fmaxf(acc[j], 0.0f) : acc[j];
            }
        }
        __syncthreads();
        cur ^= 1;
    }

    const int C = a.dims[a.n_layers];
    const float* logit = H[cur];

    if (a.mode == LMI_ROUTER_ARGMAX) {
        if (tid < TQ && q0 + tid < a.nq) {
            const float* lr = logit + tid * S;
            float best = lr[0];
            int bi = 0;
            for (int i = 1; i < C; ++i)
                if (lr[i] > best) { best = lr[i]; bi = i; }
            a.classes[q0 + tid] = bi;
        }
        return;
    }

    // softmax statistics (torch: exp(x - max) / sum)
    if (tid < TQ) {
        const float* lr = logit + tid * S;
        float m = lr[0];
        for (int i = 1; i < C; ++i) m = fmaxf(m, lr[i]);
        float s = 0.0f;
        for (int i = 0; i < C; ++i) s += expf(lr[i] - m);
        stat[2 * tid] = m;
        stat[2 * tid + 1] = s;
    }
    __syncthreads();

    const int R = a.R;
    if (R <= 8) {
        // R selection passes, one lane per query.
        if (tid < TQ && q0 + tid < a.nq) {
            const float* lr = logit + tid * S;
            const float m = stat[2 * tid], s = stat[2 * tid + 1];
            float pl = __builtin_inff();
            int pi = -1;
            for (int r = 0; r < R; ++r) {
                float bl = -__builtin_inff();
                int bi = -1;
                for (int i = 0; i < C; ++i) {
                    const float v = lr[i];
                    // strictly after the previous pick in (desc logit, asc index) order
                    const bool after = better(pl, pi, v, i);
                    if (after && (bi < 0 || better(v, i, bl, bi))) { bl = v; bi = i; }
                }
                const size_t o = (size_t)(q0 + tid) * R + r;
                a.classes[o] = bi;
                if (a.probs) a.probs[o] = expf(bl - m) / s;
                pl = bl;
                pi = bi;
            }
        }
    } else {
        // Rank of every class: its position in (desc logit, asc index) order.
        for (int e = tid; e < TQ * C; e += kThreads) {
            const int qq = e % TQ, j = e / TQ;
            if (q0 + qq >= a.nq) continue;
            const float* lr = logit + qq * S;
            const float v = lr[j];
            int rank = 0;
            for (int i = 0; i < C; ++i) rank += better(lr[i], i, v, j) ? 1 : 0;
            if (rank < R) {
                const size_t o = (size_t)(q0 + qq) * R + rank;
                a.classes[o] = j;
                if (a.probs) a.probs[o] = expf(v - stat[2 * qq]) / stat[2 * qq + 1];
            }
        }
    }
}

template <int TQ>
int launch_router(const RouterArgs& a, size_t lds, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        LMI_HIP_TRY(hipFuncSetAttribute((const void*)router_kernel<TQ>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr_set = true;
    }
    const int grid = (a.nq + TQ - 1) / TQ;
    hipLaunchKernelGGL(router_kernel<TQ>, dim3(grid), dim3(kThreads), lds, s, a);
    LMI_LAUNCH_CHECK("router_kernel");
    return LMI_OK;
}

}  // namespace
}  // namespace lmi

extern "C" int lmi_router(const float* x, int32_t nq, int32_t ldx, const lmi_mlp_desc* mlp,
                          int32_t R, int32_t mode, int32_t* classes_out, float* probs_out,
                          void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(mlp != nullptr && x != nullptr && classes_out != nullptr, "null pointer");
    LMI_CHECK_ARG(nq >= 0, "nq < 0");
    LMI_CHECK_ARG(mlp->n_layers >= 1 && mlp->n_layers <= LMI_MAX_LAYERS, "n_layers out of range");
    LMI_CHECK_ARG(ldx >= mlp->dims[0], "ldx < input width");
    LMI_CHECK_ARG(mode == LMI_ROUTER_TOPR || mode == LMI_ROUTER_ARGMAX, "bad mode");
    const int C = mlp->dims[mlp->n_layers];
    LMI_CHECK_ARG(C >= 1, "no classes");
    if (mode == LMI_ROUTER_ARGMAX) LMI_CHECK_ARG(R == 1, "ARGMAX needs R == 1");
    LMI_CHECK_ARG(R >= 1 && R <= C, "R out of range");
    if (nq == 0) return LMI_OK;

    RouterArgs a{};
    a.x = x;
    a.nq = nq;
    a.ldx = ldx;
    a.n_layers = mlp->n_layers;
    int maxdim = 0;
    for (int l = 0; l <= mlp->n_layers; ++l) {
        LMI_CHECK_ARG(mlp->dims[l] >= 1, "dims[%d] < 1", l);
        a.dims[l] = mlp->dims[l];
        maxdim = maxdim > mlp->dims[l] ? maxdim : mlp->dims[l];
    }
    for (int l = 0; l < mlp->n_layers; ++l) {
        LMI_CHECK_ARG(mlp->W[l] && mlp->b[l], "null weight of layer %d", l);
        a.W[l] = mlp->W[l];
        a.b[l] = mlp->b[l];
    }
    // stride = maxdim rounded up to a multiple of 4, plus 1: odd => lanes that
    // read the same column of different rows hit different banks.
    a.stride = ((maxdim + 3) / 4) * 4 + 1;
    a.R = R;
    a.mode = mode;
    a.classes = classes_out;
    a.probs = probs_out;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t lds_limit = 160 * 1024;
    for (int tq : {64, 32, 16, 8}) {
        const size_t lds = (size_t)(2 * tq * a.stride + 2 * tq) * sizeof(float);
        if (lds > lds_limit) continue;
        switch (tq) {
            case 64: return launch_router<64>(a, lds, s);
            case 32: return launch_router<32>(a, lds, s);
            case 16: return launch_router<16>(a, lds, s);
            default: return launch_router<8>(a, lds, s);
        }
    }
    set_error("router layer width %d too large for LDS", maxdim);
    return LMI_E_UNSUPPORTED;
}
