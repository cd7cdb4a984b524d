// K1 — router inference (MLP bucket classifier) on gfx950.
//
// Replaces NeuralNetwork.predict_proba (reference search/li/model.py:214-229:
// Linear/ReLU stack, softmax(dim=1), topk over all classes) and
// NeuralNetwork.predict (model.py:201-212: argmax of the logits, used for the
// object labels at LearnedIndex.py:240).
//
// One workgroup (4 waves) owns a tile of TQ query rows.  The activations of
// the tile live in LDS (two ping-pong buffers, one row per query, rows 16-B
// aligned at a pitch of 4 mod 64 floats so per-lane float4 reads are
// conflict-free); every lane owns one query and kOB output neurons.  A layer is
// computed in passes of NG * kOB outputs whose weight rows are first staged in
// LDS (one coalesced copy per pass, shared by the whole tile) and then read as
// broadcasts.  Each output is the fp32 FMA chain b[o] + sum_i h[i] * W[o][i] in
// ascending i, i.e. torch's Linear up to summation order.  The last layer's
// logits stay in LDS and are reduced to the top-R classes (descending logit,
// ties to the lower class index) and their softmax probabilities, or to the
// argmax.
#include "lmi_common.hpp"

#include <mutex>

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
    int32_t w_vec4;  // every weight matrix 16-B aligned with din % 4 == 0 rows
    int32_t wpitch;  // LDS pitch of a staged weight row, floats
    int32_t R, mode;
    int32_t* classes;
    float* probs;
};

constexpr int kThreads = 256;
constexpr int kOB = 8;  // outputs per lane per pass (register blocking)

// (logit a, class ia) ranks before (logit b, class ib)?
__device__ inline bool better(float a, int ia, float b, int ib) {
    return a > b || (a == b && ia < ib);
}

extern "C" __device__ uint64_t __ockl_wfred_min_u64(uint64_t);
extern "C" __device__ float __ockl_wfred_max_f32(float);
extern "C" __device__ float __ockl_wfred_add_f32(float);

// wave-wide best (logit, class) under `better`: a DPP minimum of the u64 key
// (~ordered(logit) << 32 | class), i.e. descending logit, then ascending
// class; every lane gets the winner
__device__ inline void wave_best(float& v, int& i) {
    const uint32_t bits = v == 0.0f ? 0u : __float_as_uint(v);  // -0 ties with +0, as in `better`
    const uint32_t asc = (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
    const uint64_t key = __ockl_wfred_min_u64(((uint64_t)~asc << 32) | (uint32_t)i);
    const uint32_t wa = ~(uint32_t)(key >> 32);
    v = __uint_as_float((wa & 0x80000000u) ? (wa ^ 0x80000000u) : ~wa);
    i = (int)(uint32_t)key;
}

// The last layer's logits of TQ queries (LDS, row pitch S) -> a.classes
// (and a.probs): argmax, or the top-R picks with their softmax probabilities.
// One wave per query: the picks compare logits exactly, so they do not depend
// on the reduction order; only the softmax sum's rounding does.  `stat` is
// 2*TQ floats of LDS.
template <int TQ, int NT>
__device__ inline void select_classes(const RouterArgs& a, const float* logit, int S, int q0,
                                      float* stat) {
    const int C = a.dims[a.n_layers];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    constexpr int NW = NT / 64;
    if (a.mode == LMI_ROUTER_ARGMAX) {
        for (int qq = wave; qq < TQ && q0 + qq < a.nq; qq += NW) {
            const float* lr = logit + qq * S;
            float bv = -__builtin_inff();
            int bi = INT32_MAX;
            for (int i = lane; i < C; i += 64) {
                const float v = lr[i];
                if (better(v, i, bv, bi)) { bv = v; bi = i; }
            }
            wave_best(bv, bi);
            if (lane == 0) a.classes[q0 + qq] = bi;
        }
        return;
    }

    // softmax statistics (torch: exp(x - max) / sum)
    for (int qq = wave; qq < TQ; qq += NW) {
        const float* lr = logit + qq * S;
        float m = -__builtin_inff();
        for (int i = lane; i < C; i += 64) m = fmaxf(m, lr[i]);
        m = __ockl_wfred_max_f32(m);
        float sum = 0.0f;
        for (int i = lane; i < C; i += 64) sum += expf(lr[i] - m);
        sum = __ockl_wfred_add_f32(sum);
        if (lane == 0) {
            stat[2 * qq] = m;
            stat[2 * qq + 1] = sum;
        }
    }
    __syncthreads();

    const int R = a.R;
    if (R <= 8) {
        // R selection rounds per query, each a wave-wide best over the
        // classes strictly after the previous pick in (desc logit, asc index)
        for (int qq = wave; qq < TQ && q0 + qq < a.nq; qq += NW) {
            const float* lr = logit + qq * S;
            const float m = stat[2 * qq], sum = stat[2 * qq + 1];
            float pl = __builtin_inff();
            int pi = -1;
            for (int r = 0; r < R; ++r) {
                float bl = -__builtin_inff();
                int bi = INT32_MAX;
                for (int i = lane; i < C; i += 64) {
                    const float v = lr[i];
                    if (better(pl, pi, v, i) && better(v, i, bl, bi)) { bl = v; bi = i; }
                }
                wave_best(bl, bi);
                if (lane == 0) {
                    const size_t o = (size_t)(q0 + qq) * R + r;
                    a.classes[o] = bi;
                    if (a.probs) a.probs[o] = expf(bl - m) / sum;
                }
                pl = bl;
                pi = bi;
            }
        }
    } else {
        // Rank of every class: its position in (desc logit, asc index) order.
        for (int e = tid; e < TQ * C; e += NT) {
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
__global__ __launch_bounds__(kThreads) void router_kernel(RouterArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int G = 64 / TQ;    // query groups per wave
    constexpr int NG = 4 * G;     // output groups per workgroup
    const int S = a.stride;
    const int WP = a.wpitch;                    // staged weight row pitch (floats)
    float* wt = smem + 2 * TQ * S;              // [NG * kOB][WP] weights of one pass
    float* stat = wt + NG * kOB * WP;           // [TQ][2]: max, sum

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int ql = lane % TQ;
    const int grp = wave * G + lane / TQ;
    const int q0 = blockIdx.x * TQ;

    // Stage the query tile.
    const int din0 = a.dims[0];
    {
        constexpr int kU = 8;
        for (int e0 = tid; e0 < TQ * din0; e0 += kU * kThreads) {
            float v[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int e = e0 + u * kThreads;
                const int r = e / din0, c = e - r * din0;
                v[u] = (e < TQ * din0 && q0 + r < a.nq) ? a.x[(size_t)(q0 + r) * a.ldx + c] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int e = e0 + u * kThreads;
                if (e < TQ * din0) smem[(e / din0) * S + e % din0] = v[u];
            }
        }
    }
    __syncthreads();

    int cur = 0;
    for (int l = 0; l < a.n_layers; ++l) {
        const int din = a.dims[l], dout = a.dims[l + 1];
        const float* __restrict__ W = a.W[l];
        const float* __restrict__ bias = a.b[l];
        // (LDS pointers computed from smem directly: through an array of
        // pointers the compiler loses the address space and emits flat loads)
        const float* hin = smem + cur * TQ * S + ql * S;
        float* hout = smem + (cur ^ 1) * TQ * S + ql * S;
        const bool relu = (l + 1 < a.n_layers);
        const int din4 = din & ~3;
        for (int ob = 0; ob < dout; ob += NG * kOB) {
            // stage rows ob .. ob + NG*kOB - 1 (clamped) of W: contiguous in HBM
            const int nrow = min(NG * kOB, dout - ob);
            __syncthreads();  // the previous pass's readers are done with wt
            if (a.w_vec4) {
                // all of a thread's loads in flight before its LDS stores (a
                // load-store loop would pay one L2 round trip per element)
                constexpr int kU = 8;
                const int n4 = din >> 2, tot = nrow * n4;
                const float4* src = reinterpret_cast<const float4*>(W + (size_t)ob * din);
                for (int e0 = tid; e0 < tot; e0 += kU * kThreads) {
                    float4 v[kU];
#pragma unroll
                    for (int u = 0; u < kU; ++u) {
                        const int e = e0 + u * kThreads;
                        if (e < tot) v[u] = src[e];
                    }
#pragma unroll
                    for (int u = 0; u < kU; ++u) {
                        const int e = e0 + u * kThreads;
                        if (e < tot) {
                            const int r = e / n4, c4 = e - r * n4;
                            *reinterpret_cast<float4*>(wt + r * WP + 4 * c4) = v[u];
                        }
                    }
                }
            } else {
                for (int e = tid; e < nrow * din; e += kThreads) {
                    const int r = e / din, c = e - r * din;
                    wt[r * WP + c] = W[(size_t)ob * din + e];
                }
            }
            __syncthreads();
            float acc[kOB];
            const float* wr[kOB];
#pragma unroll
            for (int j = 0; j < kOB; ++j) {
                const int r = min(grp * kOB + j, nrow - 1);
                acc[j] = bias[ob + r];
                wr[j] = wt + r * WP;
            }
            // ascending i, one fmaf per term: the same chain as a scalar loop
            int i = 0;
#pragma unroll 2
            for (; i < din4; i += 4) {
                const float4 h4 = *reinterpret_cast<const float4*>(hin + i);
#pragma unroll
                for (int j = 0; j < kOB; ++j) {
                    const float4 w4 = *reinterpret_cast<const float4*>(wr[j] + i);
                    acc[j] = fmaf(h4.x, w4.x, acc[j]);
                    acc[j] = fmaf(h4.y, w4.y, acc[j]);
                    acc[j] = fmaf(h4.z, w4.z, acc[j]);
                    acc[j] = fmaf(h4.w, w4.w, acc[j]);
                }
            }
            for (; i < din; ++i) {
                const float h = hin[i];
#pragma unroll
                for (int j = 0; j < kOB; ++j) acc[j] = fmaf(h, wr[j][i], acc[j]);
            }
#pragma unroll
            for (int j = 0; j < kOB; ++j) {
                const int o = ob + grp * kOB + j;
                if (o < dout) hout[o] = relu ? fmaxf(acc[j], 0.0f) : acc[j];
            }
        }
        __syncthreads();
        cur ^= 1;
    }

    const float* logit = smem + cur * TQ * S;
    select_classes<TQ, kThreads>(a, logit, S, q0, stat);
}

// MFMA form of the same router (every layer's width a multiple of 16, weight
// rows 16-B aligned): one wave owns 16 queries; a layer is a chain of
// v_mfma_f32_16x16x4_f32 over 16-output tiles (A = weight rows, straight from
// L2 — every wave of the grid reads the same 28-74K weights — B = the wave's
// activations in LDS, D = [16 outputs][16 queries]).  Products and sums are
// fp32 as in torch's Linear; only the summation order differs (the input
// index k is split into four contiguous quarters, one per lane group, so each
// lane's operands are float4 runs).  The accumulators start at the bias; ReLU
// between layers; the logits go through select_classes like router_kernel's.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kMQ = 16;  // queries per wave (the N side of the MFMA)
constexpr int kMW = 4;   // waves per workgroup: they split every layer's output tiles
constexpr int kMT = 4;   // 16-output tiles per wave and pass (4 x 4 accumulator VGPRs)
constexpr int kKB = 32;  // k-quarter block whose A operands are loaded at once (kMT x 32 VGPRs)

// Sorted (desc logit, asc class) top list of kRT entries per lane; `better`
// order, so lists built from the same items are identical in every lane.
constexpr int kRT = 8;
__device__ inline void top_insert(float (&bl)[kRT], int (&bi)[kRT], float v, int i) {
    if (!better(v, i, bl[kRT - 1], bi[kRT - 1])) return;
#pragma unroll
    for (int j = kRT - 1; j > 0; --j) {
        // shift entry j-1 down if v ranks before it, else v lands at j
        const bool sh = better(v, i, bl[j - 1], bi[j - 1]);
        const bool here = !sh && better(v, i, bl[j], bi[j]);
        const float nv = sh ? bl[j - 1] : (here ? v : bl[j]);
        const int ni = sh ? bi[j - 1] : (here ? i : bi[j]);
        bl[j] = nv;
        bi[j] = ni;
    }
    if (better(v, i, bl[0], bi[0])) { bl[0] = v; bi[0] = i; }
}

template <int NQG>
__global__ __launch_bounds__(256) void router_mfma_kernel(RouterArgs a) {
    constexpr int QW = kMQ * NQG;  // queries of the workgroup: NQG groups of 16
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int S = a.stride;
    float* stat = smem + 2 * QW * S;
    const int lane = threadIdx.x & 63;
    const int ql = lane & 15;   // query column of the tile (B / D)
    const int g = lane >> 4;    // k quarter (A / B) and output row group (D)
    const int q0 = blockIdx.x * QW;

    // stage the 16 query rows: all of a lane's loads in flight before its stores
    const int din0 = a.dims[0];
    {
        constexpr int kU = 8;
        for (int e0 = threadIdx.x; e0 < QW * din0; e0 += kU * 64 * kMW) {
            float v[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int e = e0 + u * 64 * kMW;
                const int r = e / din0, c = e - r * din0;
                v[u] = (e < QW * din0 && q0 + r < a.nq) ? a.x[(size_t)(q0 + r) * a.ldx + c] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int e = e0 + u * 64 * kMW;
                if (e < QW * din0) smem[(e / din0) * S + e % din0] = v[u];
            }
        }
    }
    __syncthreads();

    int cur = 0;
    const int wave = threadIdx.x >> 6;
    for (int l = 0; l < a.n_layers; ++l) {
        const int din = a.dims[l], dout = a.dims[l + 1];
        const int kq = din >> 2;  // k quarter length (a multiple of 4)
        const int ntile = (dout + 15) >> 4;
        const float* __restrict__ W = a.W[l];
        const float* __restrict__ bias = a.b[l];
        const float* hin = smem + cur * QW * S + ql * S + g * kq;   // + 16*S per query group
        float* hout = smem + (cur ^ 1) * QW * S + ql * S;
        const bool relu = (l + 1 < a.n_layers);
        // wave w owns the output tiles t = w (mod kMW): kMT of them per pass
        for (int tb = wave; tb < ntile; tb += kMW * kMT) {
            f32x4 acc[kMT][NQG];
            const float* wr[kMT];
            bool live[kMT];
#pragma unroll
            for (int j = 0; j < kMT; ++j) {
                const int t = tb + kMW * j;
                live[j] = t < ntile;
                const int orow = 16 * t + ql;  // A row of this lane
                wr[j] = W + (size_t)min(orow, dout - 1) * din + g * kq;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int o = 16 * t + 4 * g + v;  // D row of this lane
                    const float b0 = (live[j] && o < dout) ? bias[o] : 0.0f;
#pragma unroll
                    for (int qg = 0; qg < NQG; ++qg) acc[j][qg][v] = b0;
                }
            }
            // k in blocks of kKB: every A load of a block in flight at once
            for (int kb = 0; kb < kq; kb += kKB) {
                float4 a4[kMT][kKB / 4];
#pragma unroll
                for (int j = 0; j < kMT; ++j)
#pragma unroll
                    for (int u = 0; u < kKB / 4; ++u)
                        a4[j][u] = (live[j] && kb + 4 * u < kq)
                                       ? *reinterpret_cast<const float4*>(wr[j] + kb + 4 * u)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int u = 0; u < kKB / 4; ++u) {
                    if (kb + 4 * u < kq) {
#pragma unroll
                        for (int qg = 0; qg < NQG; ++qg) {
                            const float4 b4 =
                                *reinterpret_cast<const float4*>(hin + qg * kMQ * S + kb + 4 * u);
#pragma unroll
                            for (int j = 0; j < kMT; ++j) {
                                if (live[j]) {
                                    f32x4 c = acc[j][qg];
                                    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j][u].x, b4.x, c, 0, 0, 0);
                                    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j][u].y, b4.y, c, 0, 0, 0);
                                    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j][u].z, b4.z, c, 0, 0, 0);
                                    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j][u].w, b4.w, c, 0, 0, 0);
                                    acc[j][qg] = c;
                                }
                            }
                        }
                    }
                }
            }
            // rows of A past dout read row dout-1 (in bounds); their D rows
            // land in the LDS row's padding and are never read
#pragma unroll
            for (int j = 0; j < kMT; ++j) {
                if (live[j]) {
#pragma unroll
                    for (int qg = 0; qg < NQG; ++qg) {
                        const f32x4 c = acc[j][qg];
                        float4 o4;
                        o4.x = relu ? fmaxf(c[0], 0.0f) : c[0];
                        o4.y = relu ? fmaxf(c[1], 0.0f) : c[1];
                        o4.z = relu ? fmaxf(c[2], 0.0f) : c[2];
                        o4.w = relu ? fmaxf(c[3], 0.0f) : c[3];
                        *reinterpret_cast<float4*>(hout + qg * kMQ * S + 16 * (tb + kMW * j) + 4 * g) = o4;
                    }
                }
            }
        }
        __syncthreads();
        cur ^= 1;
    }
    const float* logit = smem + cur * QW * S;
    if (a.R > kRT) {
        select_classes<QW, 64 * kMW>(a, logit, S, q0, stat);
        return;
    }
    if (wave >= NQG) return;  // the selection below: wave w, query group w
    // four lanes per query (lanes ql, ql+16, ql+32, ql+48), each over the
    // classes i = g (mod 4): a private top list, then two xor exchanges
    const int C = a.dims[a.n_layers];
    const int qi = q0 + wave * kMQ + ql;
    const float* lr = logit + (wave * kMQ + ql) * S;
    float bl[kRT];
    int bi[kRT];
#pragma unroll
    for (int j = 0; j < kRT; ++j) { bl[j] = -__builtin_inff(); bi[j] = INT32_MAX; }
    for (int i = g; i < C; i += 4) top_insert(bl, bi, lr[i], i);
#pragma unroll
    for (int x = 16; x <= 32; x <<= 1) {
        float pv[kRT];
        int pix[kRT];
#pragma unroll
        for (int j = 0; j < kRT; ++j) {
            pv[j] = __shfl_xor(bl[j], x);
            pix[j] = __shfl_xor(bi[j], x);
        }
#pragma unroll
        for (int j = 0; j < kRT; ++j) top_insert(bl, bi, pv[j], pix[j]);
    }
    if (qi >= a.nq) return;
    if (a.mode == LMI_ROUTER_ARGMAX) {
        if (g == 0) a.classes[qi] = bi[0];
        return;
    }
    // softmax (torch: exp(x - max) / sum); the max is the first pick
    const float m = bl[0];
    float sum = 0.0f;
    for (int i = g; i < C; i += 4) sum += expf(lr[i] - m);
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    if (g == 0) {
        const int R = a.R;
#pragma unroll
        for (int r = 0; r < kRT; ++r) {
            if (r < R) {
                const size_t o = (size_t)qi * R + r;
                a.classes[o] = bi[r];
                if (a.probs) a.probs[o] = expf(bl[r] - m) / sum;
            }
        }
    }
}

int router_qg_or(int dflt) {
    const int x = env_config().router_qg;
    return (x == 1 || x == 2 || x == 4) ? x : dflt;
}

template <int TQ>
int launch_router(const RouterArgs& a, size_t lds, hipStream_t s) {
    // the attribute is the kernel's maximum (160 KiB), set once per process
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [] {
        attr_err = hipFuncSetAttribute((const void*)router_kernel<TQ>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    });
    LMI_HIP_TRY(attr_err);
    (void)lds;
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
    // stride = maxdim rounded up to a multiple of 64, plus 4: 16-B aligned
    // rows whose float4 reads by 16 lanes cover all 64 banks once
    a.stride = ((maxdim + 63) / 64) * 64 + 4;
    a.w_vec4 = 1;
    for (int l = 0; l < mlp->n_layers; ++l)
        if ((mlp->dims[l] & 3) || ((uintptr_t)mlp->W[l] & 15)) a.w_vec4 = 0;
    a.R = R;
    a.mode = mode;
    a.classes = classes_out;
    a.probs = probs_out;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // MFMA path: hidden and input widths multiples of 16 (k quarters of
    // float4 runs), 16-B aligned weights; the classes may be any width
    bool mfma = a.w_vec4 && !env_config().router_fma;
    for (int l = 0; l < mlp->n_layers; ++l)
        if (mlp->dims[l] % 16) mfma = false;
    if (mfma) {
        const int sm = ((maxdim + 15) / 16) * 16 + 4;  // room for the last tile's padding rows
        // 64 queries per workgroup (every weight load feeds 4 query groups)
        // when the grid still covers the CUs; else 32 or 16
        int nqg = router_qg_or(nq >= 64 * 128 ? 4 : nq >= 32 * 128 ? 2 : 1);
        for (; nqg >= 1; nqg >>= 1) {
            const size_t lds = (size_t)(2 * kMQ * nqg * sm + 2 * kMQ * nqg) * sizeof(float);
            if (lds > 160 * 1024) continue;
            const void* fn = nqg == 4 ? (const void*)router_mfma_kernel<4>
                           : nqg == 2 ? (const void*)router_mfma_kernel<2>
                                      : (const void*)router_mfma_kernel<1>;
            static std::once_flag once[3];
            static hipError_t attr_err[3] = {hipSuccess, hipSuccess, hipSuccess};
            const int ai = nqg == 4 ? 2 : nqg - 1;
            std::call_once(once[ai], [&] {
                attr_err[ai] = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   160 * 1024);
            });
            LMI_HIP_TRY(attr_err[ai]);
            RouterArgs m = a;
            m.stride = sm;
            const dim3 grid((nq + kMQ * nqg - 1) / (kMQ * nqg));
            if (nqg == 4)
                hipLaunchKernelGGL(router_mfma_kernel<4>, grid, dim3(64 * kMW), lds, s, m);
            else if (nqg == 2)
                hipLaunchKernelGGL(router_mfma_kernel<2>, grid, dim3(64 * kMW), lds, s, m);
            else
                hipLaunchKernelGGL(router_mfma_kernel<1>, grid, dim3(64 * kMW), lds, s, m);
            LMI_LAUNCH_CHECK("router_mfma_kernel");
            return LMI_OK;
        }
    }
    a.wpitch = ((maxdim + 3) / 4) * 4 + 4;  // two rows read together sit 4 banks apart
    const size_t lds_limit = 160 * 1024;
    for (int tq : {32, 16, 8}) {
        const int ng = 4 * (64 / tq);
        const size_t lds =
            (size_t)(2 * tq * a.stride + ng * kOB * a.wpitch + 2 * tq) * sizeof(float);
        if (lds > lds_limit) continue;
        switch (tq) {
            case 32: return launch_router<32>(a, lds, s);
            case 16: return launch_router<16>(a, lds, s);
            default: return launch_router<8>(a, lds, s);
        }
    }
    set_error("router layer width %d too large for LDS", maxdim);
    return LMI_E_UNSUPPORTED;
}
