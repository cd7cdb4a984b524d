// K2 scan kernels v1 and v2 (gfx950), split from lmi_scan.hip.
//
// scan v3 (lmi_scan.hip) serves the fp16 / d_pad == 768 search path; these
// two remain for what v3 does not take and as measured A/B baselines:
//   scan_kernel  (v1, round 1)  any d_pad <= the LDS budget, fp16 or fp32
//                corpus, fp16-math or fp32-math queries, the LO (replay
//                lower-bound) variant; queries staged in LDS, rows streamed
//                from HBM straight into MFMA A fragments
//   scan2_kernel (v2, round 2)  fp16 / d_pad == 768, queries in registers,
//                rows through an LDS-DMA ring (LMI_SCAN_V=2)
// Both replace the same reference code as v3 (see lmi_scan.hip's header).
#include "lmi_scan_internal.hpp"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <utility>

namespace lmi {
namespace {

// ---------------------------------------------------------------------------
// scan
// ---------------------------------------------------------------------------
template <int KL, bool F16MATH>
struct ScanCfg {
    static constexpr int QB = F16MATH ? 64 : 32;  // queries per tile
    static constexpr int NQF = QB / 32;            // 32-query MFMA fragments per wave
    static constexpr int QPAD = F16MATH ? 8 : 4;   // LDS row pad (elements): 16 B
    using QT = typename std::conditional<F16MATH, _Float16, float>::type;
};

template <int KL, bool F16MATH>
size_t scan_lds_bytes(int d_pad) {
    using Cfg = ScanCfg<KL, F16MATH>;
    const size_t qs = (size_t)Cfg::QB * (d_pad + Cfg::QPAD) * sizeof(typename Cfg::QT);
    const size_t merge = (size_t)Cfg::QB * 2 * kWaves * KL * sizeof(uint64_t);
    const size_t queue = (size_t)kWaves * kQCap * 64 * sizeof(uint64_t);
    return std::max(qs, merge) + queue + Cfg::QB * (sizeof(uint64_t) + sizeof(float)) + 16;
}

// The epilogue of one 32x32 accumulator tile: lane holds query column
// (lane & 31) and rows (reg&3) + 8*(reg>>2) + 4*(lane>>5), reg = 0..15
// (C/D layout of the 32x32 MFMAs, dtype-independent on gfx950).
// Lower-bound test of the k > 16 passes (lmi_bucket_topk with k > 16): keep
// only objects after (distance, global position) `lo` of their pair, i.e. the
// next entries of the (d, position) order; lo = 0 keeps everything.
__device__ inline bool above_lo(float d, uint64_t lo, const int32_t* __restrict__ gpos,
                                uint32_t row) {
    const uint32_t o = f2ord(d), hi = (uint32_t)(lo >> 32);
    return o > hi || (o == hi && (uint32_t)gpos[row] > (uint32_t)lo);
}

template <int KL, bool LO = false>
__device__ inline void tile_epilogue(const f32x16& acc, uint64_t (&L)[KL], uint64_t* thr_slot,
                                     float invq, const float* __restrict__ inv_norm,
                                     uint32_t row_base, int valid_rows, uint64_t* queue,
                                     int lane, uint64_t lo = 0,
                                     const int32_t* __restrict__ gpos = nullptr) {
    const int h = lane >> 5;
    uint64_t thr = *thr_slot;
    float bound = key_dist_bound(thr);
    int cnt = 0;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int i = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const bool valid = i < valid_rows;
        const float inv = valid ? inv_norm[row_base + i] : 0.0f;
        const float d = fmaf(-acc[reg], invq * inv, 1.0f);
        if (valid && d <= bound && (!LO || above_lo(d, lo, gpos, row_base + (uint32_t)i))) {
            const uint64_t key = make_key(d, row_base + (uint32_t)i);
            if (key < thr) {
                queue[cnt * 64] = key;
                ++cnt;
            }
        }
    }
    for (int i = 0; __any(i < cnt); ++i) {
        if (i < cnt) {
            const uint64_t key = queue[i * 64];
            if (key < L[KL - 1]) list_insert<KL>(L, key);
        }
    }
    // publish this partial list's k-th key; the query's bound is the min
    // over its partial lists (the union's k-th is <= each partial k-th).
    if (L[KL - 1] < thr) atomicMin(reinterpret_cast<unsigned long long*>(thr_slot),
                                   (unsigned long long)L[KL - 1]);
}

template <int KL, bool F16MATH, typename TC, bool LO = false>
__global__ __launch_bounds__(kThreads, 1) void scan_kernel(ScanArgs a) {
    using Cfg = ScanCfg<KL, F16MATH>;
    using QT = typename Cfg::QT;
    constexpr int QB = Cfg::QB, NQF = Cfg::NQF;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int d_pad = a.d_pad;
    const int ldq = d_pad + Cfg::QPAD;
    const size_t qs_bytes = std::max((size_t)QB * ldq * sizeof(QT),
                                     (size_t)QB * 2 * kWaves * KL * sizeof(uint64_t));
    QT* Qs = reinterpret_cast<QT*>(smem);
    uint64_t* mergebuf = reinterpret_cast<uint64_t*>(smem);  // aliases Qs after the scan
    uint64_t* queue_all = reinterpret_cast<uint64_t*>(smem + qs_bytes);
    uint64_t* thr_s = queue_all + kWaves * kQCap * 64;
    float* invq_s = reinterpret_cast<float*>(thr_s + QB);
    // no static __shared__ in this kernel: it would shift the dynamic base
    // off 16-B alignment and every ds_read_b128 would replay (guide G17)
    int& s_tile = *reinterpret_cast<int*>(invq_s + QB);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int h = lane >> 5;
    const int col = lane & 31;
    uint64_t* queue = queue_all + wave * kQCap * 64 + lane;

    const TC* __restrict__ corpus = reinterpret_cast<const TC*>(a.corpus);
    const QT* __restrict__ qbuf = reinterpret_cast<const QT*>(a.qbuf);
    const int ntiles = a.meta[2 * kGroups];

    for (;;) {
        if (tid == 0) s_tile = atomicAdd(&a.work[kGroups], 1);
        __syncthreads();
        const int t = s_tile;
        if (t >= ntiles) break;
        const Tile tile = a.tiles[t];
        const int64_t bstart = a.bucket_off[tile.c];
        const int64_t bend = a.bucket_off[tile.c + 1];
        const int64_t row0 = bstart + (int64_t)tile.chunk * a.chunk_rows;
        const int nrows = (int)std::min<int64_t>(a.chunk_rows, bend - row0);

        // ---- stage the tile's queries (16 B per lane per step) ----------
        {
            constexpr int EPV = 16 / sizeof(QT);
            const int vpr = d_pad / EPV;
            for (int e = tid; e < QB * vpr; e += kThreads) {
                const int r = e / vpr, v = e - r * vpr;
                uint4 val = make_uint4(0, 0, 0, 0);
                if (r < tile.np) {
                    const int q = a.pair_q[tile.pp0 + r] / a.R;
                    val = *reinterpret_cast<const uint4*>(qbuf + (size_t)q * d_pad + v * EPV);
                }
                *reinterpret_cast<uint4*>(Qs + r * ldq + v * EPV) = val;
            }
            for (int r = tid; r < QB; r += kThreads) {
                const bool live = r < tile.np;
                invq_s[r] = live ? a.invq[a.pair_q[tile.pp0 + r] / a.R] : 0.0f;
                thr_s[r] = live ? kEmptyKey : 0ull;  // dead slots reject everything
            }
        }
        __syncthreads();

        uint64_t L[NQF][KL];
        uint64_t lo[NQF];
#pragma unroll
        for (int f = 0; f < NQF; ++f) {
            list_clear<KL>(L[f]);
            const int r = 32 * f + col;
            lo[f] = (LO && r < tile.np) ? (uint64_t)a.lo_g[a.pair_q[tile.pp0 + r]] : 0ull;
        }

        const int nsub = (nrows + 31) / 32;
        for (int st = wave; st < nsub; st += kWaves) {
            const int sub0 = st * 32;
            const int myrow = std::min(sub0 + col, nrows - 1);
            const TC* yrow = corpus + (size_t)(row0 + myrow) * d_pad;
            f32x16 acc[NQF];
#pragma unroll
            for (int f = 0; f < NQF; ++f)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[f][i] = 0.0f;

            if constexpr (F16MATH) {
                // 64-wide k block: lane half h covers k = kb + 32h + [0, 32);
                // MFMA step s (0..3), element j  <->  k = kb + 32h + 8s + j.
                // A and B use the same permutation of k, so the dot is exact.
                static_assert(sizeof(TC) == 2, "fp16 math needs an fp16 corpus");
                const half8* ysrc = reinterpret_cast<const half8*>(yrow) + 4 * h;
                half8 acur[4], anext[4];
#pragma unroll
                for (int s = 0; s < 4; ++s) acur[s] = ysrc[s];
                const int nkb = d_pad / 64;
                for (int kb = 0; kb < nkb; ++kb) {
                    if (kb + 1 < nkb) {
#pragma unroll
                        for (int s = 0; s < 4; ++s) anext[s] = ysrc[(kb + 1) * 8 + s];
                    }
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
#pragma unroll
                        for (int f = 0; f < NQF; ++f) {
                            const half8 b = *reinterpret_cast<const half8*>(
                                Qs + (32 * f + col) * ldq + kb * 64 + 32 * h + 8 * s);
                            acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(acur[s], b, acc[f], 0, 0, 0);
                        }
                    }
#pragma unroll
                    for (int s = 0; s < 4; ++s) acur[s] = anext[s];
                }
                // d_pad is a multiple of 32: a trailing 32-wide half block
                if (d_pad % 64) {
                    const int kb = nkb;
                    // only lane-half h covers k = kb*64 + 16h + [0,16) here
                    const half8* ys2 = reinterpret_cast<const half8*>(yrow + kb * 64) + 2 * h;
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const half8 av = ys2[s];
#pragma unroll
                        for (int f = 0; f < NQF; ++f) {
                            const half8 b = *reinterpret_cast<const half8*>(
                                Qs + (32 * f + col) * ldq + kb * 64 + 16 * h + 8 * s);
                            acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, b, acc[f], 0, 0, 0);
                        }
                    }
                }
            } else {
                // fp32 math, 32-wide k block: lane half h covers kb + 16h + [0,16);
                // group s (0..3) of 4 MFMAs 32x32x2, element j <-> k = kb + 16h + 4s + j.
                const int nkb = d_pad / 32;
                for (int kb = 0; kb < nkb; ++kb) {
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        f32x4 av;
                        if constexpr (sizeof(TC) == 2) {
                            const half4 hv = *reinterpret_cast<const half4*>(yrow + kb * 32 + 16 * h + 4 * s);
#pragma unroll
                            for (int j = 0; j < 4; ++j) av[j] = (float)hv[j];
                        } else {
                            av = *reinterpret_cast<const f32x4*>(yrow + kb * 32 + 16 * h + 4 * s);
                        }
#pragma unroll
                        for (int f = 0; f < NQF; ++f) {
                            const f32x4 b = *reinterpret_cast<const f32x4*>(
                                Qs + (32 * f + col) * ldq + kb * 32 + 16 * h + 4 * s);
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                acc[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], b[j], acc[f], 0, 0, 0);
                        }
                    }
                }
            }

            const uint32_t row_base = (uint32_t)(row0 + sub0);
            const int valid_rows = nrows - sub0;
#pragma unroll
            for (int f = 0; f < NQF; ++f) {
                const int qslot = 32 * f + col;
                tile_epilogue<KL, LO>(acc[f], L[f], &thr_s[qslot], invq_s[qslot], a.inv_norm,
                                      row_base, valid_rows, queue, lane, lo[f], a.gpos);
            }
        }
        __syncthreads();  // all waves done with Qs -> reuse as merge buffer

        // ---- merge the 2*kWaves partial lists of every query --------------
        // list index of (wave, half) = 2*wave + h; layout [qslot][list][KL]
#pragma unroll
        for (int f = 0; f < NQF; ++f) {
            uint64_t* dst = mergebuf + ((size_t)(32 * f + col) * (2 * kWaves) + 2 * wave + h) * KL;
#pragma unroll
            for (int i = 0; i < KL; ++i) dst[i] = L[f][i];
        }
        __syncthreads();
        if (tid < tile.np) {
            const uint64_t* src = mergebuf + (size_t)tid * (2 * kWaves) * KL;
            uint64_t M[KL];
#pragma unroll
            for (int i = 0; i < KL; ++i) M[i] = src[i];
            for (int l = 1; l < 2 * kWaves; ++l) {
                for (int i = 0; i < KL; ++i) {
                    const uint64_t key = src[l * KL + i];
                    if (key >= M[KL - 1]) break;
                    list_insert<KL>(M, key);
                }
            }
            uint64_t* out = a.partial + ((size_t)(tile.pp0 + tid) * a.max_chunks + tile.chunk) * KL;
#pragma unroll
            for (int i = 0; i < KL; ++i) out[i] = M[i];
        }
        __syncthreads();
    }
}

__device__ inline void vm_wait(int n_stages_after) {
    // wait until at most 5 * n of this wave's DMA pieces are outstanding
    switch (n_stages_after) {
        case 0: __builtin_amdgcn_s_waitcnt(waitcnt_vm(0)); break;
        case 1: __builtin_amdgcn_s_waitcnt(waitcnt_vm(5)); break;
        case 2: __builtin_amdgcn_s_waitcnt(waitcnt_vm(10)); break;
        case 3: __builtin_amdgcn_s_waitcnt(waitcnt_vm(15)); break;
        case 4: __builtin_amdgcn_s_waitcnt(waitcnt_vm(20)); break;
        default: __builtin_amdgcn_s_waitcnt(waitcnt_vm(25)); break;
    }
}

// MFMA with the B operand (query fragment) and the accumulator in AGPRs.
// hipcc pads no hazards inside asm: the chain needs none (the previous MFMA's
// D is this one's C), the first MFMA of a block takes C = 0 (no
// v_accvgpr_write -> MFMA hazard), and mfma_drain adds the 18 wait states a
// 16-pass MFMA result needs before a v_accvgpr_read (cdna4_isa §4.2).
__device__ __forceinline__ f32x16 mfma_first(const half8& a, const half8& b) {
    f32x16 d;
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&a"(d) : "v"(a), "a"(b));
    return d;
}
__device__ __forceinline__ f32x16 mfma_acc(const f32x16& c, const half8& a, const half8& b) {
    f32x16 d = c;
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "a"(b));
    return d;
}
__device__ __forceinline__ f32x16 mfma_drain(const f32x16& c) {
    f32x16 d = c;
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+a"(d));
    return d;
}


// Candidate filter of one accumulator register: d = 1 - dot/(|q||y|); rows
// past the chunk end become NaN so every compare rejects them.
__device__ __forceinline__ float cand_dist(float dot, float invq, float invy, int i, int valid_rows) {
    const float d = fmaf(-dot, invq * invy, 1.0f);
    return (i < valid_rows) ? d : __builtin_nanf("");
}

// Survivors of a block: appended to the lane's private LDS queue, then
// inserted into the lane's register list in lockstep (iterations = the
// largest per-lane count, not one per register).  The queue accesses are
// inline asm on purpose: hipcc drains every in-flight LDS-DMA (vmcnt(0))
// before an LDS write it cannot prove disjoint from the DMA targets, which
// would empty the ring; the queue never aliases the ring.  The same wave's
// LDS operations complete in order, and each read carries its own wait.
template <int KL>
__device__ __forceinline__ void insert_survivors(const float (&dv)[16], float bound, uint64_t thr,
                                                 uint32_t row_base, int h, uint32_t qaddr,
                                                 uint64_t (&L)[KL]) {
    int cnt = 0;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        if (dv[reg] <= bound) {
            const int i = (reg & 3) + 8 * (reg >> 2) + 4 * h;
            // dv <= bound (the distance part of a bound that may come from
            // another chunk, whose rows are ordered differently): no key test
            const uint64_t key = make_key(dv[reg], row_base + (uint32_t)i);
            lds_put_u64(qaddr + cnt * 512, key);
            ++cnt;
            (void)thr;
        }
    }
    for (int i = 0; __any(i < cnt); ++i) {
        if (i < cnt) {
            const uint64_t key = lds_get_u64(qaddr + i * 512);
            if (key < L[KL - 1]) list_insert<KL>(L, key);
        }
    }
}

// ABL (round-1 diagnostic variants, no longer instantiated): 1 = no top-k insertion,
// 2 = no MFMA / LDS reads (DMA + barriers only), 3 = no DMA (compute on
// whatever the ring holds); scan v3 also: 4 = no DMA, no insertion, 5 = no
// DMA, no epilogue, 6 = 5 without the per-stage barrier.  Results are wrong
// for ABL != 0: timing only.
template <int KL, int ABL = 0>
__global__ __launch_bounds__(kThreads, 1) void scan2_kernel(Scan2Args a) {
    using namespace v2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* ring = smem;
    // [wave][16][64] u64: the candidate queues, and after the ring loop the
    // buffer of the end-of-tile list merge
    uint64_t* merge_all = reinterpret_cast<uint64_t*>(smem + NSLOT * STAGE);
    int& s_tile = *reinterpret_cast<int*>(merge_all + kWaves * 64 * 16);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int col = lane & 31;
    const int ng = a.ng;
    const int gx = blockIdx.x & (ng - 1);

    // per-lane constant DMA offsets: this wave stages rows 8w..8w+7 of every
    // stage; lane writes LDS chunk `col` of row (8w + 2i + h) and reads the
    // source chunk col ^ (row & 15) (XOR swizzle applied on the source side)
    uint32_t voff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = 8 * wave + 2 * i + h;
        voff[i] = (uint32_t)(row * (D * 2) + ((col ^ (row & 15)) << 4));
    }
    const uint32_t voff_n = (uint32_t)(col * 4);
    // this lane's queue: entry e at qaddr + e * 512 (64 lanes x 8 B per entry)
    const uint32_t qaddr = (uint32_t)(uintptr_t)(merge_all + wave * 64 * 16 + lane);

    for (;;) {
        if (tid == 0) s_tile = dequeue_tile(a.meta, a.work, gx, ng);
        __syncthreads();
        const int t = s_tile;
        if (t < 0) break;
        const Tile tile = a.tiles[t];
        const int64_t bstart = a.bucket_off[tile.c];
        const int64_t row0 = bstart + (int64_t)tile.chunk * a.chunk_rows;
        const int nrows = __builtin_amdgcn_readfirstlane(
            (int)std::min<int64_t>(a.chunk_rows, a.bucket_off[tile.c + 1] - row0));
        const uint32_t r0lo = __builtin_amdgcn_readfirstlane((uint32_t)row0);
        const uint32_t r0hi = __builtin_amdgcn_readfirstlane((uint32_t)(row0 >> 32));
        const int64_t row0u = (int64_t)(((uint64_t)r0hi << 32) | r0lo);
        const int slot_q = 32 * wave + col;
        const bool live = slot_q < tile.np;
        const bool wave_live = 32 * wave < tile.np;
        const int pp = tile.pp0 + slot_q;

        // ---- this lane's query fragments (B operand, AGPRs), 1/||q||, bound --
        half8 qf[NQF];
        {
            const int q = live ? a.pair_q[pp] / a.R : 0;
            const half8* qrow = reinterpret_cast<const half8*>(a.qbuf + (size_t)q * D) + h;
            // (dead columns keep query 0's fragments here: zeroing them as
            // scan v3 does broke this kernel's KL = 16 lists on gfx950)
#pragma unroll
            for (int s = 0; s < NQF; ++s) qf[s] = qrow[2 * s];
        }
        // the query's bound: min over the k-th keys of its partial lists and of
        // the other chunks' tiles of the same pair; dead slots reject all
        uint64_t thr = live ? (uint64_t)a.thr_g[pp] : 0ull;
        const float my_invq = live ? a.invq[a.pair_q[pp] / a.R] : 0.0f;
        uint64_t L[KL];
        list_clear<KL>(L);
        // retire the fragment loads where hipcc can see it (see waitcnt_vm)
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
        __syncthreads();

        // buffer descriptors over this chunk (<= chunk_rows rows: far below the
        // 4 GiB record limit); the range check zero-fills rows past the end
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.corpus + row0u * D), (short)0, nrows * D * 2, 0x00020000);
        const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.inv_norm + row0u), (short)0, nrows * 4, 0x00020000);

        const int nblk = (nrows + 31) / 32;
        const int T = nblk * NST;
        // one DMA piece (i = 0..3: two rows x 512 B; i = 4: the 32 norms)
        auto dma = [&](int st, int i) {
            if (ABL == 3 || st >= T) return;
            const int blk = st / NST, j = st - blk * NST;
            unsigned char* sl = ring + (st % NSLOT) * STAGE;
            if (i < 4)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (lds_t)(sl + (8 * wave + 2 * i) * ROWB), 16, voff[i],
                    blk * (32 * D * 2) + j * ROWB, 0, 0);
            else
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rn, (lds_t)(sl + 32 * ROWB + wave * 256), 4,
                                                         voff_n, blk * 128, 0, 0);
        };

        const int pro = std::min(T, NSLOT - 1);
        for (int st = 0; st < pro; ++st)
            for (int i = 0; i < 5; ++i) dma(st, i);

        f32x16 acc, accp;
#pragma unroll
        for (int i = 0; i < 16; ++i) accp[i] = 0.0f;
        f32x4 nrmp[4] = {};
        uint32_t rbp = 0;   // row base of the pending block
        int vrp = 0;        // valid rows of the pending block (0: nothing pending)

        for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll
            for (int j = 0; j < NST; ++j) {
                const int s = blk * NST + j;
                // stage s must have landed; stages s+1 .. s+5 stay in flight
                const int issued = std::min(T - 1, s + NSLOT - 2);
                if (ABL != 3) vm_wait(issued - std::min(s + a.lag, issued));
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                const int nx = s + NSLOT - 1;  // stage whose DMA rides in this stage
                if (ABL == 2 || !wave_live) {
                    for (int i = 0; i < 5; ++i) dma(nx, i);
                    continue;
                }
                const unsigned char* rp = ring + (s % NSLOT) * STAGE + col * ROWB;
#define LMI_A(tt) (*reinterpret_cast<const half8*>(rp + (((2 * (tt) + h) ^ (col & 15)) << 4)))
                half8 af[16];
#pragma unroll
                for (int tt = 0; tt < 8; ++tt) af[tt] = LMI_A(tt);
                if (j == 0) {
                    // block start: the previous block's filter rides in the
                    // shadow of this block's first 16 MFMAs, with the DMA
                    float dv[16];
                    bool anyp = false;
                    const float bound = key_dist_bound(thr);
#pragma unroll
                    for (int tt = 0; tt < 16; ++tt) {
                        if (tt + 8 < 16) af[tt + 8] = LMI_A(tt + 8);
                        acc = (tt == 0) ? mfma_first(af[0], qf[0]) : mfma_acc(acc, af[tt], qf[tt]);
                        if (tt % 3 == 2) dma(nx, tt / 3);
                        const int reg = tt;
                        const int i = (reg & 3) + 8 * (reg >> 2) + 4 * h;
                        dv[reg] = cand_dist(accp[reg], my_invq, nrmp[reg >> 2][reg & 3], i, vrp);
                        anyp |= dv[reg] <= bound;
                    }
                    if (ABL != 1 && __any(anyp)) {
                        insert_survivors<KL>(dv, bound, thr, rbp, h, qaddr, L);
                        const uint64_t kth = L[KL - 1];
                        const uint64_t pk = partner_u64(kth, h);
                        thr = std::min(thr, std::min(kth, pk));
                    }
                } else {
#pragma unroll
                    for (int tt = 0; tt < 16; ++tt) {
                        if (tt + 8 < 16) af[tt + 8] = LMI_A(tt + 8);
                        acc = mfma_acc(acc, af[tt], qf[j * 16 + tt]);
                        if (tt % 3 == 2) dma(nx, tt / 3);
                    }
                }
#undef LMI_A
            }
            if (ABL != 2 && wave_live) {
                // park this block: its accumulator, norms, row range
                // wait states on the MFMA's own registers first: a copy taken
                // before them would read the accumulator mid-write
                acc = mfma_drain(acc);
                accp = acc;
                const int s = blk * NST + NST - 1;
                const float* nrm = reinterpret_cast<const float*>(ring + (s % NSLOT) * STAGE +
                                                                  32 * ROWB + wave * 256);
#pragma unroll
                for (int g = 0; g < 4; ++g) nrmp[g] = *reinterpret_cast<const f32x4*>(nrm + 8 * g + 4 * h);
                rbp = (uint32_t)(row0u + blk * 32);
                vrp = nrows - blk * 32;
            }
        }
        if (ABL == 0 && wave_live && vrp > 0) {
            // the last block's epilogue (nothing left to hide it behind)
            float dv[16];
            const float bound = key_dist_bound(thr);
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int i = (reg & 3) + 8 * (reg >> 2) + 4 * h;
                dv[reg] = cand_dist(accp[reg], my_invq, nrmp[reg >> 2][reg & 3], i, vrp);
            }
            insert_survivors<KL>(dv, bound, thr, rbp, h, qaddr, L);
        }
        __syncthreads();  // ring drained: every DMA was waited for above

        // ---- merge the two partial lists of each query (lanes col, col+32) ----
        uint64_t* mb = merge_all + (size_t)wave * 64 * KL;
#pragma unroll
        for (int i = 0; i < KL; ++i) mb[i * 64 + lane] = L[i];
        __syncthreads();
        if (h == 0 && live) {
#pragma unroll
            for (int i = 0; i < KL; ++i) {
                const uint64_t key = mb[i * 64 + lane + 32];
                if (key >= L[KL - 1]) break;
                list_insert<KL>(L, key);
            }
            uint64_t* out = a.partial + ((size_t)pp * a.max_chunks + tile.chunk) * KL;
#pragma unroll
            for (int i = 0; i < KL; ++i) out[i] = L[i];
            if (L[KL - 1] != kEmptyKey) atomicMin(&a.thr_g[pp], (unsigned long long)L[KL - 1]);
        }
        __syncthreads();
    }
}

}  // namespace

template <int KL, bool F16MATH, typename TC, bool LO>
int launch_scan(const ScanArgs& a, int d_pad, hipStream_t s) {
    const size_t lds = scan_lds_bytes<KL, F16MATH>(d_pad);
    if (lds > 160 * 1024) {
        set_error("d_pad=%d needs %zu B of LDS per workgroup", d_pad, lds);
        return LMI_E_UNSUPPORTED;
    }
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [] {
        attr_err = hipFuncSetAttribute((const void*)scan_kernel<KL, F16MATH, TC, LO>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    });
    LMI_HIP_TRY(attr_err);
    const bool timed = timing().on;
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (timed) {
        const int rc = timing_record(s, true, ev);
        if (rc != LMI_OK) return rc;
    }
    hipLaunchKernelGGL((scan_kernel<KL, F16MATH, TC, LO>), dim3(num_cus()), dim3(kThreads), lds, s, a);
    LMI_LAUNCH_CHECK("scan_kernel");
    if (timed) return timing_record(s, false, ev);
    return LMI_OK;
}

namespace {
template <int KL, int ABL>
int launch_scan2_v(const Scan2Args& b, hipStream_t s) {
    constexpr size_t lds = v2::lds_bytes<KL>();
    static_assert(lds <= 160 * 1024, "scan2 LDS budget");
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [] {
        attr_err = hipFuncSetAttribute((const void*)scan2_kernel<KL, ABL>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    });
    LMI_HIP_TRY(attr_err);
    const bool timed = timing().on;
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (timed) {
        const int rc = timing_record(s, true, ev);
        if (rc != LMI_OK) return rc;
    }
    hipLaunchKernelGGL((scan2_kernel<KL, ABL>), dim3(num_cus()), dim3(kThreads), lds, s, b);
    LMI_LAUNCH_CHECK("scan2_kernel");
    if (timed) return timing_record(s, false, ev);
    return LMI_OK;
}

}  // namespace

template <int KL>
int launch_scan2(const Scan2Args& b, hipStream_t s) {
    return launch_scan2_v<KL, 0>(b, s);
}


template int launch_scan<10, true, _Float16>(const ScanArgs&, int, hipStream_t);
template int launch_scan<16, true, _Float16>(const ScanArgs&, int, hipStream_t);
template int launch_scan<10, false, _Float16>(const ScanArgs&, int, hipStream_t);
template int launch_scan<16, false, _Float16>(const ScanArgs&, int, hipStream_t);
template int launch_scan<10, false, float>(const ScanArgs&, int, hipStream_t);
template int launch_scan<16, false, float>(const ScanArgs&, int, hipStream_t);
template int launch_scan<16, true, _Float16, true>(const ScanArgs&, int, hipStream_t);
template int launch_scan<16, false, _Float16, true>(const ScanArgs&, int, hipStream_t);
template int launch_scan<16, false, float, true>(const ScanArgs&, int, hipStream_t);
template int launch_scan2<10>(const Scan2Args&, hipStream_t);
template int launch_scan2<16>(const Scan2Args&, hipStream_t);

}  // namespace lmi
