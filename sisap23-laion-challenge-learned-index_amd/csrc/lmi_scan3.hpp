// scan3_kernel (scan v3, the K2 roofline kernel) and its device helpers.
// Included by lmi_scan.hip (the product: ABL == 0) and by lmi_scan_abl.hip
// (the diagnostic library of `make ablation`: the ABL != 0 variants that
// DESIGN.md §3 / §5 measure).  Each includer gets its own internal copy.
#pragma once
#include "lmi_scan_internal.hpp"

namespace lmi {
namespace {

// The seed of a pair (q, r >= 1) under LMI_Q_SEED_ROUND0: the current bound of
// pair (q, 0) -- an upper bound of its final k-th distance, which bounds every
// later round's threshold -- as a distance ordinal (+ seed_margin), or
// 0xffffffff (no bound yet / not seeded).
__device__ __forceinline__ uint32_t round0_seed(const Scan2Args& a, int pp) {
    const int pp0 = a.pair_pos[pp];  // (seed_pos_kernel: -1 for r = 0 pairs)
    if (pp0 < 0) return 0xffffffffu;
    const uint32_t s = (uint32_t)(__hip_atomic_load(&a.thr_g[pp0], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT) >> 32);
    if (s == 0xffffffffu || a.seed_margin == 0.0f) return s;
    // (+1: the next float up, whatever the rounding of the sum)
    const uint32_t m = f2ord(ord2f(s) + a.seed_margin) + 1u;
    return m == 0u ? 0xffffffffu : m;
}

// ---------------------------------------------------------------------------
// scan v3 (fp16 corpus, fp16-exact queries, d_pad == 768, k <= 10): the v2
// ring with 8 waves = two per SIMD.
//
//   per wave : 32 queries, B fragments (K = 768) in VGPRs for the whole tile
//              (VGPR-form MFMAs: a kernel with no AGPR gets all 256 registers);
//              the wave serves query group `slot` of the tile, slots being a
//              SIMD-balanced numbering (groups 0-3 land on four different
//              SIMDs, whatever the wave -> SIMD placement)
//   per tile : one chunk of one bucket x up to 256 pairs: every staged
//              object byte serves 256 queries (v2: 128), halving the
//              L2 -> LDS traffic, and the two waves of a SIMD hide each
//              other's filter / insertion VALU behind their MFMAs
//   ring     : 6 slots = two 32-row blocks of 3 stages (32 rows x 256 k,
//              16 pieces of two interleaved rows, see v3::PIECEP) + each
//              block's 32 norms in its last stage's slot; block b+1's DMA
//              rides in block b (each wave two 1-KiB pieces per stage and its
//              4 norms per block, at different MFMAs for the two waves of a
//              SIMD); one s_barrier per block
//   lists    : each lane's partial top-k list lives in LDS (registers are
//              taken by the query fragments); the filter bound stays in
//              registers, so the list is touched only on insertion
//   epilogue : per 32-row block, right after its last MFMA: a 16-bit
//              candidate mask from d = 1 - dot/(|q||y|) <= bound; only if
//              some lane has a candidate, every lane walks its own candidates
//              (accumulator picked by a select tree): the first KL are
//              appended unsorted, later ones inserted into the sorted list
// ---------------------------------------------------------------------------
namespace v3 {
constexpr int D = 768;
constexpr int ROWB = 512;              // bytes of one row in one stage (256 k)
// LDS image of a stage: 16 pieces of two rows each (one 1-KiB DMA), the two
// rows interleaved at 16-B granularity (row 2p+x, chunk c at 32c + 16x of
// piece p), pieces at a 1056-B pitch.  Row r chunk c then sits at
// (r>>1)*1056 + 32c + 16(r&1): affine in c, so a lane's A-fragment reads
// share one base register + immediate offsets, and the 32-row reads are
// bank-conflict free (bank start 4r + 8h mod 64).
constexpr int PIECEP = 2 * ROWB + 32;  // piece pitch
constexpr int NST = D * 2 / ROWB;      // stages per 32-row block
constexpr int NORM_OFF = 16 * PIECEP;  // the block's 32 norms (last stage's slot)
constexpr int STAGE = NORM_OFF + 128;
constexpr int NSLOT = 2 * NST;         // two blocks: one read, the next in flight
constexpr int NW = 8;
constexpr int QB = NW * 32;
constexpr int NQF = D / 16;
// lists of KL = 10 (k <= 10) or 15 (the float64 mode's 10 + 5 guard entries,
// the most the 160-KiB LDS holds beside the ring)
// lists: KL = 10 lane-interleaved ([entry][lane]); KL = 15 (cooperative
// insertion) one lane's entries contiguous, lanes list_stride entries apart
// (an odd number of 8-byte bank pairs: both the per-lane accesses of 32 lanes
// and the one-list-per-16-lanes accesses are free of bank conflicts)
template <int KL>
constexpr int list_stride() { return KL == 10 ? 11 : KL; }
template <int KL>
constexpr size_t lds_bytes() { return (size_t)NSLOT * STAGE + (size_t)NW * 64 * list_stride<KL>() * 8 + 64; }
static_assert(lds_bytes<15>() <= 160 * 1024, "LDS budget");
}  // namespace v3


// VGPR-form MFMAs for scan v3: a kernel that uses no AGPR gets the whole
// 256-register budget of a two-waves-per-SIMD launch as VGPRs (with AGPRs in
// use, the compiler splits it 128/128, too few for 192 query registers).
__device__ __forceinline__ f32x16 mfma_first_v(const half8& a, const half8& b) {
    f32x16 d;
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ f32x16 mfma_acc_v(const f32x16& c, const half8& a, const half8& b) {
    f32x16 d = c;
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
    return d;
}
// The block's last MFMA with the wait for its result in the same asm
// statement: the compiler does not know these are matrix instructions, so it
// inserts no wait states before reading their results, and it may copy the
// accumulators to other registers (a read) anywhere after the last MFMA;
// nothing can come between this MFMA and its drain (16 passes: >= 18 wait
// states before a VALU reads the result).  tests/test_codeobj.py checks it.
__device__ __forceinline__ f32x16 mfma_last_v(const f32x16& c, const half8& a, const half8& b) {
    f32x16 d = c;
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3"
                 : "+v"(d) : "v"(a), "v"(b));
    return d;
}
// (diagnostic ABL 66 / 68: the 16x16x32 shape, timing only)
__device__ __forceinline__ void mfma16_v(f32x4& c, const half8& a, const half8& b) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
// (diagnostic ABL 61: the wait at the epilogue instead)
__device__ __forceinline__ f32x16 mfma_drain_v(const f32x16& c) {
    f32x16 d = c;
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(d));
    return d;
}


// LDS list entries at a base VGPR + immediate offset (one address register
// for a whole list; plain-C++ addressing would hoist one register per entry)
template <int OFF>
__device__ __forceinline__ void lds_put_u64_at(uint32_t addr, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ uint64_t lds_get_u64_at(uint32_t addr) {
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
    return v;
}
// an LDS atomic add returning the old value (inline asm like the list
// accesses: the compiler would put a vmcnt wait -- the LDS-DMA writes into the
// ring -- in front of a C++ LDS access in the block loop)
__device__ __forceinline__ uint32_t lds_add_rtn_u32(uint32_t addr, uint32_t v) {
    uint32_t r;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr), "v"(v) : "memory");
    return r;
}
template <int KL, int OFF = 0, int ES = 512>
__device__ __forceinline__ void list_store(uint32_t addr, const uint64_t (&L)[KL]) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (lds_put_u64_at<OFF + I * ES>(addr, L[I]), ...);
    }(std::make_integer_sequence<int, KL>{});
}
// entry i at addr + OFF + i * ES (ES = 512: the lane-interleaved layout of
// round 1, 8: one lane's entries contiguous)
template <int KL, int OFF = 0, int ES = 512>
__device__ __forceinline__ void list_load(uint32_t addr, uint64_t (&L)[KL]) {
    static_assert(KL == 10 || KL == 15, "one asm block of 10 or 15 reads");
    // all reads in flight, one wait (a wait per read would serialise the LDS
    // round trips); one asm statement so no use can slip before the wait
    if constexpr (KL == 10) {
        asm volatile(
            "ds_read_b64 %0, %10 offset:%11\n\t"
            "ds_read_b64 %1, %10 offset:%12\n\t"
            "ds_read_b64 %2, %10 offset:%13\n\t"
            "ds_read_b64 %3, %10 offset:%14\n\t"
            "ds_read_b64 %4, %10 offset:%15\n\t"
            "ds_read_b64 %5, %10 offset:%16\n\t"
            "ds_read_b64 %6, %10 offset:%17\n\t"
            "ds_read_b64 %7, %10 offset:%18\n\t"
            "ds_read_b64 %8, %10 offset:%19\n\t"
            "ds_read_b64 %9, %10 offset:%20\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(L[0]), "=&v"(L[1]), "=&v"(L[2]), "=&v"(L[3]), "=&v"(L[4]), "=&v"(L[5]),
              "=&v"(L[6]), "=&v"(L[7]), "=&v"(L[8]), "=&v"(L[9])
            : "v"(addr), "i"(OFF), "i"(OFF + ES), "i"(OFF + 2 * ES), "i"(OFF + 3 * ES),
              "i"(OFF + 4 * ES), "i"(OFF + 5 * ES), "i"(OFF + 6 * ES), "i"(OFF + 7 * ES),
              "i"(OFF + 8 * ES), "i"(OFF + 9 * ES)
            : "memory");
    } else {
        asm volatile(
            "ds_read_b64 %0, %15 offset:%16\n\t"
            "ds_read_b64 %1, %15 offset:%17\n\t"
            "ds_read_b64 %2, %15 offset:%18\n\t"
            "ds_read_b64 %3, %15 offset:%19\n\t"
            "ds_read_b64 %4, %15 offset:%20\n\t"
            "ds_read_b64 %5, %15 offset:%21\n\t"
            "ds_read_b64 %6, %15 offset:%22\n\t"
            "ds_read_b64 %7, %15 offset:%23\n\t"
            "ds_read_b64 %8, %15 offset:%24\n\t"
            "ds_read_b64 %9, %15 offset:%25\n\t"
            "ds_read_b64 %10, %15 offset:%26\n\t"
            "ds_read_b64 %11, %15 offset:%27\n\t"
            "ds_read_b64 %12, %15 offset:%28\n\t"
            "ds_read_b64 %13, %15 offset:%29\n\t"
            "ds_read_b64 %14, %15 offset:%30\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(L[0]), "=&v"(L[1]), "=&v"(L[2]), "=&v"(L[3]), "=&v"(L[4]), "=&v"(L[5]),
              "=&v"(L[6]), "=&v"(L[7]), "=&v"(L[8]), "=&v"(L[9]), "=&v"(L[10]), "=&v"(L[11]),
              "=&v"(L[12]), "=&v"(L[13]), "=&v"(L[14])
            : "v"(addr), "i"(OFF), "i"(OFF + ES), "i"(OFF + 2 * ES), "i"(OFF + 3 * ES),
              "i"(OFF + 4 * ES), "i"(OFF + 5 * ES), "i"(OFF + 6 * ES), "i"(OFF + 7 * ES),
              "i"(OFF + 8 * ES), "i"(OFF + 9 * ES), "i"(OFF + 10 * ES), "i"(OFF + 11 * ES),
              "i"(OFF + 12 * ES), "i"(OFF + 13 * ES), "i"(OFF + 14 * ES)
            : "memory");
    }
}

// In-place odd-even transposition sort of a short list (ascending keys).
template <int KL>
__device__ __forceinline__ void list_sort(uint64_t (&L)[KL]) {
#pragma unroll
    for (int r = 0; r < KL; ++r) {
#pragma unroll
        for (int i = r & 1; i + 1 < KL; i += 2) {
            const uint64_t x = L[i], y = L[i + 1];
            L[i] = x < y ? x : y;
            L[i + 1] = x < y ? y : x;
        }
    }
}

// The same on distance words only, equal distances kept in arrival order
// (stable): the scan's per-lane lists, whose rows arrive in ascending order.
template <int KL>
__device__ __forceinline__ void list_sort_hi(uint64_t (&L)[KL]) {
#pragma unroll
    for (int r = 0; r < KL; ++r) {
#pragma unroll
        for (int i = r & 1; i + 1 < KL; i += 2) {
            const uint64_t x = L[i], y = L[i + 1];
            const bool sw = (uint32_t)(y >> 32) < (uint32_t)(x >> 32);
            L[i] = sw ? y : x;
            L[i + 1] = sw ? x : y;
        }
    }
}
// list_insert on distance words: x goes after the entries of equal distance
// (it arrived later); caller guarantees dist(x) < dist(L[KL-1]).
template <int KL>
__device__ __forceinline__ void list_insert_hi(uint64_t (&L)[KL], uint64_t x) {
    const uint32_t xh = (uint32_t)(x >> 32);
    bool lt_i = xh < (uint32_t)(L[KL - 1] >> 32);
#pragma unroll
    for (int i = KL - 1; i > 0; --i) {
        const bool lt_p = xh < (uint32_t)(L[i - 1] >> 32);
        L[i] = lt_p ? L[i - 1] : (lt_i ? x : L[i]);
        lt_i = lt_p;
    }
    L[0] = lt_i ? x : L[0];
}

extern "C" __device__ uint32_t __ockl_wfred_or_u32(uint32_t);
extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);

// Diagnostic instantiations (ABL != 0, lmi_scan_abl.hip, `make ablation`)
// count into Scan2Args::dbg: ABL == 7 the full kernel plus event counters
// [0] blocks with a candidate in some lane (wave events), [1] candidates,
// [2] appends, [3] sorted insertions, [4] buffer fills (sorts), [5] blocks;
// every ABL: [8] sum over workgroups of shader-clock cycles (s_memtime) and
// [9] of 100-MHz ticks (s_memrealtime) between kernel entry and exit,
// [10] earliest entry tick, [11] latest exit tick, [12] workgroups.  The
// product instantiates ABL == 0 only, where all of it compiles away.

// lowest set bit of a wave-uniform mask, -1 if none (s_ff1_i32_b64)
__device__ __forceinline__ int sff1_u64(uint64_t m) {
    int r;
    asm("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(m));
    return r;
}

// Per-lane pick of acc[rg] (rg differs by lane): a 4-level select tree on
// lane masks (inline asm: written as C++ ternaries the compiler turns the
// tree back into a dynamically indexed array on scratch).
__device__ __forceinline__ float sel_mask(float a, float b, uint64_t m) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
__device__ __forceinline__ float select16(const f32x16& acc, int rg) {
    const uint64_t b3 = __builtin_amdgcn_ballot_w64((rg & 8) != 0);
    const uint64_t b2 = __builtin_amdgcn_ballot_w64((rg & 4) != 0);
    const uint64_t b1 = __builtin_amdgcn_ballot_w64((rg & 2) != 0);
    const uint64_t b0 = __builtin_amdgcn_ballot_w64((rg & 1) != 0);
    float v8[8], v4[4], v2[2];
#pragma unroll
    for (int e = 0; e < 8; ++e) v8[e] = sel_mask(acc[e], acc[e + 8], b3);
#pragma unroll
    for (int e = 0; e < 4; ++e) v4[e] = sel_mask(v8[e], v8[e + 4], b2);
#pragma unroll
    for (int e = 0; e < 2; ++e) v2[e] = sel_mask(v4[e], v4[e + 2], b1);
    return sel_mask(v2[0], v2[1], b0);
}

// Keeps the compiler from hoisting lane-dependent address arithmetic out of
// the tile loop (each hoisted value would pin a VGPR for the whole kernel).
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ uint32_t opaque_u(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}

// MODE (k > 16, bucket_topk_wide): 0 the product scan; 1 chunk lists -- every
// (pair, chunk part) list is that part's own top-KL (no global bound read,
// exchanged or published), the rows behind the wide path's per-pair bound;
// 2 collect -- every row of a pair within its fixed bound (thr_g, set by the
// plan) is appended to the pair's candidate buffer (Scan2Args::cand), no lists.
// MODE 3 (the float64 mode's band lists, KL = 10): the product scan with the
// filter widened by Scan2Args::band (2 eps) and, per (pair, chunk part), the
// first 15 of the two lanes' lists plus a bound below which every unlisted
// row of the part that passed the filter lies (kBandSlot entries, see
// chunk_merge_band_kernel).
template <int KL, int ABL = 0, bool LO = false, int MODE = 0>
__global__ __launch_bounds__(512, 1) void scan3_kernel(Scan2Args a) {
    using namespace v3;
    static_assert(MODE == 0 || (ABL == 0 && !LO), "the wide modes are product variants");
    static_assert(MODE != 3 || KL == 10, "band lists are built from 10-entry lane lists");
    // diagnostic builds only (results wrong for ABL != 0): 1 no insertion,
    // 2 DMA + barriers only, 3 no DMA, 4 no DMA and no insertion, 5 no DMA and
    // no epilogue, 6 = 5 without barriers, 7 event counters, 14 no DMA wait,
    // 21 no barrier, 31 every block's DMA re-reads the tile's first 4 blocks
    // (L2-resident source: the cost of DMA without HBM misses), 32 = 2 with
    // the source of 31, 33 non-temporal row loads (aux = nt)
    constexpr int kAux = ABL == 33 ? 2 : 0;
    constexpr bool kDmaOnly = ABL == 2 || ABL == 32;
    constexpr bool kL2Src = ABL == 31 || ABL == 32;
    // 66 = 6 with v_mfma_f32_16x16x32_f16 (same operand registers, same LDS
    // bytes, 96 MFMAs of 16 cycles per wave-block: timing of the shape only),
    // 67 = the full kernel without the epilogue, 68 = 67 with 16x16x32
    constexpr bool kM16 = ABL == 66 || ABL == 68;
    constexpr bool kNoDma = ABL == 3 || ABL == 4 || ABL == 5 || ABL == 6 || ABL == 66 || ABL == 69 || ABL == 70;
    constexpr bool kNoEpi = kDmaOnly || ABL == 5 || ABL == 6 || ABL == 66 || ABL == 67 || ABL == 68 ||
                            ABL == 69 || ABL == 70;
    constexpr bool kNoIns = ABL == 1 || ABL == 4;
    constexpr bool kNoBar = ABL == 6 || ABL == 66 || ABL == 21 || ABL == 69 || ABL == 70;
    // bound exchange period in blocks (diagnostic: 40 none, 41 every 4, 42 every 8, 43 every 16)
    constexpr int kXch = (ABL == 40 || MODE != 0) ? 0 : ABL == 41 ? 4 : ABL == 42 ? 8 : ABL == 43 ? 16 : 32;
    // (ABL 53, round 1's placement: an LDS-DMA issue holds its wave for ~45-60
    // cycles, so the two waves of a SIMD issued theirs at different MFMAs)
    constexpr int kDmaTT = 2, kDmaLate = 10;
    // Top-k insertion.  KL = 10: every lane inserts into its own list (a
    // register copy of it: load, insert, store).  KL = 15: a register copy of
    // 15 entries does not fit beside the query fragments (the compiler
    // spills them into the MFMA stream), so the lists are updated
    // cooperatively, 16 lanes per list, an entry per lane, four lists per
    // wave instruction.  ABL 65: cooperative at KL = 10 too (slower there).
    constexpr bool kCoop = KL > 10 || ABL == 65;
    // entries per lane column (MODE 3: slot KL holds the smallest distance
    // ordinal the lane dropped -- evicted, or not inserted -- see below)
    constexpr int LS = kCoop ? list_stride<KL>() : (MODE == 3 ? KL + 1 : KL);
    static_assert(LS <= list_stride<KL>(), "lane slots beyond the LDS budget");
    constexpr int ES = kCoop ? 8 : 512;                  // bytes between a list's entries
    constexpr uint32_t LSTR = kCoop ? LS * 8 : 8;        // bytes between lanes' lists
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* ring = smem;
    // every lane's partial top-k list in LDS (registers are all spoken for
    // by the query fragments): entry i of lane l at l * LSTR + i * ES
    uint64_t* lists = reinterpret_cast<uint64_t*>(smem + NSLOT * STAGE);
    int* wtab = reinterpret_cast<int*>(lists + NW * 64 * LS);  // [NW] SIMD ids, [NW] tile
    int& s_tile = wtab[NW];
    // MODE 2 (collect): the lists' area holds instead each of the tile's 256
    // pairs' candidate stage (kXS keys) and its count
    constexpr int kXS = 19;
    static_assert(MODE != 2 || (size_t)NW * 32 * (kXS * 8 + 4) <= (size_t)NW * 64 * LS * 8, "collect stage");
    uint64_t* xst = lists;
    uint32_t* xcnt = reinterpret_cast<uint32_t*>(lists + NW * 32 * kXS);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ng = a.ng;

    // SIMD-balanced slot of this wave: order waves by (rank on their SIMD, SIMD)
    int simd, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 4, 2)" : "=s"(simd));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    if (lane == 0) wtab[wave] = simd;
    __syncthreads();
    int slot = 0;
    {
        int key_me = simd;
        for (int w = 0; w < wave; ++w) key_me += (wtab[w] == simd) ? 4 : 0;  // + rank * 4
        for (int w = 0; w < NW; ++w) {
            int kw = wtab[w];
            for (int v = 0; v < w; ++v) kw += (wtab[v] == wtab[w]) ? 4 : 0;
            slot += (kw < key_me || (kw == key_me && w < wave)) ? 1 : 0;
        }
        slot = __builtin_amdgcn_readfirstlane(slot);
    }
    const int gx = xcc & (ng - 1);
    const bool late = slot >= NW / 2;
    int partner = wave;  // the other wave of this SIMD
    for (int w = 0; w < NW; ++w)
        if (w != wave && wtab[w] == simd) partner = w;
    partner = __builtin_amdgcn_readfirstlane(partner);
    // (diagnostic builds: the entry clocks wait in LDS, not in registers --
    // two live 64-bit values spilled a query fragment into the MFMA stream)
    uint64_t* clk_lds = reinterpret_cast<uint64_t*>(wtab + NW + 2);
    if constexpr (ABL != 0) {
        if (tid == 0) {
            clk_lds[0] = __builtin_amdgcn_s_memtime();
            clk_lds[1] = __builtin_amdgcn_s_memrealtime();
        }
    }
    const uint32_t wbase = (uint32_t)(uintptr_t)(lists + wave * 64 * LS);  // this wave's lists
    const uint32_t lbase = wbase + (uint32_t)lane * LSTR;                   // this lane's

    for (;;) {
        if (tid == 0) s_tile = dequeue_tile(a.meta, a.work, gx, ng);
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(s_tile);
        if (t < 0) break;
        const Tile tile = a.tiles[t];
        const int64_t bstart = a.bucket_off[tile.c];
        // (chunk-list mode: the bucket's own list rows, and of each list the
        // first sub_take rows, a sample)
        const int64_t row0 = bstart + (int64_t)tile.chunk * (MODE == 1 ? a.sub_rows[tile.c] : a.chunk_rows);
        const int nrows = __builtin_amdgcn_readfirstlane(
            (int)std::min<int64_t>(MODE == 1 ? a.sub_take[tile.c] : a.chunk_rows, a.bucket_off[tile.c + 1] - row0));
        const uint32_t r0lo = __builtin_amdgcn_readfirstlane((uint32_t)row0);
        const uint32_t r0hi = __builtin_amdgcn_readfirstlane((uint32_t)(row0 >> 32));
        const int64_t row0u = (int64_t)(((uint64_t)r0hi << 32) | r0lo);
        const int np = __builtin_amdgcn_readfirstlane(tile.np);
        const bool wave_live = 32 * slot < np;
        const int h = opaque(lane) >> 5;
        const int col = lane & 31;
        const bool live = 32 * slot + col < np;
        const int pp = tile.pp0 + 32 * slot + col;

        // Block 0's DMA goes out before the query fragments are loaded, so
        // the two memory latencies of a tile's start overlap (the ring is
        // free: the previous tile drained it before its closing barrier)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.corpus + row0u * D), (short)0, nrows * D * 2, 0x00020000);
        const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.inv_norm + row0u), (short)0, nrows * 4, 0x00020000);

        const int nblk = (nrows + 31) / 32;
        // DMA of one stage (block b, phase j) into the LDS slot at byte offset
        // `so`: pieces 0, 1 = rows 4w+2i, 4w+2i+1 (lane l: row 4w + 2i + (l&1),
        // chunk l >> 1; piece 1 is piece 0 + 2 rows through soffset); in the
        // block's last phase the wave's 4 norms too.
        // the pieces of wave w (its 4 rows of the block and their norms)
        auto dma_stage_w = [&](int so, int b, int j, int w) {
            if (kNoDma) return;
            unsigned char* sl = ring + so;
            const int nb_area = b % 3;  // norms of block b: slot (b % 3)'s norm area
            if (kL2Src) b &= 3;
            const uint32_t vo_row = (uint32_t)((4 * w + (lane & 1)) * (D * 2) + (lane >> 1) * 16);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t)(sl + (2 * w) * PIECEP), 16, vo_row,
                                                     b * (32 * D * 2) + j * ROWB, 0, kAux);
            // (+2 rows through soffset: an instruction offset would move the
            // LDS destination as well, LDS_ADDR = M0 + inst_offset + lane * 16)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t)(sl + (2 * w + 1) * PIECEP), 16,
                                                     vo_row, b * (32 * D * 2) + j * ROWB + 2 * D * 2,
                                                     0, kAux);
            if (j == NST - 1 && lane < 4)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rn, (lds_t)(ring + nb_area * STAGE + NORM_OFF + 16 * w),
                                                         4, (uint32_t)((4 * w + opaque(lane)) * 4), b * 128, 0, 0);
        };
        auto dma_stage = [&](int so, int b, int j) { dma_stage_w(so, b, j, wave); };
        // block b lives in slots NST*(b&1) .. +NST-1; block 0 is the prologue,
        // block b+1's DMA rides in block b
#pragma unroll
        for (int j = 0; j < NST; ++j) dma_stage(j * STAGE, 0, j);

        half8 qf[NQF];
        // the lane's bound: only objects with ord(d) <= thr can enter the
        // pair's top-KL (the distance part of a key: the bound may come from
        // another chunk, whose rows are ordered differently, so ties at it
        // survive to the chunk merge)
        uint32_t thr = 0u;
        float my_invq = 0.0f;
        float lo_d = -__builtin_inff();  // LO: the distance of this pair's lower-bound key,
        int lo_row = 0;                  // and the chunk's first row after its position
        int cnt = 0;  // entries in this lane's list; < KL: an unsorted append buffer
        if (wave_live) {
            bool done = false;
            const int q = live ? a.pair_q[pp] / a.R : 0;
            if (LO && live) {
                // positions ascend inside a chunk, so "after the lower bound's
                // position" is "at or after local row lo_row" (binary search,
                // once per tile; the walk then needs no memory access)
                const uint64_t lo = a.lo_g[a.pair_q[pp]];
                if (lo == kEmptyKey) {
                    done = true;  // the pair's objects are all listed: take nothing
                } else if ((uint32_t)(lo >> 32) != 0u) {
                    lo_d = ord2f((uint32_t)(lo >> 32));
                    int l = 0, r = nrows;
                    while (l < r) {
                        const int mid = (l + r) >> 1;
                        if ((uint32_t)a.gpos[row0u + mid] > (uint32_t)lo) r = mid;
                        else l = mid + 1;
                    }
                    lo_row = l;
                }
            }
            const half8* qrow = reinterpret_cast<const half8*>(a.qbuf + (size_t)q * D) + h;
            // dead columns of a partial wave multiply zeros: their results
            // are never read, and zero operands draw less MFMA power (the
            // chip holds a power-limited clock under this kernel; diagnostic
            // ABL 57: query 0's fragments, round 1's)
            const half8 z{};
#pragma unroll
            for (int s = 0; s < NQF; ++s) qf[s] = (live || ABL == 57) ? qrow[2 * s] : z;
            // dead slots (and exhausted pairs) reject everything
            thr = live && !done ? (uint32_t)(a.thr_g[pp] >> 32) : 0u;
            if constexpr (!LO) {  // (the k > 16 passes are never seeded)
                if (a.pair_pos && live) thr = std::min(thr, round0_seed(a, pp));
            }
            my_invq = live ? a.invq[q] : 0.0f;
            if constexpr (MODE == 1) {
                // (no bound until every bin holds a finished list's 15th)
                if (live) {
                    uint32_t bmax = 0u;
                    for (int j = 0; j < a.nbins; ++j) bmax = std::max(bmax, a.bins[(size_t)pp * a.nbins + j]);
                    thr = std::min(thr, bmax);
                }
            }
        }
        if constexpr (MODE != 2) {
            uint64_t E[KL];
            list_clear<KL>(E);
            list_store<KL, 0, ES>(opaque_u(lbase), E);
            if constexpr (MODE == 3) lds_put_u64_at<KL * ES>(opaque_u(lbase), kEmptyKey);
        } else {
            if (h == 0) xcnt[32 * slot + col] = 0u;
        }
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
        __syncthreads();

        // a lane's A-fragment base inside a slot (row col = lane & 31, half h)
        const uint32_t lane_off = (uint32_t)(((lane >> 1) & 15) * PIECEP + (lane & 1) * 16 + (lane >> 5) * 32);

        f32x16 acc;
        f32x4 acc4[4] = {};  // (diagnostic 66 / 68 only)
        uint32_t xg_carry = 0xffffffffu;  // global bound fetched, not yet applied
        // ---- epilogue of block eb (accumulators of its 48 MFMAs in acc) ------
        auto epilogue = [&](int eb) {
            // (acc is complete: the block's last MFMA carried its drain)
            if (ABL == 61) acc = mfma_drain_v(acc);
            const int ln = opaque(lane);
            const int hh = ln >> 5;
            // block eb's norms: the norm area of slot eb % 3 (three blocks in
            // flight: the late waves read block b's during block b + 1)
            const unsigned char* nb = ring + (eb % 3) * STAGE + NORM_OFF + hh * 16;
            const int vr = nrows - eb * 32 - 4 * hh;  // valid rows past this lane's offset
            thr = std::min(thr, xg_carry);
            xg_carry = 0xffffffffu;
            // (MODE 3: rows up to 2 eps past the bound pass the filter, so a
            // row the band lists do not hold lies above the pair's d32 k-th
            // + 2 eps or at / above the part's bound; the lane lists and the
            // bounds published stay the plain k-th)
            float bound = key_dist_bound((uint64_t)thr << 32);
            if constexpr (MODE == 3) bound += a.band;
            // the filter: a candidate mask, one bit per register, register 0
            // in bit 15 (mask = 2 mask + ok); only the chunk's last block
            // checks the row count
            uint32_t mask = 0;
            auto filter = [&]<bool TAIL>() {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 n4 = *reinterpret_cast<const f32x4*>(nb + 32 * g);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int reg = 4 * g + e;
                        const float d = fmaf(-acc[reg], my_invq * n4[e], 1.0f);
            
                        // (LO: lo_d <= d <= bound as one med3 and one compare)
                        bool ok = LO ? __builtin_amdgcn_fmed3f(d, lo_d, bound) == d : d <= bound;
                        if (TAIL) ok = ok && e + 8 * g < vr;
                        mask = mask + mask + (ok ? 1u : 0u);
                    }
                }
            };
            if (eb + 1 < nblk && ABL != 62)
                filter.template operator()<false>();
            else
                filter.template operator()<true>();
            if constexpr (ABL == 7) {
                const uint32_t nc = __ockl_wfred_add_u32(__builtin_popcount(mask));
                if (lane == 0) {
                    atomicAdd(&a.dbg[5], 1ull);
                    if (nc) atomicAdd(&a.dbg[0], 1ull);
                    atomicAdd(&a.dbg[1], (unsigned long long)nc);
                }
            }
            if constexpr (MODE == 2) {
                // collect: each lane reserves slots of its pair's stage in
                // LDS (an LDS atomic) and writes its candidates there -- no
                // global memory op in the block loop, whose return the early
                // wave would wait for behind its next block's DMA (vmcnt);
                // the stage goes to the pair's candidate buffer at the tile
                // end.  Keys past kXS go to the buffer directly (a global
                // atomic each: rare); slots past cap are counted, not stored.
                if (__any(mask != 0)) {
                    const uint32_t rb = (uint32_t)(row0u + eb * 32 + 4 * hh);
                    const uint32_t c = (uint32_t)__builtin_popcount(mask);
                    const int lp = 32 * slot + col;
                    uint32_t at = 0;
                    if (c != 0) at = lds_add_rtn_u32((uint32_t)(uintptr_t)(xcnt + lp), c);
                    const uint32_t sa = (uint32_t)(uintptr_t)(xst + lp * kXS);
                    uint32_t m = mask;
#pragma unroll 1
                    while (__any(m != 0)) {
                        if (m != 0) {
                            const int hb = 31 - __builtin_clz(m);
                            m ^= 1u << hb;
                            const int rg = 15 - hb;
                            const int i = (rg & 3) + 8 * (rg >> 2);
                            const float n1 = *reinterpret_cast<const float*>(nb + i * 4);
                            const float d = fmaf(-select16(acc, rg), my_invq * n1, 1.0f);
                            const uint64_t key = make_key(d, rb + (uint32_t)i);
                            if (at < (uint32_t)kXS) {
                                lds_put_u64_at<0>(sa + 8u * at, key);
                            } else {
                                const uint32_t g = atomicAdd(&a.ccount[pp], 1u);
                                if (g < (uint32_t)a.cap) a.cand[(size_t)pp * (uint32_t)a.cap + g] = key;
                            }
                            ++at;
                        }
                    }
                }
            } else
            if (!kNoIns && __any(mask != 0)) {
                const uint32_t rb = (uint32_t)(row0u + eb * 32 + 4 * hh);
                // Every lane walks its own candidates, lowest register first:
                // iterations = the largest per-lane count (usually 1-2), the
                // accumulator picked by a select tree.  Candidates: d <= the
                // distance part of thr, a bound that may come from another
                // chunk (rows ordered differently there), so no key test
                // against it; ties at the bound are resolved by the chunk
                // merge.  A lane meets its rows in ascending order (registers
                // ascending inside a block, blocks ascending), so a list
                // ordered by distance with equal distances in arrival order is
                // ordered by key: the list compares distance words only.
                uint32_t m = mask;
                if constexpr (kCoop) {
                    // Round r: every lane with a candidate left offers its
                    // next one; lane group g (16 lanes, lane j = entry j)
                    // takes the list of the g-th offering lane: entry j stays
                    // if it comes before the key, else takes the key (entry
                    // j-1 comes before it, or j = 0) or entry j-1 (DPP row
                    // shift).  "Before" = smaller distance, or equal distance
                    // (it arrived earlier).
                    const int grp = ln >> 4, j = ln & 15;
#pragma unroll 1
                    while (__any(m != 0)) {
                        uint64_t key = kEmptyKey;
                        if (m != 0) {
                            const int hb = 31 - __builtin_clz(m);
                            m ^= 1u << hb;
                            const int rg = 15 - hb;
                            const int i = (rg & 3) + 8 * (rg >> 2);
                            const float n1 = *reinterpret_cast<const float*>(nb + i * 4);
                            const float d = fmaf(-select16(acc, rg), my_invq * n1, 1.0f);
                            key = make_key(d, rb + (uint32_t)i);
                            // (at or before the pair's lower bound: not this pass's)
                            if (LO && d == lo_d && eb * 32 + 4 * hh + i < lo_row) key = kEmptyKey;
                        }
                        const bool offer = key != kEmptyKey && (uint32_t)(key >> 32) <= thr;
                        uint64_t pend = __builtin_amdgcn_ballot_w64(offer);
                        const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
#pragma unroll 1
                        while (pend != 0) {
                            // this batch's offering lanes (s_ff1 gives -1 once
                            // pend is empty); group g takes the g-th one's key
                            const int s0 = sff1_u64(pend);
                            pend &= pend - 1;
                            const int s1 = sff1_u64(pend);
                            pend &= pend - 1;
                            const int s2 = sff1_u64(pend);
                            pend &= pend - 1;
                            const int s3 = sff1_u64(pend);
                            pend &= pend - 1;
                            const int my = grp == 0 ? s0 : grp == 1 ? s1 : grp == 2 ? s2 : s3;
                            const int sl = my < 0 ? 0 : my;
                            const uint32_t kl = (uint32_t)__builtin_amdgcn_ds_bpermute(sl << 2, (int)klo);
                            const uint32_t kh = (uint32_t)__builtin_amdgcn_ds_bpermute(sl << 2, (int)khi);
                            const bool act = my >= 0 && j < KL;
                            const uint32_t ea = wbase + (uint32_t)sl * LSTR + (uint32_t)j * 8u;
                            uint64_t e = kEmptyKey;
                            if (act) e = lds_get_u64(ea);
                            const bool before = (uint32_t)(e >> 32) <= kh;
                            const uint32_t pl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)e, 0x111, 0xf, 0xf, false);
                            const uint32_t ph = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(e >> 32), 0x111, 0xf, 0xf, false);
                            const int pb = __builtin_amdgcn_update_dpp(0, before ? 1 : 0, 0x111, 0xf, 0xf, false);
                            const uint64_t nv = (j == 0 || pb != 0) ? (((uint64_t)kh << 32) | kl)
                                                                     : (((uint64_t)ph << 32) | pl);
                            if (act && !before) lds_put_u64(ea, nv);
                        }
                        // the offering lanes' lists changed: their KL-th key
                        if (offer) thr = std::min(thr, (uint32_t)(lds_get_u64(lbase + (KL - 1) * 8) >> 32));
                    }
                } else {
                const uint32_t la = opaque_u(lbase);
#pragma unroll 1
                while (__any(m != 0)) {
                    if (m != 0) {
                        const int hb = 31 - __builtin_clz(m);
                        m ^= 1u << hb;
                        const int rg = 15 - hb;
                        const int i = (rg & 3) + 8 * (rg >> 2);
                        const float n1 = *reinterpret_cast<const float*>(nb + i * 4);
                        const float d = fmaf(-select16(acc, rg), my_invq * n1, 1.0f);
                        const uint64_t key = make_key(d, rb + (uint32_t)i);
                        if (LO && d == lo_d && eb * 32 + 4 * hh + i < lo_row) {
                            // at or before the pair's lower bound: not this pass's
                        } else if (cnt < KL) {
                            // append mode: the first KL candidates are stored
                            // unsorted; a full buffer is sorted once (stable)
                            // and the lane switches to list mode
                            lds_put_u64(la + (uint32_t)cnt * 512u, key);
                            if (++cnt == KL) {
                                uint64_t L[KL];
                                list_load<KL>(la, L);
                                list_sort_hi<KL>(L);
                                list_store<KL>(la, L);
                                thr = std::min(thr, (uint32_t)(L[KL - 1] >> 32));
                            }
                        } else {
                            uint64_t L[KL];
                            list_load<KL>(la, L);
                            // (MODE 3: the distance this candidate drops, the
                            // list's old KL-th when it is evicted, else its own)
                            uint32_t drop = (uint32_t)(key >> 32);
                            if (ABL == 64 ? key < L[KL - 1] : (uint32_t)(key >> 32) < (uint32_t)(L[KL - 1] >> 32)) {
                                if constexpr (MODE == 3) drop = (uint32_t)(L[KL - 1] >> 32);
                                if (ABL == 64)
                                    list_insert<KL>(L, key);
                                else
                                    list_insert_hi<KL>(L, key);
                                list_store<KL>(la, L);
                            }
                            if constexpr (MODE == 3) {
                                const uint64_t dm = lds_get_u64_at<KL * 512>(la);
                                if ((uint64_t)drop << 32 < dm) lds_put_u64_at<KL * 512>(la, (uint64_t)drop << 32);
                            }
                            thr = std::min(thr, (uint32_t)(L[KL - 1] >> 32));
                        }
                    }
                }
                }
                // every bound is an upper bound of the pair's k-th key: share it
                thr = std::min(thr, partner_u32(thr, hh));
            }
        };
        // The two waves of a SIMD are staggered (MI355X_MICROARCH "two waves
        // per SIMD", item 9): the early wave (slots 0-3) runs block b's MFMAs
        // and then its epilogue; the late wave (slots 4-7) runs block b-1's
        // epilogue first (its accumulators carried across the barrier) and
        // then block b's MFMAs, so one wave's filter / insertion VALU runs
        // beside the other's matrix work instead of both idling the pipe.
        const bool defer = late && !kNoEpi && wave_live;
        for (int blk = 0; blk < nblk; ++blk) {
            const bool more = blk + 1 < nblk;
            const int rs0 = (blk & 1) * NST * STAGE;        // this block's slots
            const int ws0 = ((blk + 1) & 1) * NST * STAGE;  // the next block's (= block blk-1's)
            // one barrier per block: this wave's DMA of block blk has landed
            // (nothing newer is in flight yet) and, past the barrier, every
            // wave's has, and every wave is done with block blk-1's slots
            if (ABL != 14) __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
            if (!kNoBar) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            // Block blk+1's DMA (its slots are block blk-1's, free past the
            // barrier): the early wave issues its pieces of all three stages
            // right here, ahead of its MFMAs; the late wave right after its
            // deferred epilogue.  A whole block of MFMAs then covers the
            // fetch (7.45 vs 8.29 ms at 10M against issuing each stage's
            // pieces inside that stage's MFMA stream, tools/prof_scan.py).
            // Diagnostic placements: 53 = inside the MFMA stream (round 1),
            // 50 = every wave at the head, 52 = the early wave issues its
            // partner's pieces too.
            constexpr bool kDmaStream = ABL == 53;
            constexpr bool kDmaHead = !kDmaStream;
            if (kDmaHead && more && !(ABL != 50 && late))
                for (int j = 0; j < NST; ++j) {
                    dma_stage(ws0 + j * STAGE, blk + 1, j);
                    if (ABL == 52 && partner != wave) dma_stage_w(ws0 + j * STAGE, blk + 1, j, partner);
                }
            if (defer && blk > 0) epilogue(blk - 1);
            if (kDmaHead && ABL != 50 && ABL != 52 && more && late)
                for (int j = 0; j < NST; ++j) dma_stage(ws0 + j * STAGE, blk + 1, j);
            // every kXch blocks: publish this lane's bound to the pair's global
            // bound and take the global one back (tiles of the same pair on
            // other chunks run concurrently); the returning atomic is consumed
            // in the next epilogue, behind this block's MFMAs
            if (kXch > 0 && (blk & (kXch - 1)) == kXch - 1 && live) {
                xg_carry = std::min(xg_carry, (uint32_t)(atomicMin(&a.thr_g[pp], ((unsigned long long)thr << 32) | 0xffffffffull) >> 32));

            }
            if (kDmaOnly || !wave_live) {
                // (no MFMA stream: a branch out of the middle of one would
                // join its accumulators to a path without the drain)
                if (more && !kDmaHead)
                    for (int j = 0; j < NST; ++j) dma_stage(ws0 + j * STAGE, blk + 1, j);
            } else {
            if constexpr (kM16) {
#pragma unroll
                for (int j = 0; j < NST; ++j) {
                    const unsigned char* rp = ring + rs0 + j * STAGE + opaque_u(lane_off);
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk) {
                        const half8 a0 = *reinterpret_cast<const half8*>(rp + 64 * (2 * kk));
                        const half8 a1 = *reinterpret_cast<const half8*>(rp + 64 * (2 * kk + 1));
#pragma unroll
                        for (int qt = 0; qt < 2; ++qt) {
                            mfma16_v(acc4[2 * qt], a0, qf[j * 16 + 2 * kk + qt]);
                            mfma16_v(acc4[2 * qt + 1], a1, qf[j * 16 + 2 * kk + qt]);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            } else
#pragma unroll
            for (int j = 0; j < NST; ++j) {
                const unsigned char* rp = ring + rs0 + j * STAGE + opaque_u(lane_off);
#define LMI_A3(tt) (*reinterpret_cast<const half8*>(rp + 64 * (tt)))
                half8 af[16];
#pragma unroll
                for (int tt = 0; tt < 3; ++tt) af[tt] = LMI_A3(tt);
#pragma unroll
                for (int tt = 0; tt < 16; ++tt) {
                    // (ABL 69: every other A fragment re-used instead of read;
                    //  ABL 70: only the first three read: the LDS reads' share
                    //  of the MFMA stream's power, timing only)
                    if (tt + 3 < 16)
                        af[tt + 3] = (ABL == 70 || (ABL == 69 && ((tt + 3) & 1))) ? af[tt + 2 - (ABL == 70 ? 2 : 0)]
                                                                                   : LMI_A3(tt + 3);
                    acc = (j == 0 && tt == 0)        ? mfma_first_v(af[0], qf[0])
                          : (j == NST - 1 && tt == 15 && ABL != 61) ? mfma_last_v(acc, af[tt], qf[j * 16 + tt])
                                                       : mfma_acc_v(acc, af[tt], qf[j * 16 + tt]);
                    if (!kDmaHead && tt == (late ? kDmaLate : kDmaTT) && more)
                        dma_stage(ws0 + j * STAGE, blk + 1, j);
                    // keep the A-fragment reads 3 MFMAs ahead, no further
                    __builtin_amdgcn_sched_barrier(0);
                }
#undef LMI_A3
            }
            }
            if (kNoEpi || !wave_live || defer) continue;
            epilogue(blk);
        }
        if (defer && nblk > 0) epilogue(nblk - 1);
        // lanes still in append mode hold an unsorted (EMPTY-padded) buffer
        if (MODE != 2 && !kCoop && __any(cnt < KL)) {
            if (cnt < KL) {
                uint64_t L[KL];
                list_load<KL>(lbase, L);
                list_sort<KL>(L);
                list_store<KL>(lbase, L);
            }
        }
        __syncthreads();  // every wave's DMA drained (the tail waited vmcnt(0))

        // ---- collect: each pair's stage to its candidate buffer ------------
        if (MODE == 2 && h == 0 && live) {
            const int lp = 32 * slot + col;
            const uint32_t n = std::min<uint32_t>(xcnt[lp], (uint32_t)kXS);
            if (n != 0) {
                const uint32_t base = atomicAdd(&a.ccount[pp], n);
                uint64_t* dst = a.cand + (size_t)pp * (uint32_t)a.cap;
#pragma unroll 1
                for (uint32_t i = 0; i < n; ++i)
                    if (base + i < (uint32_t)a.cap) dst[base + i] = xst[lp * kXS + i];
            }
        }

        // ---- merge the two partial lists of each query (lanes col, col+32) ----
        if (MODE == 3 && h == 0 && live) {
            // the union's first 15 by a two-pointer merge over the two LDS
            // lists (no register list: the kernel has no VGPR to spare) and
            // the part's bound: every unlisted row that passed the filter was
            // dropped by its lane (d >= the lane's smallest dropped distance)
            // or is the union's 16th or later
            const uint32_t pb = lbase + 32 * LSTR;
            uint64_t x = lds_get_u64(lbase), y = lds_get_u64(pb);
            int ia = 0, ib = 0;
            uint64_t* out = a.partial + ((size_t)pp * a.max_chunks + tile.chunk) * kBandSlot;
            uint64_t tenth = kEmptyKey;
#pragma unroll 1
            for (int o = 0; o < kBandSlot - 1; ++o) {
                const bool ta = x <= y;
                const uint64_t v = ta ? x : y;
                out[o] = v;
                if (o == KL - 1) tenth = v;
                if (ta) {
                    ++ia;
                    x = ia < KL ? lds_get_u64(lbase + (uint32_t)ia * ES) : kEmptyKey;
                } else {
                    ++ib;
                    y = ib < KL ? lds_get_u64(pb + (uint32_t)ib * ES) : kEmptyKey;
                }
            }
            // (each lane's smallest dropped distance: its 10 entries are the
            // lane's best, so every other row it met lies at or above it)
            const uint32_t l9 = (uint32_t)(lds_get_u64(lbase + KL * ES) >> 32);
            const uint32_t p9 = (uint32_t)(lds_get_u64(pb + KL * ES) >> 32);
            const uint32_t ub = std::min(std::min(l9, p9), (uint32_t)((x <= y ? x : y) >> 32));
            out[kBandSlot - 1] = ((uint64_t)ub << 32) | 0xffffffffu;
            if (tenth != kEmptyKey) atomicMin(&a.thr_g[pp], (unsigned long long)tenth);
        }
        if (MODE != 2 && MODE != 3 && h == 0 && live) {
            uint64_t L[KL], P[KL];
            list_load<KL, 0, ES>(lbase, L);
            list_load<KL, 32 * LSTR, ES>(lbase, P);
#pragma unroll
            for (int i = 0; i < KL; ++i) {
                if (P[i] >= L[KL - 1]) break;
                list_insert<KL>(L, P[i]);
            }
            uint64_t* out = a.partial + ((size_t)pp * a.max_chunks + tile.chunk) * KL;
#pragma unroll
            for (int i = 0; i < KL; ++i) out[i] = L[i];
            if (MODE == 0 && L[KL - 1] != kEmptyKey) atomicMin(&a.thr_g[pp], (unsigned long long)L[KL - 1]);
            if (MODE == 1 && L[KL - 1] != kEmptyKey)
                atomicMin(&a.bins[(size_t)pp * a.nbins + tile.chunk % a.nbins], (uint32_t)(L[KL - 1] >> 32));
        }
    }
    if constexpr (ABL != 0) {
        if (tid == 0) {
            const uint64_t clk1 = __builtin_amdgcn_s_memtime();
            const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
            const uint64_t clk0 = clk_lds[0], rt0 = clk_lds[1];
            atomicAdd(&a.dbg[8], (unsigned long long)(clk1 - clk0));
            atomicAdd(&a.dbg[9], (unsigned long long)(rt1 - rt0));
            atomicMin(&a.dbg[10], (unsigned long long)rt0);
            atomicMax(&a.dbg[11], (unsigned long long)rt1);
            atomicAdd(&a.dbg[12], 1ull);
            atomicMax(&a.dbg[13], (unsigned long long)rt0);  // the last workgroup start
            atomicMin(&a.dbg[14], (unsigned long long)rt1);  // the first workgroup end
        }
    }
}

// one launch of the persistent grid (one workgroup per CU, dynamic LDS);
// HIP events around it while lmi_timing_enable is on
template <int KL, int ABL, bool LO = false, int MODE = 0>
int launch_scan3_v(const Scan2Args& b, hipStream_t s) {
    constexpr size_t lds = v3::lds_bytes<KL>();
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [] {
        attr_err = hipFuncSetAttribute((const void*)scan3_kernel<KL, ABL, LO, MODE>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    });
    LMI_HIP_TRY(attr_err);
    const bool timed = timing().on;
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (timed) {
        const int rc = timing_record(s, true, ev);
        if (rc != LMI_OK) return rc;
    }
    hipLaunchKernelGGL((scan3_kernel<KL, ABL, LO, MODE>), dim3(num_cus()), dim3(v3::NW * 64), lds, s, b);
    LMI_LAUNCH_CHECK("scan3_kernel");
    if (timed) return timing_record(s, false, ev);
    return LMI_OK;
}

}  // namespace
}  // namespace lmi
