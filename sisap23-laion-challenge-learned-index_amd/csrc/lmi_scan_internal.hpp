// Internal declarations shared by the K2 scan translation units
// (lmi_scan.hip: prep / plan / scan v3 / chunk merge / host entry points;
// lmi_scan_v12.hip: the round-1 and round-2 scan kernels, kept as fallbacks
// for shapes scan v3 does not take and as A/B baselines).  Not an ABI.
#pragma once
#include "lmi_common.hpp"

#include <mutex>
#include <utility>
#include <vector>

namespace lmi {

using half8 = _Float16 __attribute__((ext_vector_type(8)));
using half4 = _Float16 __attribute__((ext_vector_type(4)));
using f32x16 = float __attribute__((ext_vector_type(16)));
using f32x4 = float __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;  // 4 waves
constexpr int kWaves = 4;
constexpr int kQCap = 16;      // queue entries per lane (= candidates of one 32x32 tile)

struct Tile {
    int32_t c;        // bucket
    int32_t pp0;      // first pair position (into the bucket-grouped pair list)
    int32_t np;       // pairs in this tile (<= QB)
    int32_t chunk;    // chunk index inside the bucket
};

struct ScanArgs {
    const void* corpus;
    int32_t d_pad;
    const float* inv_norm;
    const int64_t* bucket_off;
    int32_t chunk_rows;
    int32_t max_chunks;
    const void* qbuf;       // [nq][d_pad] f16 or f32
    const float* invq;      // [nq]
    const int32_t* pair_q;  // [P] pair id p = q*R + r, grouped by bucket
    int32_t R;
    const Tile* tiles;
    const int32_t* meta;    // tile groups (plan_fill_kernel)
    int32_t* work;          // dequeue counters
    uint64_t* partial;      // [P][max_chunks][KL]
    const int32_t* gpos;    // [n_rows] global positions (LO: ties at the lower bound)
    const unsigned long long* lo_g;  // [nq*R] LO: keep only keys above (d, gpos) of the pair
};


// tail split: at most this many tiles per queue are halved (tail_split_kernel)
constexpr int kSplitMaxK = 256;
constexpr int kSplitMaxParts = 8;
// row parts of a tail-split tile (LMI_SCAN_SPLIT_PARTS, clamped to [2, kSplitMaxParts])
int split_parts();
// tile groups of the persistent scans' dequeue (XCD round-robin, see
// plan_fill_kernel in lmi_scan.hip)
constexpr int kGroups = 8;

// The next tile for a workgroup of group `gx`: its own group first, then steal.
__device__ inline int dequeue_tile(const int32_t* meta, int32_t* work, int gx, int ng) {
    for (int k = 0; k < ng; ++k) {
        const int g = (gx + k) & (ng - 1);
        const int sz = meta[kGroups + g];
        if (__hip_atomic_load(&work[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= sz) continue;
        const int v = atomicAdd(&work[g], 1);
        if (v < sz) return meta[g] + v;
    }
    return -1;
}

// ---------------------------------------------------------------------------
// scan v2 (fp16 corpus, fp16-exact queries, d_pad == 768): queries in
// registers, object rows staged once per workgroup through an LDS ring by
// global_load_lds DMA, shared by the 4 waves (128 queries per staged row).
//
//   per wave : 32 queries; their 48 MFMA B fragments (K = 768) live in VGPRs
//              for the whole tile (192 registers)
//   per stage: 32 object rows x 256 k (16 KiB) + each wave's copy of the 32
//              rows' 1/||y||; 7-slot ring, 4 stages in flight, one raw
//              s_barrier per stage (never __syncthreads inside the ring: its
//              vmcnt(0) would drain the DMA, guide §5 "Pipelining")
//   LDS image: row r, 16-B chunk c stored at chunk c ^ (r & 15) (the XOR
//              is applied to the DMA *source* address, LDS stays lane-linear),
//              so the 32-row A-fragment ds_read_b128 is bank-conflict free
//   per block of 32 rows: 48 x v_mfma_f32_32x32x16_f16 per wave, then the
//              top-k epilogue of v1 with 1/||y|| read from LDS
// A per-pair threshold in global memory (min over the k-th keys published
// by finished tiles of the same pair) seeds every tile's filter.
// ---------------------------------------------------------------------------
namespace v2 {
constexpr int D = 768;
constexpr int KSEG = 256;
constexpr int NST = D / KSEG;          // stages per 32-row block
constexpr int ROWB = KSEG * 2;         // bytes of one row in one stage
constexpr int TRAIL = 4 * 256;         // per-wave copies of the 32 norms
constexpr int STAGE = 32 * ROWB + TRAIL;
constexpr int NSLOT = 7;
constexpr int QB = 128;
constexpr int NQF = D / 16;            // B fragments per lane

template <int KL>
constexpr size_t lds_bytes() {
    return (size_t)NSLOT * STAGE + (size_t)kWaves * 64 * 16 * 8 + 16;
}
}  // namespace v2

// the float64 mode's band lists (scan3_kernel MODE 3): 15 entries + a bound
// per (pair, chunk part)
constexpr int kBandSlot = 16;

struct Scan2Args {
    const _Float16* corpus;
    const float* inv_norm;
    const int64_t* bucket_off;
    int32_t chunk_rows;
    int32_t max_chunks;
    const _Float16* qbuf;
    const float* invq;
    const int32_t* pair_q;
    int32_t R;
    const Tile* tiles;
    const int32_t* meta;
    int32_t* work;
    uint64_t* partial;
    unsigned long long* thr_g;  // [P] per-pair bound, EMPTY at start
    int32_t ng;                 // tile groups (power of two <= kGroups)
    int32_t lag;                // extra ring stages waited for (tuning knob, 0)
    const int32_t* gpos;        // LO: global positions of the rows
    const unsigned long long* lo_g;  // LO: [nq*R] lower-bound key (d, gpos) per pair id
    const int32_t* pair_pos;    // LMI_Q_SEED_ROUND0: [P] grouped position of the pair's (q, 0), -1 if none; else null
    float seed_margin;          //   (distance added to the seed: 2 eps in the float64 mode)
    float band;                 // MODE 3 (the float64 mode's band lists): distance added to the filter bound
    unsigned long long* dbg;    // diagnostic counters of the ABL != 0 variants (lmi_scan_abl.hip); null
    // collect mode (k > 16, scan3_kernel MODE 2): every row of a pair within
    // its fixed bound goes to cand[pp * cap + i], i from ccount[pp] (grouped
    // position pp; a count past cap means the pair overflowed)
    uint64_t* cand;
    uint32_t* ccount;
    int32_t cap;
    // chunk-list mode (MODE 1): nbins distance ordinals per grouped pair, bin
    // j = the smallest 15th entry of the pair's finished chunk lists j mod
    // nbins; their maximum bounds nbins * 15 >= kw entries, so entries above
    // it cannot change the kw-th smallest of the lists (the bound)
    uint32_t* bins;
    int32_t nbins;
    const int32_t* sub_rows;  // MODE 1: [C] rows per list of each bucket (its chunks)
    const int32_t* sub_take;  //   and the rows scanned from the start of each (a sample)
};

// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] + vmcnt[5:4] at [15:14],
// expcnt [6:4], lgkmcnt [11:8]); other counters left at their maximum.
// The builtin (not inline asm) keeps hipcc's wait-count scoreboard in sync,
// so it does not add its own conservative vmcnt waits later in the loop.
constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

// The same value from the partner lane (lane ^ 32): both halves of a 32x32
// accumulator column hold one query.  v_permlane32_swap is a VALU op, so no
// LDS write happens inside the DMA ring (hipcc would drain the LDS-DMA with a
// vmcnt(0) before any LDS write it cannot prove disjoint from the ring).
__device__ __forceinline__ uint32_t partner_u32(uint32_t x, int h) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return h ? r[0] : r[1];
}
__device__ __forceinline__ uint64_t partner_u64(uint64_t x, int h) {
    const uint32_t lo = partner_u32((uint32_t)x, h);
    const uint32_t hi = partner_u32((uint32_t)(x >> 32), h);
    return ((uint64_t)hi << 32) | lo;
}

// LDS destination of the buffer_load ... lds DMA builtins
typedef __attribute__((address_space(3))) void* lds_t;

// Raw LDS accesses at a byte address (no implicit waits beyond the read's own).
__device__ __forceinline__ void lds_put_u64(uint32_t addr, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ uint64_t lds_get_u64(uint32_t addr) {
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

// ---- host side shared by the scan launchers ---------------------------------
int num_cus();

// optional event timing of the scan kernels (lmi_timing_enable / _read)
struct Timing {
    std::mutex mu;
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, pool;
};
Timing& timing();
int timing_record(hipStream_t s, bool start, std::pair<hipEvent_t, hipEvent_t>& pr);

// lmi_scan_v12.hip (explicitly instantiated there for the shapes the host
// dispatch in lmi_scan.hip uses)
template <int KL, bool F16MATH, typename TC, bool LO = false>
int launch_scan(const ScanArgs& a, int d_pad, hipStream_t s);
template <int KL>
int launch_scan2(const Scan2Args& b, hipStream_t s);

}  // namespace lmi
