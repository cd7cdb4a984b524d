// K2 — per-(query, probe) exact top-k inside the probed bucket (gfx950).
//
// Replaces, for every probe r < R of every query, the reference's
//   utils.py:10-11   pairwise_cosine = 1 - sklearn cosine_similarity
//                    (normalize both sides, BLAS GEMM),
//   LearnedIndex.py:170-172  full-row argsort, first k,
//   LearnedIndex.py:152-153, :168  pandas .loc gathers of the bucket rows,
// with one bucket-major pass over the corpus.
//
// Pipeline (all on one stream, no host synchronisation, no allocation):
//   prep_kernel        queries -> fp16 (or fp32) padded rows + 1/||q||;
//                      output lists pre-filled with (+inf, -1)
//   plan_count_kernel  (query, probe) pairs per bucket
//   plan_fill_kernel   pairs grouped by bucket (ascending q), and the tile
//                      list: tile = (bucket, chunk of <= chunk_rows rows,
//                      block of <= QB pairs), chunk-major so the query blocks
//                      that re-read one chunk run back to back (L2 / MALL)
//   scan_kernel        persistent; each workgroup dequeues tiles.  The QB
//                      query rows of a tile sit in LDS; each wave streams
//                      32-row sub-tiles of the chunk from HBM straight into
//                      MFMA A fragments and multiplies them against all QB
//                      queries (v_mfma_f32_32x32x16_f16: exact fp16 products,
//                      fp32 accumulation; or v_mfma_f32_32x32x2_f32 for fp32
//                      data).  The top-k epilogue runs on the accumulators:
//                      d = 1 - dot/(|q||y|), a threshold filter against the
//                      query's current k-th key (shared by all partial lists
//                      of the query through an LDS atomic-min), survivors
//                      appended to a per-lane LDS queue and inserted into a
//                      per-lane register list in lockstep.  At the end of the
//                      tile the 8 partial lists of each query are merged and
//                      written as the tile's chunk list.
//   chunk_merge_kernel per pair: merge its bucket's chunk lists -> top-k,
//                      positions -> global positions.
#include "lmi_scan_internal.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <type_traits>
#include <vector>

// diagnostic hook: defined by lmi_scan_abl.hip in the `make ablation` library
// (the ABL != 0 instantiations of scan3_kernel), absent from the product
extern "C" __attribute__((weak)) int lmi_abl_launch_scan3(int kl, int abl, const void* args,
                                                          void* stream);

namespace lmi {
namespace {

// ---------------------------------------------------------------------------
// prep
// ---------------------------------------------------------------------------
// One wave per query (4 per workgroup: a latency-bound pass over 30 MB at
// 10k queries; round 1's 256-thread workgroup per query took 19 us, most of
// it workgroup launch and block reductions): each lane takes runs of 4
// consecutive elements, float4 loads when the rows allow (VEC).
// Word fills of the plan's per-pair arrays, folded into prep (one kernel
// launch instead of one per array): array f gets value v[f] in words
// [row * per_q[f], (row + 1) * per_q[f]) from the wave of query `row`.
struct PrepFills {
    uint32_t* p[5];
    uint32_t v[5];
    int32_t per_q[5];
    int32_t n;
};

template <bool F16, bool VEC>
__global__ __launch_bounds__(kThreads) void prep_kernel(const float* __restrict__ q, int32_t nq,
                                                        int32_t ldq, int32_t d, int32_t d_pad,
                                                        void* __restrict__ qbuf,
                                                        float* __restrict__ invq,
                                                        int32_t* __restrict__ status,
                                                        float* __restrict__ out_d,
                                                        int32_t* __restrict__ out_pos,
                                                        int32_t* __restrict__ out_row,
                                                        int32_t out_per_q, PrepFills fills) {
    const int row = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= nq) return;  // (wave-uniform; no block-wide barrier below)
    const float* src = q + (size_t)row * ldq;
    float ss = 0.0f;
    bool inexact = false;
    for (int c0 = 4 * lane; c0 < d_pad; c0 += 256) {  // d_pad is a multiple of 32
        float v[4];
        if (VEC && c0 + 3 < d) {
            const float4 f = *reinterpret_cast<const float4*>(src + c0);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (c0 + e < d) ? src[c0 + e] : 0.0f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) ss = fmaf(v[e], v[e], ss);
        if constexpr (F16) {
            _Float16 h[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                h[e] = (_Float16)v[e];
                inexact |= ((float)h[e] != v[e]);
            }
            uint2 pk;
            pk.x = (uint32_t)__builtin_bit_cast(uint16_t, h[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[1]) << 16);
            pk.y = (uint32_t)__builtin_bit_cast(uint16_t, h[2]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[3]) << 16);
            *reinterpret_cast<uint2*>(reinterpret_cast<_Float16*>(qbuf) + (size_t)row * d_pad + c0) = pk;
        } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(qbuf) + (size_t)row * d_pad + c0) =
                make_float4(v[0], v[1], v[2], v[3]);
        }
    }
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    if constexpr (F16) {
        if (__any(inexact) && lane == 0) atomicOr(status, LMI_STATUS_QUERY_NOT_F16);
    }
    if (lane == 0) {
        const float n = sqrtf(ss);
        // sklearn _handle_zeros_in_scale: norms < 10*eps are replaced by 1
        invq[row] = (n < 10.0f * 1.1920929e-07f) ? 1.0f : 1.0f / n;
    }
    for (int e = lane; e < out_per_q; e += 64) {
        out_d[(size_t)row * out_per_q + e] = __builtin_inff();
        out_pos[(size_t)row * out_per_q + e] = -1;
        if (out_row) out_row[(size_t)row * out_per_q + e] = -1;
    }
    for (int f = 0; f < fills.n; ++f)
        for (int e = lane; e < fills.per_q[f]; e += 64)
            fills.p[f][(size_t)row * fills.per_q[f] + e] = fills.v[f];
}

// ---------------------------------------------------------------------------
// plan
// ---------------------------------------------------------------------------
template <int NT = kThreads>
__device__ inline int block_sum(int v, int* sh) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < NT / 64; ++w) t += sh[w];
    return t;
}

// The two plan kernels: one workgroup per bucket reads all P classes, a
// latency-bound pass, so they run 16 waves wide (4x fewer dependent rounds)
constexpr int kPlanThreads = 1024;

__global__ __launch_bounds__(kPlanThreads) void plan_count_kernel(const int32_t* __restrict__ classes,
                                                              int32_t P, int32_t* __restrict__ counts) {
    __shared__ int sh[kPlanThreads / 64];
    const int c = blockIdx.x;
    int n = 0;
    for (int e0 = threadIdx.x; e0 < P; e0 += 8 * kPlanThreads) {  // eight loads in flight
        int v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (e0 + u * kPlanThreads < P) ? classes[e0 + u * kPlanThreads] : -1;
#pragma unroll
        for (int u = 0; u < 8; ++u) n += (v[u] == c) ? 1 : 0;
    }
    n = block_sum<kPlanThreads>(n, sh);
    if (threadIdx.x == 0) counts[c] = n;
}

// Tile list layout (a permutation of all tiles):
//   8 groups, group x = tiles whose global chunk index (chunk_first[c] + j)
//   is = x mod 8; inside a group, every bucket's chunk-0 tiles first, then
//   the other chunks, bucket-major, chunk-major, query-block-minor.
// The persistent scan dequeues from group (blockIdx.x mod 8) — the blocks that
// share an XCD under the observed round-robin placement — and steals from the
// other groups when its own is empty; the query blocks of one chunk therefore
// run back to back on one XCD and re-read the chunk from its L2.  Placement
// only affects speed.  Chunk-0 tiles first: they publish each pair's k-th key
// early, so later chunks start with a tight bound.
//   meta[0..7] group offsets, meta[8..15] group sizes, meta[16] total
//   work[0..7] group dequeue counters, work[8] the single counter of v1
__device__ inline int count_mod(int a, int n, int x, int ng) {
    // #{t in [0, n) : (a + t) mod ng == x}, ng a power of two
    if (n <= 0) return 0;
    const int first = (x - a) & (ng - 1);
    return n / ng + ((first < (n & (ng - 1))) ? 1 : 0);
}

__global__ __launch_bounds__(kPlanThreads) void plan_fill_kernel(
    const int32_t* __restrict__ classes, int32_t P, int32_t C, const int32_t* __restrict__ counts,
    const int32_t* __restrict__ chunk_first, int32_t QB, int32_t* __restrict__ pair_q,
    int32_t* __restrict__ pair_bucket, Tile* __restrict__ tiles, int32_t* __restrict__ meta,
    int32_t* __restrict__ work, int32_t ng, int32_t* __restrict__ pair_pos, int32_t qpad) {
    __shared__ int sh[kPlanThreads / 64];
    __shared__ int wcnt[kPlanThreads / 64];
    __shared__ int g0_all[kGroups], gr_all[kGroups], g0_lt[kGroups], gr_lt[kGroups];
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    if (tid < kGroups) g0_all[tid] = gr_all[tid] = g0_lt[tid] = gr_lt[tid] = 0;
    __syncthreads();
    int off = 0;
    for (int b = tid; b < C; b += kPlanThreads) {
        const int nch = chunk_first[b + 1] - chunk_first[b];
        const int nqb = nch > 0 ? (counts[b] + QB - 1) / QB : 0;
        if (b < c) off += counts[b];
        if (nqb == 0) continue;
        const int cf = chunk_first[b];
        atomicAdd(&g0_all[cf & (ng - 1)], nqb);
        if (b < c) atomicAdd(&g0_lt[cf & (ng - 1)], nqb);
        for (int x = 0; x < ng; ++x) {
            const int r = nqb * count_mod(cf + 1, nch - 1, x, ng);
            if (r) {
                atomicAdd(&gr_all[x], r);
                if (b < c) atomicAdd(&gr_lt[x], r);
            }
        }
    }
    off = block_sum<kPlanThreads>(off, sh);  // (contains the __syncthreads the atomics need)
    int goff[kGroups];
    {
        int acc = 0;
        for (int x = 0; x < kGroups; ++x) {
            goff[x] = acc + x * qpad;  // (each queue region followed by qpad free slots)
            acc += g0_all[x] + gr_all[x];
        }
        if (c == C - 1 && tid == 0) {
            for (int x = 0; x < kGroups; ++x) {
                meta[x] = goff[x];
                meta[kGroups + x] = g0_all[x] + gr_all[x];
                meta[2 * kGroups + 1 + x] = g0_all[x];  // the group's chunk-0 (seed) tiles
                work[x] = 0;
            }
            meta[2 * kGroups] = acc;
            work[kGroups] = 0;
        }
    }
    const int cnt = counts[c];
    const int nch = chunk_first[c + 1] - chunk_first[c];
    const int nqb = (cnt + QB - 1) / QB;
    if (cnt == 0) return;
    // ordered fill of this bucket's pairs (ascending pair id = ascending q):
    // every wave takes a contiguous segment, reads it coalesced (64 pairs per
    // instruction) and ranks its matches by ballot; a wave's base is the
    // count of the segments before it
    {
        const int lane = tid & 63, w = tid >> 6;
        const int seg = ((P + kPlanThreads / 64 - 1) / (kPlanThreads / 64) + 63) & ~63;
        const int sa = min(P, w * seg), sb = min(P, sa + seg);
        constexpr int kU = 8;  // loads in flight per lane (each pass is latency-bound)
        int n = 0;
        for (int e0 = sa; e0 < sb; e0 += kU * 64) {
            int v[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int e = e0 + 64 * u + lane;
                v[u] = e < sb ? classes[e] : -1;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) n += __popcll(__ballot(v[u] == c));
        }
        if (lane == 0) wcnt[w] = n;
        __syncthreads();
        int o = off;
        for (int i = 0; i < w; ++i) o += wcnt[i];
        const uint64_t lt = (1ull << lane) - 1ull;
        for (int e0 = sa; e0 < sb; e0 += kU * 64) {
            int v[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int e = e0 + 64 * u + lane;
                v[u] = e < sb ? classes[e] : -1;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint64_t m = __ballot(v[u] == c);
                if (v[u] == c) {
                    pair_q[o + __popcll(m & lt)] = e0 + 64 * u + lane;
                    pair_bucket[o + __popcll(m & lt)] = c;
                    if (pair_pos) pair_pos[e0 + 64 * u + lane] = o + __popcll(m & lt);
                }
                o += __popcll(m);
            }
        }
    }
    const int cf = chunk_first[c];
    for (int i = tid; i < nch * nqb; i += kPlanThreads) {
        const int j = i / nqb, b = i - j * nqb;
        const int x = (cf + j) & (ng - 1);
        Tile t;
        t.c = c;
        t.pp0 = off + b * QB;
        t.np = min(QB, cnt - b * QB);
        t.chunk = j;
        int pos;
        if (j == 0) {
            pos = goff[x] + g0_lt[x] + b;
        } else {
            // chunks 1 .. j-1 of this bucket that fall in group x, before this one
            pos = goff[x] + g0_all[x] + gr_lt[x] + nqb * count_mod(cf + 1, j - 1, x, ng) + b;
        }
        tiles[pos] = t;
    }
}

// Tail split (scan v3; LMI_SCAN_SPLIT): the last K tiles of every group queue
// are replaced by S row parts each (LMI_SCAN_SPLIT_PARTS, default 2), so the
// launch ends on small tiles.  The scan kernel is unchanged: a part is an
// ordinary tile whose bucket is a virtual entry of an extended bucket table,
// chosen so that the scan's own
//     row0 = off[c] + chunk * chunk_rows,  rows = min(chunk_rows, off[c + 1] - row0)
// give the part's rows, and whose chunk is its partial-list slot: part s of
// chunk j writes slot s*X + j (X = max_chunks, the stride is S*X; part 0 keeps
// chunk j's slot); bit j of mask[pp] tells the chunk merge to read slots
// X + j .. (S-1)*X + j too (chunks j < 32 only).  Every part but the last has
// a whole number of 32-row blocks, and at least two.  In place: plan_fill left
// K (S - 1) free slots after every queue, so only the last K tiles move.
__global__ __launch_bounds__(256) void tail_split_kernel(Tile* __restrict__ tiles,
                                                         int32_t* __restrict__ meta,
                                                         const int64_t* __restrict__ bucket_off,
                                                         int64_t* __restrict__ ext_off, int32_t C,
                                                         int32_t chunk_rows, int32_t X, int32_t K,
                                                         int32_t S, uint32_t* __restrict__ mask) {
    __shared__ int wsp[4];
    __shared__ int s_pp0[256], s_np[256], s_bit[256];  // the split tiles' pair blocks
    const int x = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (x == 0)
        for (int i = tid; i <= C; i += 256) ext_off[i] = bucket_off[i];
    const int o = meta[x], n = meta[kGroups + x];
    const int seeds = meta[2 * kGroups + 1 + x];
    const int k2 = max(0, min(K, n - seeds));  // the candidates: the queue's last k2 tiles
    Tile t{};
    int64_t rs = 0, re = 0;
    bool sp = false;
    if (tid < k2) {
        t = tiles[o + n - k2 + tid];
        rs = bucket_off[t.c] + (int64_t)t.chunk * chunk_rows;
        re = min(rs + (int64_t)chunk_rows, bucket_off[t.c + 1]);
        sp = re - rs >= 2 * 32 * S && t.chunk < 32;
        s_pp0[tid] = t.pp0;
        s_np[tid] = sp ? t.np : 0;
        s_bit[tid] = 1 << (t.chunk & 31);
    }
    const uint64_t m = __ballot(sp);
    if (lane == 0) wsp[w] = __popcll(m);
    __syncthreads();
    int before = __popcll(m & ((1ull << lane) - 1ull)), total = 0;
    for (int v = 0; v < 4; ++v) {
        before += (v < w) ? wsp[v] : 0;
        total += wsp[v];
    }
    if (tid < k2) {
        const int at = o + (n - k2) + tid + before * (S - 1);
        if (!sp) {
            tiles[at] = t;
        } else {
            const int pr = (int)((re - rs) / (32 * S)) * 32;  // rows of every part but the last
            const int v = C + 1 + 2 * S * (x * K + tid);
            for (int p = 0; p < S; ++p) {
                const int64_t a0 = rs + (int64_t)p * pr;
                const int slot = p * X + t.chunk;
                ext_off[v + 2 * p] = a0 - (int64_t)slot * chunk_rows;
                ext_off[v + 2 * p + 1] = (p == S - 1) ? re : a0 + pr;
                tiles[at + p] = Tile{v + 2 * p, t.pp0, t.np, slot};
            }
        }
    }
    // the pairs of every split tile: bit chunk of their mask (the whole
    // workgroup per tile, fire-and-forget atomics)
    for (int i = 0; i < k2; ++i)
        for (int e = tid; e < s_np[i]; e += 256) atomicOr(&mask[s_pp0[i] + e], (uint32_t)s_bit[i]);
    __syncthreads();  // (every thread read meta[x] above)
    if (tid == 0) {
        meta[kGroups + x] = n + total * (S - 1);
        atomicAdd(&meta[2 * kGroups], total * (S - 1));
    }
}

// ---------------------------------------------------------------------------
// nearest-chunk-first plan (scan v3, index with chunk centroids)
//
// Each (query, probe) pair scans every chunk of its bucket; the order only
// decides how early its pruning bound gets tight.  With the bucket's rows
// laid out by sub-cluster (one sub-cluster per chunk), a pair's nearest
// neighbours sit mostly in the chunk whose centroid is nearest, so:
//   pref_kernel       pair -> its nearest chunk (max cosine to the centroid)
//   pref_sort_kernel  the bucket's pairs re-ordered by (nearest chunk, pair),
//                     so a 256-pair tile group shares few nearest chunks
//   tile3_fill_kernel the tile list: one "seed" tile per group first (the
//                     nearest chunk of the group's median pair; they publish
//                     each pair's bound through thr_g), then the rest
//                     chunk-major
// ---------------------------------------------------------------------------
__device__ inline int bucket_pair_off(const int32_t* counts, int c, int* sh) {
    int off = 0;
    for (int b = threadIdx.x; b < c; b += kThreads) off += counts[b];
    return block_sum(off, sh);
}

__global__ __launch_bounds__(kThreads) void pref_kernel(
    const int32_t* __restrict__ pair_bucket, const int32_t* __restrict__ chunk_first,
    const float* __restrict__ centroid, int32_t d_pad, const _Float16* __restrict__ qbuf,
    const int32_t* __restrict__ pair_q, int32_t R, int32_t P, int32_t* __restrict__ pref) {
    // one wave per pair (thousands of waves hide the L2 latency of the loads)
    const int lane = threadIdx.x & 63;
    const int pp = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (pp >= P) return;
    const int c = pair_bucket[pp];
    if (c < 0) return;
    const int c0 = chunk_first[c], nch = chunk_first[c + 1] - c0;
    if (nch <= 1) {
        if (lane == 0) pref[pp] = 0;
        return;
    }
    const _Float16* qr = qbuf + (size_t)(pair_q[pp] / R) * d_pad;
    float best = -3.0f;
    int bj = 0;
    for (int j = 0; j < nch; ++j) {
        const float* cr = centroid + (size_t)(c0 + j) * d_pad;
        float s = 0.0f;
        for (int e = lane; e < d_pad; e += 64) s = fmaf((float)qr[e], cr[e], s);
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (s > best) {  // wave-uniform after the butterfly; ties -> lower chunk
            best = s;
            bj = j;
        }
    }
    if (lane == 0) pref[pp] = bj;
}

__global__ __launch_bounds__(kThreads) void pref_sort_kernel(
    const int32_t* __restrict__ counts, const int32_t* __restrict__ chunk_first,
    int32_t* __restrict__ pair_q, int32_t* __restrict__ pref, int32_t* __restrict__ tmp,
    int32_t* __restrict__ tmp_pref, int32_t QB, int32_t* __restrict__ n_seed) {
    __shared__ int sh[kThreads / 64];
    __shared__ int wcnt[kThreads / 64];
    const int c = blockIdx.x;
    const int off = bucket_pair_off(counts, c, sh);
    const int cnt = counts[c];
    const int nch = chunk_first[c + 1] - chunk_first[c];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (nch <= 1) {  // nothing to order (an empty bucket has no tiles at all)
        if (tid == 0) n_seed[c] = (nch == 1) ? (cnt + QB - 1) / QB : 0;
        return;
    }
    // stable counting sort by pref: one ordered compaction pass per chunk
    int run = 0;
    for (int j = 0; j < nch; ++j) {
        for (int base = 0; base < cnt; base += kThreads) {
            const int e = base + tid;
            const bool pred = (e < cnt) && (pref[off + e] == j);
            const uint64_t m = __ballot(pred);
            const int rank = __popcll(m & ((1ull << lane) - 1ull));
            __syncthreads();
            if (lane == 0) wcnt[w] = __popcll(m);
            __syncthreads();
            int wpre = 0, tot = 0;
            for (int i = 0; i < kThreads / 64; ++i) {
                wpre += (i < w) ? wcnt[i] : 0;
                tot += wcnt[i];
            }
            if (pred) {
                tmp[off + run + wpre + rank] = pair_q[off + e];
                tmp_pref[off + run + wpre + rank] = j;
            }
            run += tot;
        }
    }
    __syncthreads();
    for (int e = tid; e < cnt; e += kThreads) {
        pair_q[off + e] = tmp[off + e];
        pref[off + e] = tmp_pref[off + e];
    }
    // one seed tile per group of QB pairs (see tile3_fill_kernel)
    if (tid == 0) n_seed[c] = (cnt + QB - 1) / QB;
}

__global__ __launch_bounds__(kThreads) void tile3_fill_kernel(
    const int32_t* __restrict__ counts, const int32_t* __restrict__ chunk_first,
    const int32_t* __restrict__ pref, const int32_t* __restrict__ n_seed, int32_t C, int32_t QB,
    Tile* __restrict__ tiles, int32_t* __restrict__ meta, int32_t* __restrict__ work) {
    __shared__ int sh[kThreads / 64];
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    int s_lt = 0, r_lt = 0, s_all = 0, r_all = 0, off = 0;
    for (int b = tid; b < C; b += kThreads) {
        const int nch = chunk_first[b + 1] - chunk_first[b];
        const int ng = nch > 0 ? (counts[b] + QB - 1) / QB : 0;
        const int rest = ng * nch - n_seed[b];
        s_all += n_seed[b];
        r_all += rest;
        if (b < c) {
            s_lt += n_seed[b];
            r_lt += rest;
            off += counts[b];
        }
    }
    s_lt = block_sum(s_lt, sh);
    r_lt = block_sum(r_lt, sh);
    s_all = block_sum(s_all, sh);
    r_all = block_sum(r_all, sh);
    off = block_sum(off, sh);
    if (c == 0 && tid == 0) {
        for (int x = 0; x < kGroups; ++x) {
            meta[x] = 0;
            meta[kGroups + x] = (x == 0) ? s_all + r_all : 0;
            work[x] = 0;
        }
        meta[2 * kGroups] = s_all + r_all;
        work[kGroups] = 0;
    }
    if (tid != 0) return;  // per-bucket tile lists are short: one thread writes them
    const int cnt = counts[c];
    const int nch = chunk_first[c + 1] - chunk_first[c];
    if (cnt == 0 || nch == 0) return;
    // the seed chunk of group g: the nearest chunk of its median pair (the
    // group's pairs are sorted by nearest chunk, so it is the most common one)
    const int ngr = (cnt + QB - 1) / QB;
    int ps = s_lt, pr = s_all + r_lt;
    for (int g = 0; g < ngr; ++g) {
        const int n = min(QB, cnt - g * QB);
        tiles[ps++] = Tile{c, off + g * QB, n, pref[off + g * QB + n / 2]};
    }
    for (int j = 0; j < nch; ++j)
        for (int g = 0; g < ngr; ++g) {
            const int n = min(QB, cnt - g * QB);
            if (j != pref[off + g * QB + n / 2]) tiles[pr++] = Tile{c, off + g * QB, n, j};
        }
}


// LMI_Q_SEED_ROUND0: per grouped pair position pp, the grouped position of
// its round-0 pair (q, 0), or -1 for r = 0 pairs (pair_pos: grouped position
// of every pair id, plan_fill_kernel; pairs of out-of-range classes keep -1)
__global__ __launch_bounds__(256) void seed_pos_kernel(const int32_t* __restrict__ pair_q,
                                                       const int32_t* __restrict__ pair_pos,
                                                       int32_t P, int32_t R,
                                                       int32_t* __restrict__ seed_pos) {
    const int pp = blockIdx.x * 256 + threadIdx.x;
    if (pp >= P) return;
    // (positions past the grouped pairs -- classes out of range -- hold stale
    // pair ids that no tile reads; any id outside [0, P) maps to -1)
    const int p = pair_q[pp];
    seed_pos[pp] = (p < 0 || p >= P || p % R == 0) ? -1 : pair_pos[p - p % R];
}

}  // namespace
}  // namespace lmi

#include "lmi_scan3.hpp"  // scan3_kernel (scan v3) and its helpers

namespace lmi {
namespace {

// ---------------------------------------------------------------------------
// chunk merge
// ---------------------------------------------------------------------------
// kMergeLanes lanes per pair (round 6; was one thread per pair): lane s of a
// pair merges the pair's chunk lists j = s, s + kMergeLanes, ... into a
// register list (each list read with all its loads in flight, then its global
// positions gathered the same way; the next list's keys load while this
// one's positions are gathered), then the lanes' lists are merged by a
// butterfly of shuffles (log2 kMergeLanes rounds: insert the partner lane's
// entries).  Every lane ends with the same list: the KL smallest keys of the
// union, exactly the one-thread merge's.  At 40,000 pairs one thread per pair
// was 625 waves for 1,024 SIMDs -- latency-bound, ~41 us at W = 8 (58 at
// W = 1) on the finish chain's critical path.
constexpr int kMergeLanes = 8;
constexpr int kMergeBlock = 256;

// slot of the pair's j-th list: chunks 0 .. nch_c - 1, then the other parts
// (1 .. S-1) of the tail-split chunks in ascending chunk order (bit b of the
// pair's mask: chunk b was split; part p lives at slot p * X + b)
__device__ inline int chunk_slot(int j, int nch_c, uint32_t sm, int S, int X) {
    if (j < nch_c) return j;
    const int idx = j - nch_c;
    int n = idx / (S - 1);
    const int part = 1 + idx % (S - 1);
    while (n-- > 0) sm &= sm - 1u;
    return part * X + __builtin_ctz(sm);
}

// (the pair's list keys are (distance, local row) in the partial lists and
// (distance, global position) in M; rows inside a chunk ascend in global
// position, so mapping keeps each list ordered and the merge is by the
// reference's (distance, g.index) order)
//
// The merges are bitonic over kMergeN = 16 register slots: two ascending
// lists A, B -> A[i] = min(A[i], B[15 - i]) is bitonic and holds the union's
// 16 smallest; four half-cleaner stages sort it.  48 compare-exchanges a merge
// where inserting a list entry by entry cost up to 16 shifting inserts of 16
// (the band lists' merge, 16 slots, took 2.4x the plain 10-slot merge's time
// at W = 8: ~126 against 53 us after the scan, profiles/r06aj_w8_*_trace.txt).
constexpr int kMergeN = 16;
__device__ inline void bitonic_top(uint64_t (&A)[kMergeN], int32_t (&AW)[kMergeN], const uint64_t (&B)[kMergeN],
                                   const int32_t (&BW)[kMergeN]) {
#pragma unroll
    for (int i = 0; i < kMergeN; ++i) {
        const bool t = B[kMergeN - 1 - i] < A[i];
        A[i] = t ? B[kMergeN - 1 - i] : A[i];
        AW[i] = t ? BW[kMergeN - 1 - i] : AW[i];
    }
#pragma unroll
    for (int d = kMergeN / 2; d > 0; d >>= 1) {
#pragma unroll
        for (int i = 0; i < kMergeN; ++i) {
            if ((i & d) == 0) {
                const uint64_t x = A[i], y = A[i + d];
                const int32_t xw = AW[i], yw = AW[i + d];
                const bool sw = y < x;
                A[i] = sw ? y : x;
                A[i + d] = sw ? x : y;
                AW[i] = sw ? yw : xw;
                AW[i + d] = sw ? xw : yw;
            }
        }
    }
}

// one ascending list K of NE (distance, local row) entries into M (its first
// KL exact): entries past M's KL-th distance are dropped before the gather
template <int KL, int NE>
__device__ inline void merge_chunk_list(const uint64_t (&K)[NE], uint64_t (&M)[kMergeN], int32_t (&W)[kMergeN],
                                        const int32_t* __restrict__ gpos, int64_t n_rows,
                                        int32_t* __restrict__ status) {
    static_assert(NE <= kMergeN && KL <= kMergeN, "merge slots");
    const uint32_t thr = (uint32_t)(M[KL - 1] >> 32);
    uint64_t B[kMergeN];
    int32_t BW[kMergeN];
#pragma unroll
    for (int i = 0; i < kMergeN; ++i) {
        B[i] = kEmptyKey;
        BW[i] = -1;
    }
    int32_t g[NE];
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        const uint32_t lp = (uint32_t)K[i];
        const bool live = K[i] != kEmptyKey && (uint32_t)(K[i] >> 32) <= thr;
        const bool ok = lp < (uint32_t)n_rows;
        if (live && !ok) atomicOr(status, LMI_STATUS_INTERNAL);  // never for a sound scan
        g[i] = (live && ok) ? gpos[lp] : -1;
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        if (g[i] >= 0) {
            B[i] = (K[i] & 0xffffffff00000000ull) | (uint32_t)g[i];
            BW[i] = (int32_t)(uint32_t)K[i];
        }
    }
    bitonic_top(M, W, B, BW);
}

// The lanes of a pair merge their lists (xor butterfly inside the pair's
// kMergeLanes-lane group): after the rounds every lane holds the union's
// kMergeN smallest keys
__device__ inline void merge_lanes(uint64_t (&M)[kMergeN], int32_t (&W)[kMergeN]) {
#pragma unroll
    for (int off = 1; off < kMergeLanes; off <<= 1) {
        uint64_t o[kMergeN];
        int32_t ow[kMergeN];
#pragma unroll
        for (int i = 0; i < kMergeN; ++i) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)M[i], off);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(M[i] >> 32), off);
            o[i] = ((uint64_t)hi << 32) | lo;
            ow[i] = __shfl_xor(W[i], off);
        }
        bitonic_top(M, W, o, ow);
    }
}

// one pair's lists -> the merged list in M/W (every lane of the pair's group);
// NE entries read per list (KL, or the band lists' kBandSlot - 1), the
// list's slot stride LS; BAND: *ub = the smallest of the lists' bound slots
template <int KL, int NE, int LS, bool BAND>
__device__ inline void merge_pair(const uint64_t* __restrict__ partial, int32_t max_chunks, int pp, int nch_c,
                                  uint32_t sm, int S, const int32_t* __restrict__ gpos, int64_t n_rows,
                                  int32_t* __restrict__ status, int sub, uint64_t (&M)[KL], int32_t (&W)[KL],
                                  uint32_t* ub) {
    const int nch = nch_c + (S - 1) * __popc(sm);
    const int X = max_chunks / S;
    uint64_t MM[kMergeN];
    int32_t WW[kMergeN];
#pragma unroll
    for (int i = 0; i < kMergeN; ++i) {
        MM[i] = kEmptyKey;
        WW[i] = -1;
    }
    uint64_t Kn[NE];
    uint32_t ubn = 0xffffffffu;
    auto load = [&](int j) {
        const uint64_t* src = partial + ((size_t)pp * max_chunks + chunk_slot(j, nch_c, sm, S, X)) * LS;
#pragma unroll
        for (int i = 0; i < NE; ++i) Kn[i] = src[i];
        if constexpr (BAND) ubn = (uint32_t)(src[LS - 1] >> 32);
    };
    if (sub < nch) load(sub);
    for (int j = sub; j < nch; j += kMergeLanes) {
        uint64_t K[NE];
#pragma unroll
        for (int i = 0; i < NE; ++i) K[i] = Kn[i];
        if constexpr (BAND) *ub = std::min(*ub, ubn);
        if (j + kMergeLanes < nch) load(j + kMergeLanes);
        merge_chunk_list<KL, NE>(K, MM, WW, gpos, n_rows, status);
    }
    merge_lanes(MM, WW);
#pragma unroll
    for (int i = 0; i < KL; ++i) {
        M[i] = MM[i];
        W[i] = WW[i];
    }
}

template <int KL, bool ROWS>
__global__ __launch_bounds__(kMergeBlock) void chunk_merge_kernel(
    const uint64_t* __restrict__ partial, int32_t max_chunks, const int32_t* __restrict__ pair_q,
    const int32_t* __restrict__ pair_bucket, const int32_t* __restrict__ chunk_first,
    const int32_t* __restrict__ gpos, int32_t P, int32_t k, int32_t ldo, float* __restrict__ out_d,
    int32_t* __restrict__ out_pos, int32_t* __restrict__ out_row, int64_t n_rows,
    int32_t* __restrict__ status, const uint32_t* __restrict__ split_mask, int32_t S) {
    const int gt = blockIdx.x * kMergeBlock + threadIdx.x;
    const int pp = gt / kMergeLanes, sub = gt % kMergeLanes;
    // (a pair's lanes are one aligned group of a wave: they return together)
    if (pp >= P) return;
    const int c = pair_bucket[pp];
    if (c < 0) return;
    const int nch_c = chunk_first[c + 1] - chunk_first[c];
    const uint32_t sm = split_mask != nullptr ? split_mask[pp] : 0u;
    uint64_t M[KL];
    int32_t W[KL];
    merge_pair<KL, KL, KL, false>(partial, max_chunks, pp, nch_c, sm, S, gpos, n_rows, status, sub, M, W,
                                  nullptr);
    const size_t o = (size_t)pair_q[pp] * ldo;
#pragma unroll
    for (int i = 0; i < KL; ++i) {
        if (i < k && i % kMergeLanes == sub) {
            const uint64_t key = M[i];
            const bool empty = key == kEmptyKey;
            out_d[o + i] = empty ? __builtin_inff() : ord2f((uint32_t)(key >> 32));
            out_pos[o + i] = empty ? -1 : (int32_t)(uint32_t)key;
            if constexpr (ROWS) out_row[o + i] = empty ? -1 : W[i];
        }
    }
}

// The float64 mode's band lists (scan3_kernel MODE 3): per pair, its parts'
// 15-entry lists merged to the first 15 by (distance, global position), and
// out_bound[pair id] = the smallest of the parts' bounds and of the merge's
// 16th distance: every row of the pair's shard not in its list either failed
// the scan's widened filter or has d32 >= out_bound (refine_kernel falls back
// to the whole shard when that bound enters the float64 band).
__global__ __launch_bounds__(kMergeBlock) void chunk_merge_band_kernel(
    const uint64_t* __restrict__ partial, int32_t max_chunks, const int32_t* __restrict__ pair_q,
    const int32_t* __restrict__ pair_bucket, const int32_t* __restrict__ chunk_first,
    const int32_t* __restrict__ gpos, int32_t P, int32_t k, int32_t ldo, float* __restrict__ out_d,
    int32_t* __restrict__ out_pos, int32_t* __restrict__ out_row, float* __restrict__ out_bound,
    int64_t n_rows, int32_t* __restrict__ status, const uint32_t* __restrict__ split_mask, int32_t S,
    float* __restrict__ kth_out, int32_t kth_k, const int32_t* __restrict__ classes, int32_t C) {
    constexpr int NB = kBandSlot, KB = kBandSlot - 1;
    const int gt = blockIdx.x * kMergeBlock + threadIdx.x;
    const int pp = gt / kMergeLanes, sub = gt % kMergeLanes;
    if (pp >= P) return;
    // (kth_out of a pair whose class is out of range -- it has no grouped
    // position -- is +inf: lane 1 of grouped position pp takes pair id pp)
    if (kth_out != nullptr && sub == 1) {
        const int cl = classes[pp];
        if (cl < 0 || cl >= C)
            for (int i = 0; i < kth_k; ++i) kth_out[(size_t)pp * kth_k + i] = __builtin_inff();
    }
    const int c = pair_bucket[pp];
    if (c < 0) return;
    const int nch_c = chunk_first[c + 1] - chunk_first[c];
    const uint32_t sm = split_mask != nullptr ? split_mask[pp] : 0u;
    uint64_t M[NB];
    int32_t W[NB];
    uint32_t ub = 0xffffffffu;
    merge_pair<NB, KB, NB, true>(partial, max_chunks, pp, nch_c, sm, S, gpos, n_rows, status, sub, M, W, &ub);
#pragma unroll
    for (int off = 1; off < kMergeLanes; off <<= 1) ub = std::min(ub, (uint32_t)__shfl_xor((int)ub, off));
    ub = std::min(ub, (uint32_t)(M[NB - 1] >> 32));
    const int pid = pair_q[pp];
    const size_t o = (size_t)pid * ldo;
#pragma unroll
    for (int i = 0; i < KB; ++i) {
        if (i < k && i % kMergeLanes == sub) {
            const uint64_t key = M[i];
            const bool empty = key == kEmptyKey;
            const float dv = empty ? __builtin_inff() : ord2f((uint32_t)(key >> 32));
            out_d[o + i] = dv;
            out_pos[o + i] = empty ? -1 : (int32_t)(uint32_t)key;
            out_row[o + i] = empty ? -1 : W[i];
            if (kth_out != nullptr && i < kth_k) kth_out[(size_t)pid * kth_k + i] = dv;
        }
    }
    if (sub == 0) out_bound[pid] = ub == 0xffffffffu ? __builtin_inff() : ord2f(ub);
}

// ---------------------------------------------------------------------------
// k > 16: lower-bound passes
// ---------------------------------------------------------------------------
// After pass j (entries [j*kp, (j+1)*kp) of every pair's list): the next
// pass's lower bound is the (distance, global position) key of the pass's last
// entry; a pair whose pass came back short is exhausted (a key above every
// real key: nothing passes).
__global__ __launch_bounds__(256) void next_lo_kernel(const float* __restrict__ d,
                                                      const int32_t* __restrict__ pos, int32_t P,
                                                      int32_t ldo, int32_t last,
                                                      unsigned long long* __restrict__ lo) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    const size_t o = (size_t)p * ldo + last;
    const int32_t g = pos[o];
    lo[p] = g < 0 ? ~0ull : (((unsigned long long)f2ord(d[o]) << 32) | (uint32_t)g);
}

// ---------------------------------------------------------------------------
// k > 16: bound + collect (bucket_topk_wide)
// ---------------------------------------------------------------------------
// slot of the j-th list of a pair in the partial lists: chunks first, then
// parts 1..S-1 of every split chunk (bit of sm) in ascending order (the order
// chunk_merge_kernel reads them in; X = max_chunks / S)
__device__ inline int wide_slot(int j, int nch_c, uint32_t sm, int S, int X) {
    if (j < nch_c) return j;
    const int jj = j - nch_c;
    int nth = jj / (S - 1);
    const int part = 1 + jj % (S - 1);
    for (; nth > 0; --nth) sm &= sm - 1u;
    return part * X + __builtin_ctz(sm);
}

// The bound pass's lists (one workgroup): bucket c of n_c rows gets L =
// min(lists, n_c / 32) lists of r_c = n_c / L rows (up to a multiple of 32),
// each scanning its first take_c = max(128, r_c / 4) rows (a sample); chunk_first
// is the prefix of the list counts (a thread per contiguous run of buckets, then
// a prefix over the threads).
__global__ __launch_bounds__(256) void bound_lists_kernel(const int64_t* __restrict__ bucket_off, int32_t C,
                                                          int32_t lists, int32_t* __restrict__ chunk_first,
                                                          int32_t* __restrict__ sub_rows,
                                                          int32_t* __restrict__ sub_take) {
    __shared__ int32_t part[256];
    const int t = threadIdx.x;
    const int per = (C + 255) / 256;
    const int c0 = min(C, t * per), c1 = min(C, c0 + per);
    auto count = [&](int c) {
        const int64_t n = bucket_off[c + 1] - bucket_off[c];
        if (n <= 0) return 0;
        const int64_t L = std::max<int64_t>(1, std::min<int64_t>(lists, n / 32));
        const int64_t r = (n + L - 1) / L;
        const int32_t rr = (int32_t)((r + 31) / 32 * 32);
        sub_rows[c] = rr;
        sub_take[c] = std::min(rr, std::max(128, (rr / 4 + 31) / 32 * 32));
        return (int)((n + rr - 1) / rr);
    };
    int32_t acc = 0;
    for (int c = c0; c < c1; ++c) acc += count(c);
    part[t] = acc;
    __syncthreads();
    if (t == 0) {
        int32_t run = 0;
        for (int i = 0; i < 256; ++i) {
            const int32_t v = part[i];
            part[i] = run;
            run += v;
        }
    }
    __syncthreads();
    acc = part[t];
    for (int c = c0; c < c1; ++c) {
        chunk_first[c] = acc;
        const int64_t n = bucket_off[c + 1] - bucket_off[c];
        acc += n <= 0 ? 0 : (int32_t)((n + sub_rows[c] - 1) / sub_rows[c]);
    }
    if (c0 < C && c1 == C) chunk_first[C] = acc;
}

// outputs padded (+inf, -1), bounds and the fix-up flags cleared
__global__ __launch_bounds__(256) void wide_init_kernel(int64_t P, int32_t ldo, float* __restrict__ d,
                                                        int32_t* __restrict__ pos, int32_t* __restrict__ row,
                                                        uint32_t* __restrict__ bound_ord,
                                                        int32_t* __restrict__ fix) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < P * ldo) {
        d[t] = __builtin_inff();
        pos[t] = -1;
        if (row) row[t] = -1;
    }
    if (t < P) {
        bound_ord[t] = 0u;
        fix[t] = 0;
    }
}

// Per grouped pair of the chunk-list scan (one 64-lane workgroup): the kw-th
// smallest distance ordinal over its chunk lists (each the part's own top-15,
// so at least kw rows lie within it) by a 4-digit radix select; fewer than
// kw entries: no bound, the pair goes to the fix-up passes.
__global__ __launch_bounds__(64) void kth_bound_kernel(
    const uint64_t* __restrict__ partial, int32_t max_chunks, int32_t S,
    const int32_t* __restrict__ pair_q, const int32_t* __restrict__ pair_bucket,
    const int32_t* __restrict__ chunk_first, const uint32_t* __restrict__ split_mask, int32_t P,
    int32_t kw, const int64_t* __restrict__ bucket_off, int32_t cap, uint32_t* __restrict__ bound_ord,
    int32_t* __restrict__ fix) {
    constexpr int KL = 15;
    const int pp = blockIdx.x;
    const int c = pair_bucket[pp];
    if (c < 0) return;
    const int p = pair_q[pp];
    if (p < 0 || p >= P) return;
    const uint32_t sm = split_mask != nullptr ? split_mask[pp] : 0u;
    const int nch_c = chunk_first[c + 1] - chunk_first[c];
    const int nl = nch_c + (S - 1) * __popc(sm);
    const int X = max_chunks / S;
    const uint64_t* base = partial + (size_t)pp * max_chunks * KL;
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_prefix, s_mask, s_rem, s_n;
    const int tid = threadIdx.x;
    if (tid == 0) s_n = 0u;
    __syncthreads();
    uint32_t n = 0;
    for (int e = tid; e < nl * KL; e += 64) {
        const uint64_t key = base[(size_t)wide_slot(e / KL, nch_c, sm, S, X) * KL + e % KL];
        n += key != kEmptyKey ? 1u : 0u;
    }
    atomicAdd(&s_n, n);
    if (tid == 0) {
        s_prefix = 0u;
        s_mask = 0u;
        s_rem = (uint32_t)kw;
    }
    __syncthreads();
    if (s_n < (uint32_t)kw) {
        // too few list entries: a bucket of no more rows than the slots is
        // collected whole (no bound), else the pair takes the fix-up passes
        // (bound_ord stays 0: the collect takes nothing)
        if (tid == 0) {
            if (bucket_off[c + 1] - bucket_off[c] <= cap) bound_ord[p] = 0xffffffffu;
            else fix[p] = 1;
        }
        return;
    }
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = tid; i < 256; i += 64) hist[i] = 0u;
        __syncthreads();
        const uint32_t prefix = s_prefix, mask = s_mask;
        for (int e = tid; e < nl * KL; e += 64) {
            const uint64_t key = base[(size_t)wide_slot(e / KL, nch_c, sm, S, X) * KL + e % KL];
            const uint32_t h = (uint32_t)(key >> 32);
            if (key != kEmptyKey && (h & mask) == prefix) atomicAdd(&hist[(h >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t rem = s_rem, dg = 0;
            for (; dg < 255u && hist[dg] < rem; ++dg) rem -= hist[dg];
            s_rem = rem;
            s_prefix = prefix | (dg << shift);
            s_mask = mask | (255u << shift);
        }
        __syncthreads();
    }
    if (tid == 0) bound_ord[p] = s_prefix;
}

// the collect scan's per-grouped-pair bound (thr_g: the distance ordinal in
// the high word) and candidate count; a pair whose bucket has skipped rows in
// front of it (WideScan::app_d) starts with the skipped rows' own list
__global__ __launch_bounds__(256) void set_bound_kernel(const int32_t* __restrict__ pair_q, int32_t P,
                                                        const uint32_t* __restrict__ bound_ord,
                                                        unsigned long long* __restrict__ thr_g,
                                                        uint32_t* __restrict__ ccount,
                                                        const int32_t* __restrict__ pair_bucket,
                                                        const int64_t* __restrict__ bucket_off,
                                                        const float* __restrict__ app_d,
                                                        const int32_t* __restrict__ app_row, int32_t app_k,
                                                        uint64_t* __restrict__ cand, int32_t cap) {
    const int pp = blockIdx.x * 256 + threadIdx.x;
    if (pp >= P) return;
    const int p = pair_q[pp];
    const uint32_t b = (p < 0 || p >= P) ? 0u : bound_ord[p];
    thr_g[pp] = ((unsigned long long)b << 32) | 0xffffffffull;
    uint32_t n = 0u;
    const int c = pair_bucket[pp];
    if (app_d && b != 0u && c > 0 && (c & 1) && bucket_off[c - 1] < bucket_off[c]) {
        for (int i = 0; i < app_k && (int)n < cap; ++i) {
            const float dv = app_d[(size_t)p * app_k + i];
            const int32_t r = app_row[(size_t)p * app_k + i];
            if (r < 0 || !(dv < __builtin_inff())) continue;
            cand[(size_t)pp * cap + n++] = ((uint64_t)f2ord(dv) << 32) | (uint32_t)r;
        }
    }
    ccount[pp] = n;
}

// Per grouped pair of the collect scan (one 256-lane workgroup): its
// candidates sorted by (distance, row) -- rows ascend with global position
// inside a bucket, so this is the reference's (distance, g.index) order --
// and the first kw written as (d, global position, row).  A pair whose
// candidates overflowed (or, never for a sound scan, came back short) goes to
// the fix-up passes.
__global__ __launch_bounds__(256) void collect_select_kernel(
    const uint64_t* __restrict__ cand, const uint32_t* __restrict__ ccount, int32_t cap,
    const int32_t* __restrict__ pair_q, const int32_t* __restrict__ pair_bucket,
    const int32_t* __restrict__ gpos, int32_t P, int32_t kw, int32_t ldo,
    const uint32_t* __restrict__ bound_ord, int32_t* __restrict__ fix, float* __restrict__ out_d,
    int32_t* __restrict__ out_pos, int32_t* __restrict__ out_row) {
    extern __shared__ uint64_t keys[];
    const int pp = blockIdx.x;
    if (pair_bucket[pp] < 0) return;
    const int p = pair_q[pp];
    if (p < 0 || p >= P || fix[p]) return;
    const uint32_t n = ccount[pp];
    const int tid = threadIdx.x;
    // (fewer than kw: only a bucket collected whole, every row under the
    // all-ones bound; never for a sound scan otherwise)
    if (n > (uint32_t)cap || (n < (uint32_t)kw && bound_ord[p] != 0xffffffffu)) {
        if (tid == 0) fix[p] = 1;
        return;
    }
    uint32_t m = 1;
    while (m < n) m <<= 1;
    const uint64_t* src = cand + (size_t)pp * cap;
    for (uint32_t i = tid; i < m; i += 256) keys[i] = i < n ? src[i] : kEmptyKey;
    __syncthreads();
    for (uint32_t k2 = 2; k2 <= m; k2 <<= 1) {
        for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
            for (uint32_t i = tid; i < m; i += 256) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t x = keys[i], y = keys[l];
                    const bool up = (i & k2) == 0;
                    if ((x > y) == up) {
                        keys[i] = y;
                        keys[l] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    const size_t o = (size_t)p * ldo;
    for (int i = tid; i < kw && i < (int)n; i += 256) {
        const uint64_t key = keys[i];
        const uint32_t r = (uint32_t)key;
        out_d[o + i] = ord2f((uint32_t)(key >> 32));
        out_pos[o + i] = gpos[r];
        if (out_row) out_row[o + i] = (int32_t)r;
    }
}

// the fix-up passes' classes: the pair's class where it needs them, else -1
// (out of range: the plan skips the pair)
__global__ __launch_bounds__(256) void fix_classes_kernel(const int32_t* __restrict__ classes,
                                                          const int32_t* __restrict__ fix, int32_t P,
                                                          int32_t* __restrict__ cls_fix) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p < P) cls_fix[p] = fix[p] ? classes[p] : -1;
}

// the fix-up passes' lists over the outputs of the pairs that took them
__global__ __launch_bounds__(256) void fix_combine_kernel(const int32_t* __restrict__ fix, int64_t P,
                                                          int32_t ldo, const float* __restrict__ fd,
                                                          const int32_t* __restrict__ fpos,
                                                          const int32_t* __restrict__ frow,
                                                          float* __restrict__ d, int32_t* __restrict__ pos,
                                                          int32_t* __restrict__ row) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= P * ldo) return;
    if (!fix[t / ldo]) return;
    d[t] = fd[t];
    pos[t] = fpos[t];
    if (row) row[t] = frow[t];
}

// first k of every pair's pass list -> the caller's [P][k] outputs
__global__ __launch_bounds__(256) void take_k_kernel(const float* __restrict__ d,
                                                     const int32_t* __restrict__ pos, int64_t P,
                                                     int32_t ldo, int32_t k, float* __restrict__ out_d,
                                                     int32_t* __restrict__ out_pos) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= P * k) return;
    const int64_t p = t / k;
    const int j = (int)(t - p * k);
    out_d[t] = d[(size_t)p * ldo + j];
    out_pos[t] = pos[(size_t)p * ldo + j];
}

// ---------------------------------------------------------------------------
// the split mode (ABI 9, idx->corpus32; bucket_topk_x below)
// ---------------------------------------------------------------------------
// One wave per query: q^ = q / |q| (float64 norm, sklearn's zero rule) rounded
// to fp16, written as float32 rows of d_pad (zero-padded) -- the fp16-exact
// queries the fp16 scan takes; float64 queries (q64) are rounded the same way.
__global__ __launch_bounds__(kThreads) void x_round_queries_kernel(const float* __restrict__ q, int32_t ldq,
                                                                   const double* __restrict__ q64,
                                                                   int32_t ldq64, int32_t nq, int32_t d,
                                                                   int32_t d_pad, float* __restrict__ out) {
    const int row = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= nq) return;
    double ss = 0.0;
    for (int e = lane; e < d; e += 64) {
        const double v = q64 ? q64[(size_t)row * ldq64 + e] : (double)q[(size_t)row * ldq + e];
        ss = fma(v, v, ss);
    }
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    double n = sqrt(ss);
    if (n < 10.0 * 1.1920928955078125e-07) n = 1.0;
    for (int e = lane; e < d_pad; e += 64) {
        float h = 0.0f;
        if (e < d) {
            const double v = q64 ? q64[(size_t)row * ldq64 + e] : (double)q[(size_t)row * ldq + e];
            h = (float)(_Float16)(float)(v / n);
        }
        out[(size_t)row * d_pad + e] = h;
    }
}

// (+inf, -1) over every output entry (pairs whose class is out of range keep it)
__global__ __launch_bounds__(256) void x_prefill_kernel(int64_t n, void* __restrict__ out_d, int32_t out_f64,
                                                        int32_t* __restrict__ out_pos) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n) return;
    if (out_f64) reinterpret_cast<double*>(out_d)[t] = __builtin_inf();
    else reinterpret_cast<float*>(out_d)[t] = __builtin_inff();
    out_pos[t] = -1;
}

// Per pair (by id): the collect bound d~_k + 2 eps as a distance ordinal,
// rounded up (every row whose rounded distance is at most the real sum
// passes); a list with fewer than k entries (a bucket shard of fewer rows)
// collects its whole shard.
__global__ __launch_bounds__(256) void x_bound_kernel(int64_t P, int32_t k, const float* __restrict__ ld,
                                                      double two_eps, uint32_t* __restrict__ bound_ord) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    const float dk = ld[(size_t)p * k + k - 1];
    if (!(dk < __builtin_inff())) {
        bound_ord[p] = 0xffffffffu;
        return;
    }
    const double b = (double)dk + two_eps;
    const float f = (float)b;
    // (the ordinal of the next float up when the float rounded the sum down)
    bound_ord[p] = f2ord(f) + ((double)f < b ? 1u : 0u);
}

// The split mode's sampled bound (k <= 15): the kw-th distance ordinal of the
// pair's sampled lists (kth_bound_kernel) + 2 eps, rounded up; all ones (a
// bucket collected whole) and 0 (no bound: fix[p], the whole shard exactly)
// stay as they are.
__global__ __launch_bounds__(256) void x_margin_kernel(int64_t P, double two_eps, uint32_t* __restrict__ bound_ord) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    const uint32_t b = bound_ord[p];
    if (b == 0u || b == 0xffffffffu) return;
    const double v = (double)ord2f(b) + two_eps;
    const float f = (float)v;
    bound_ord[p] = f2ord(f) + ((double)f < v ? 1u : 0u);
}

// The split mode's sample (k <= 10): a descriptor of 2C buckets over the same
// rows -- bucket 2c = the first s_c rows of bucket c, s_c = min(n_c,
// max(chunk_rows, n_c / kXSampleDiv rounded up to 32 rows)), bucket 2c + 1 =
// the rest (no chunks, never probed) -- so the product scan gives every pair
// the k-th of its bucket's sample, an upper bound of its own (and the collect
// then finds about k n_c / s_c <= k kXSampleDiv rows under it, far inside
// its buffer at any bucket size).
//
// The collect scan's descriptor (x_collect_desc) skips the sample where it is
// at most a quarter of the bucket (LMI_X_SKIP_SHARE): bucket 2c = the sample (no chunks, never
// probed), 2c + 1 = the rest; a bucket with a larger sample is collected whole
// (2c empty, 2c + 1 = the bucket).  The skipped rows' candidates are the
// sample scan's own list (set_bound_kernel appends it): every skipped row the
// select needs is in it unless the pair's band reaches the sample's k-th
// (x_select_wave_kernel checks; 0.03% of the pairs on the 10M mixture,
// tools/x_sample_cover.py), and those pairs are scored exactly over their
// sample rows and candidates (x_fallback_kernel).
constexpr int kXSampleDiv = 16;
__global__ __launch_bounds__(64) void x_sample_desc_kernel(const int64_t* __restrict__ bucket_off, int32_t C,
                                                           int64_t chunk_rows, const int32_t* __restrict__ classes,
                                                           int32_t P, int64_t* __restrict__ off2,
                                                           int32_t* __restrict__ cf2, int32_t* __restrict__ classes2,
                                                           int64_t* __restrict__ off2b, int32_t* __restrict__ cf2b,
                                                           int32_t* __restrict__ classes2b, int32_t skip_share) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int32_t nch = 0, nchb = 0;
        for (int c = 0; c < C; ++c) {
            const int64_t a = bucket_off[c], n = bucket_off[c + 1] - a;
            const int64_t want = std::max(chunk_rows, (n / kXSampleDiv + 31) / 32 * 32);
            const int64_t sc = n < want ? n : want;
            off2[2 * c] = a;
            off2[2 * c + 1] = a + sc;
            cf2[2 * c] = nch;
            nch += (int32_t)((sc + chunk_rows - 1) / chunk_rows);
            cf2[2 * c + 1] = nch;
            // (a sample of at most 1 / skip_share of the bucket, LMI_X_SKIP_SHARE)
            const int64_t skip = (skip_share > 0 && sc < n && sc * skip_share <= n) ? sc : 0;
            off2b[2 * c] = a;
            off2b[2 * c + 1] = a + skip;
            cf2b[2 * c] = nchb;
            cf2b[2 * c + 1] = nchb;
            nchb += (int32_t)((n - skip + chunk_rows - 1) / chunk_rows);
        }
        off2[2 * C] = bucket_off[C];
        cf2[2 * C] = nch;
        off2b[2 * C] = bucket_off[C];
        cf2b[2 * C] = nchb;
    }
    for (int i = blockIdx.x * 64 + threadIdx.x; i < P; i += gridDim.x * 64) {
        const int32_t c = classes[i];
        classes2[i] = c < 0 ? c : (c < C ? 2 * c : 2 * C);
        classes2b[i] = c < 0 ? c : (c < C ? 2 * c + 1 : 2 * C);
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct WsLayout {
    size_t qbuf, invq, counts, pair_q, pair_bucket, tiles, ntiles, work, partial, thr_g, pref,
        pref_tmp, pref_tmp2, n_seed, total;
    int32_t max_tiles;
    size_t ext_off, split_mask;  // tail split (scan v3)
    size_t pair_pos;  // LMI_Q_SEED_ROUND0: grouped position of every pair id
    size_t seed_pos;  //   and of every grouped pair's (q, 0)
    int32_t qb;      // queries per tile
    bool use_v2;     // scan2_kernel
    bool use_v3;     // scan3_kernel
    int32_t split_s; // row parts of a tail-split chunk (1: the tail split is off)
};

bool v2_eligible(const lmi_index_desc* idx, int qmode) {
    if (env_config().scan_v1) return false;  // diagnostic switch: force the general kernel
    return idx->dtype == LMI_F16 && qmode == LMI_Q_F16 && idx->d_pad == v2::D;
}

bool v3_capable(const lmi_index_desc* idx, int qmode) {
    if (env_config().scan_v2) return false;  // diagnostic switch: force the 4-wave ring
    return v2_eligible(idx, qmode);
}

// list length of the scan: 10 (k <= 10), 15 (k <= 15 on scan v3: the float64
// mode's 10 + 5 guard entries), else 16
int pick_kl(const lmi_index_desc* idx, int qmode, int k) {
    if (k <= 10) return 10;
    if (k <= 15 && v3_capable(idx, qmode)) return 15;
    return 16;
}

bool v3_eligible(const lmi_index_desc* idx, int qmode, int k) {
    const int kl = pick_kl(idx, qmode, k);
    return v3_capable(idx, qmode) && (kl == 10 || kl == 15);
}

WsLayout ws_layout(const lmi_index_desc* idx, int nq, int R, int k, int qmode, bool lo = false) {
    WsLayout w{};
    const int KL = pick_kl(idx, qmode, k);
    const bool f16math = (idx->dtype == LMI_F16) && (qmode == LMI_Q_F16);
    w.use_v3 = v3_eligible(idx, qmode, k);
    // the lower-bound passes (k > 16) run on v3 or the general kernel
    w.use_v2 = !w.use_v3 && !lo && v2_eligible(idx, qmode);
    const int QB = w.use_v3 ? v3::QB : w.use_v2 ? v2::QB : (f16math ? 64 : 32);
    w.qb = QB;
    const size_t P = (size_t)nq * R;
    const size_t esz = f16math ? 2 : 4;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t at = off;
        off = align_up(off + bytes, 256);
        return at;
    };
    w.qbuf = take((size_t)nq * idx->d_pad * esz);
    w.invq = take((size_t)nq * 4);
    w.counts = take((size_t)idx->n_buckets * 4);
    w.pair_q = take(P * 4);
    w.pair_bucket = take(P * 4);
    // tiles <= sum_c nch_c * ceil(cnt_c/QB) <= sum_c nch_c * (cnt_c/QB + 1)
    const size_t mt = (P / QB + 1) * (size_t)std::max(idx->max_chunks, 1) + (size_t)idx->n_chunks;
    w.max_tiles = (int32_t)std::min<size_t>(mt, (size_t)INT32_MAX);
    // (+ K (S - 1) free slots after every queue: the tail split's parts, in
    // place; S = 1 when the split is off: not scan v3, the nearest-chunk-first
    // plan, or LMI_SCAN_SPLIT < 0 -- the same predicate as bucket_topk_impl's
    // split_k)
    const bool nearest_first = w.use_v3 && idx->chunk_centroid && !env_config().scan_no_pref;
    const bool split_on = w.use_v3 && !nearest_first && env_config().scan_split >= 0;
    w.split_s = split_on ? split_parts() : 1;
    // (the buffers are sized for split_parts() on scan v3 whether the split
    // is on or not, so the total and every offset do not depend on the
    // LMI_SCAN_SPLIT / LMI_SCAN_NO_PREF knobs or on the index's centroids:
    // a workspace sized once fits every call)
    const size_t S = w.use_v3 ? (size_t)split_parts() : 1;
    w.tiles = take(((size_t)w.max_tiles + (size_t)kGroups * kSplitMaxK * (S - 1)) * sizeof(Tile));
    w.ntiles = take(4 * (3 * kGroups + 1));
    w.work = take(4 * (kGroups + 1));
    // (x S: the other parts of tail-split chunks, slot s * max_chunks + j)
    // (15-entry lists: room for the float64 mode's band slots, kBandSlot)
    w.partial = take(P * (size_t)(S * std::max(idx->max_chunks, 1)) * (KL == 15 ? kBandSlot : KL) *
                     sizeof(uint64_t));
    w.ext_off = take(((size_t)idx->n_buckets + 1 + 2 * S * (size_t)kGroups * kSplitMaxK) * 8);
    w.split_mask = take(P * 4);
    w.thr_g = take(P * sizeof(uint64_t));
    w.pref = take(P * 4);
    w.pref_tmp = take(P * 4);
    w.pref_tmp2 = take(P * 4);
    w.n_seed = take((size_t)idx->n_buckets * 4);
    w.pair_pos = take(P * 4);
    w.seed_pos = take(P * 4);
    w.total = off;
    return w;
}

}  // namespace

bool band_capable(const lmi_index_desc* idx, int qmode) { return v3_capable(idx, qmode); }

int split_parts() {
    return std::max(2, std::min(kSplitMaxParts, env_config().scan_split_parts));
}

namespace {
thread_local int t_scan_wgs = 0;  // lmi_scan_set_workgroups (0: env / every CU)
}  // namespace

int num_cus() {
    static int n = 0;
    static std::once_flag once;
    std::call_once(once, [] {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 256;
    });
    const int cus = n > 0 ? n : 256;
    const int w = t_scan_wgs > 0 ? t_scan_wgs : env_config().scan_wgs;
    return w > 0 ? std::min(w, cus) : cus;
}

// ---- optional event timing of the scan kernel ------------------------------
Timing& timing() {
    static Timing t;
    return t;
}

int timing_record(hipStream_t s, bool start, std::pair<hipEvent_t, hipEvent_t>& pr) {
    if (start) {
        Timing& t = timing();
        std::lock_guard<std::mutex> g(t.mu);
        if (!t.pool.empty()) {
            pr = t.pool.back();
            t.pool.pop_back();
        } else {
            LMI_HIP_TRY(hipEventCreate(&pr.first));
            LMI_HIP_TRY(hipEventCreate(&pr.second));
        }
        LMI_HIP_TRY(hipEventRecord(pr.first, s));
    } else {
        LMI_HIP_TRY(hipEventRecord(pr.second, s));
        Timing& t = timing();
        std::lock_guard<std::mutex> g(t.mu);
        t.pending.push_back(pr);
    }
    return LMI_OK;
}

namespace {

template <int KL>
int launch_scan3(const Scan2Args& b, hipStream_t s) {
    // the diagnostic variants (LMI_SCAN_ABL) live in lmi_scan_abl.hip, linked
    // only into the `make ablation` library; the product ignores the switch
    const int abl = env_config().scan_abl;
    if (abl != 0 && lmi_abl_launch_scan3 != nullptr) return lmi_abl_launch_scan3(KL, abl, &b, s);
    return launch_scan3_v<KL, 0>(b, s);
}

}  // namespace
}  // namespace lmi

extern "C" int32_t lmi_plan_chunks(const int64_t* bucket_off_host, int32_t n_buckets,
                                   int32_t chunk_rows, int32_t* chunk_first_out) {
    using namespace lmi;
    if (!bucket_off_host || !chunk_first_out || n_buckets < 1 || chunk_rows < 32 || chunk_rows % 32) {
        set_error("lmi_plan_chunks: bad arguments");
        return -LMI_E_INVALID;
    }
    int32_t maxc = 0;
    int64_t acc = 0;
    for (int c = 0; c < n_buckets; ++c) {
        chunk_first_out[c] = (int32_t)acc;
        const int64_t n = bucket_off_host[c + 1] - bucket_off_host[c];
        if (n < 0) {
            set_error("lmi_plan_chunks: bucket offsets not ascending at %d", c);
            return -LMI_E_INVALID;
        }
        const int64_t nch = (n + chunk_rows - 1) / chunk_rows;
        maxc = std::max<int32_t>(maxc, (int32_t)nch);
        acc += nch;
    }
    chunk_first_out[n_buckets] = (int32_t)acc;
    return maxc;
}

size_t lmi::scan_workspace_bytes(const lmi_index_desc* idx, int32_t nq, int32_t R, int32_t k,
                                 int32_t qmode, bool lo) {
    if (!idx || nq < 0 || R < 1 || k < 1) return 0;
    return lmi::ws_layout(idx, nq, R, k, qmode, lo).total;
}

extern "C" size_t lmi_scan_workspace_bytes(const lmi_index_desc* idx, int32_t nq, int32_t R,
                                           int32_t k, int32_t qmode) {
    using namespace lmi;
    qmode &= ~LMI_Q_SEED_ROUND0;
    take_phases(qmode);
    if (!idx || nq < 0 || R < 1 || k < 1 || k > LMI_MAX_K_PASSES) return 0;
    if (idx->corpus32) return k <= LMI_MAX_K ? x_ws_bytes(idx, nq, R, k) : 0;
    if (k <= LMI_MAX_K) return scan_workspace_bytes(idx, nq, R, k, qmode);
    int kp;
    const int ldo = passes_of(idx, qmode, k, &kp) * kp;
    return 2 * align_up((size_t)nq * R * ldo * 4, 256) + wide_ws_bytes(idx, nq, R, k, qmode, ldo);
}

namespace {
// tuning knobs (defaults are the tuned values; results do not depend on them)
int clamp_knob(int v, int dflt, int lo, int hi) { return v == 0 && dflt != 0 ? dflt : std::max(lo, std::min(hi, v)); }
}  // namespace

extern "C" int lmi_bucket_topk(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                               const int32_t* classes, int32_t R, int32_t k, int32_t qmode,
                               float* out_d, int32_t* out_pos, int32_t* status, void* workspace,
                               size_t ws_bytes, void* stream) {
    using namespace lmi;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool seed = (qmode & LMI_Q_SEED_ROUND0) != 0;
    qmode &= ~LMI_Q_SEED_ROUND0;
    const int phases = take_phases(qmode);
    if (idx && idx->corpus32)  // (phases: k <= 10, ABI 11)
        return bucket_topk_x(idx, q, nq, ldq, nullptr, 0, classes, R, k, out_d, 0, out_pos, status, workspace,
                             ws_bytes, s, phases);
    if (k <= LMI_MAX_K)
        return bucket_topk_impl(idx, q, nq, ldq, classes, R, k, qmode, out_d, out_pos, nullptr,
                                status, workspace, ws_bytes, s, nullptr, 0, true, seed, 0.0f, phases);
    if (phases != kPhaseAll) {
        set_error("phase flags need k <= %d (one scan pass)", LMI_MAX_K);
        return LMI_E_UNSUPPORTED;
    }
    LMI_CHECK_ARG(idx != nullptr, "null index");
    LMI_CHECK_ARG(k <= LMI_MAX_K_PASSES, "k=%d outside [1, %d]", k, LMI_MAX_K_PASSES);
    LMI_CHECK_ARG(nq >= 0 && R >= 1 && (int64_t)nq * R < INT32_MAX, "bad nq/R");
    if (nq == 0) return LMI_OK;
    LMI_CHECK_ARG(out_d && out_pos && workspace, "null pointer");
    int kp;
    const int ldo = passes_of(idx, qmode, k, &kp) * kp;
    const size_t P = (size_t)nq * R;
    const size_t lists = align_up(P * ldo * 4, 256);
    if (ws_bytes < 2 * lists) {
        set_error("workspace %zu B < required %zu B", ws_bytes, 2 * lists);
        return LMI_E_WORKSPACE;
    }
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    float* ld = reinterpret_cast<float*>(ws);
    int32_t* lp = reinterpret_cast<int32_t*>(ws + lists);
    const int rc = bucket_topk_wide(idx, q, nq, ldq, classes, R, k, qmode, ld, lp, nullptr, ldo,
                                    status, ws + 2 * lists, ws_bytes - 2 * lists, s);
    if (rc != LMI_OK) return rc;
    hipLaunchKernelGGL(take_k_kernel, dim3((unsigned)((P * k + 255) / 256)), dim3(256), 0, s, ld, lp,
                       (int64_t)P, ldo, k, out_d, out_pos);
    LMI_LAUNCH_CHECK("take_k_kernel");
    return LMI_OK;
}

int lmi::bucket_topk_impl(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                          const int32_t* classes, int32_t R, int32_t k, int32_t qmode, float* out_d,
                          int32_t* out_pos, int32_t* out_row, int32_t* status, void* workspace,
                          size_t ws_bytes, hipStream_t s, const unsigned long long* lo_g, int32_t ldo,
                          bool prefill, bool seed_r0, float seed_margin, int phases,
                          const WideScan* wide, float* out_bound, float* kth_out, int32_t kth_k) {
    const bool do_plan = phases & kPhasePlan, do_scan = phases & kPhaseScan,
               do_merge = phases & kPhaseMerge;
    using namespace lmi;
    if (ldo <= 0) ldo = k;
    LMI_CHECK_ARG(idx != nullptr, "null index");
    LMI_CHECK_ARG(idx->dtype == LMI_F16 || idx->dtype == LMI_F32, "bad corpus dtype");
    LMI_CHECK_ARG(idx->d >= 1 && idx->d_pad >= idx->d && idx->d_pad % 32 == 0, "bad d/d_pad");
    LMI_CHECK_ARG(idx->n_buckets >= 1, "n_buckets < 1");
    LMI_CHECK_ARG(idx->chunk_rows >= 32 && idx->chunk_rows % 32 == 0, "chunk_rows must be a multiple of 32");
    LMI_CHECK_ARG(idx->n_rows >= 0 && idx->n_rows < (int64_t)UINT32_MAX, "n_rows out of range");
    LMI_CHECK_ARG(nq >= 0 && R >= 1 && (int64_t)nq * R < INT32_MAX, "bad nq/R");
    LMI_CHECK_ARG(k >= 1 && k <= LMI_MAX_K, "k=%d outside [1, %d]", k, LMI_MAX_K);
    LMI_CHECK_ARG(qmode == LMI_Q_F16 || qmode == LMI_Q_F32, "bad qmode");
    LMI_CHECK_ARG(ldq >= idx->d, "ldq < d");
    if (nq == 0) return LMI_OK;
    LMI_CHECK_ARG(q && classes && out_d && out_pos && status && workspace, "null pointer");
    LMI_CHECK_ARG(idx->n_rows == 0 || (idx->corpus && idx->inv_norm && idx->gpos), "null corpus arrays");
    LMI_CHECK_ARG(idx->bucket_off && idx->chunk_first, "null bucket tables");

    const bool LOP = lo_g != nullptr;
    const WsLayout w = ws_layout(idx, nq, R, k, qmode, LOP);
    if (ws_bytes < w.total) {
        set_error("workspace %zu B < required %zu B", ws_bytes, w.total);
        return LMI_E_WORKSPACE;
    }
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    const bool f16math = (idx->dtype == LMI_F16) && (qmode == LMI_Q_F16);
    const int QB = w.qb;
    const int P = nq * R;
    const int KL = pick_kl(idx, qmode, k);

    // the plan's per-pair initial values, written by prep: pair_bucket = -1
    // (pairs whose class is out of range are never filled), pair_pos = -1 (the
    // seed), split_mask = 0, the per-pair bounds thr_g = all ones (scan v2/v3)
    PrepFills fills{};
    const bool seed_plan = seed_r0 && w.use_v3 && !(lo_g != nullptr) && R > 1;
    // the float64 mode's band lists (out_bound: every pair's bound of its
    // unlisted rows, +inf until the merge writes it)
    const bool band = out_bound != nullptr;
    if (band && !(w.use_v3 && KL == 15 && lo_g == nullptr && wide == nullptr)) {
        set_error("internal: band lists need scan v3 with 15-entry lists");
        return LMI_E_INVALID;
    }
    if (band) {
        fills.p[fills.n] = reinterpret_cast<uint32_t*>(out_bound);
        fills.v[fills.n] = 0x7f800000u;
        fills.per_q[fills.n] = R;
        ++fills.n;

    }
    if (idx->n_rows > 0) {
        auto add = [&](void* ptr, uint32_t v, int per_q) {
            fills.p[fills.n] = reinterpret_cast<uint32_t*>(ptr);
            fills.v[fills.n] = v;
            fills.per_q[fills.n] = per_q;
            ++fills.n;
        };
        add(ws + w.pair_bucket, 0xffffffffu, R);
        if (seed_plan) add(ws + w.pair_pos, 0xffffffffu, R);
        add(ws + w.split_mask, 0u, R);
        if (w.use_v2 || w.use_v3) add(ws + w.thr_g, 0xffffffffu, 2 * R);
    }
    if (do_plan) {
        const dim3 pg((nq + kThreads / 64 - 1) / (kThreads / 64));
        const bool vec = ((uintptr_t)q % 16 == 0) && (ldq % 4 == 0);
        auto* kp = f16math ? (vec ? prep_kernel<true, true> : prep_kernel<true, false>)
                           : (vec ? prep_kernel<false, true> : prep_kernel<false, false>);
        hipLaunchKernelGGL(kp, pg, dim3(kThreads), 0, s, q, nq, ldq, idx->d, idx->d_pad,
                           (void*)(ws + w.qbuf), (float*)(ws + w.invq), status, out_d, out_pos,
                           out_row, prefill ? R * ldo : 0, fills);
        LMI_LAUNCH_CHECK("prep_kernel");
    }
    if (idx->n_rows == 0) {
        // (an empty shard lists nothing: its kth block is all +inf)
        if (kth_out != nullptr && do_merge) LMI_TRY(fill_u32(kth_out, 0x7f800000u, (size_t)P * kth_k, s));
        return LMI_OK;
    }

    int32_t* counts = (int32_t*)(ws + w.counts);
    int32_t* pair_q = (int32_t*)(ws + w.pair_q);
    int32_t* pair_bucket = (int32_t*)(ws + w.pair_bucket);
    Tile* tiles = (Tile*)(ws + w.tiles);
    int32_t* meta = (int32_t*)(ws + w.ntiles);
    int32_t* work = (int32_t*)(ws + w.work);
    const int C = idx->n_buckets;
    int ng = clamp_knob(env_config().scan_groups, kGroups, 1, kGroups);
    while (ng & (ng - 1)) ng &= ng - 1;

    // (pair_bucket = -1 marks pairs whose class is out of range: never filled)
    if (do_plan) {
        hipLaunchKernelGGL(plan_count_kernel, dim3(C), dim3(kPlanThreads), 0, s, classes, P, counts);
        LMI_LAUNCH_CHECK("plan_count_kernel");
    }
    // (the seed reads the pair position of every (q, 0); pairs whose class is
    // out of range keep -1)
    const bool seed = seed_plan;
    int32_t* pair_pos = seed ? (int32_t*)(ws + w.pair_pos) : nullptr;
    const bool nearest_first = w.use_v3 && idx->chunk_centroid && !env_config().scan_no_pref;
    // tail split (scan v3): K = the queue's share of the grid; plan_fill leaves
    // K (S - 1) free slots after every queue for its parts
    // (not in the wide path's bound scan: its lists are the bucket's own)
    const int split_k = !w.use_v3 || nearest_first || env_config().scan_split < 0 ||
                        (wide && wide->mode == 1) ? 0
                        : std::min(kSplitMaxK, env_config().scan_split > 0 ? env_config().scan_split
                                                                            : (num_cus() + ng - 1) / ng);
    if (split_k > 0 && w.split_s < 2) {
        set_error("internal: tail split and workspace layout disagree");
        return LMI_E_INVALID;
    }
    const int qpad = split_k * (w.split_s - 1);
    if (do_plan) {
        hipLaunchKernelGGL(plan_fill_kernel, dim3(C), dim3(kPlanThreads), 0, s, classes, P, C, counts,
                           idx->chunk_first, QB, pair_q, pair_bucket, tiles, meta, work, ng, pair_pos,
                           qpad);
        LMI_LAUNCH_CHECK("plan_fill_kernel");
    }
    int32_t* seed_pos = seed ? (int32_t*)(ws + w.seed_pos) : nullptr;
    if (seed && do_plan) {
        hipLaunchKernelGGL(seed_pos_kernel, dim3((P + 255) / 256), dim3(256), 0, s, pair_q, pair_pos,
                           P, R, seed_pos);
        LMI_LAUNCH_CHECK("seed_pos_kernel");
    }
    if (do_plan && nearest_first) {
        int32_t* pref = (int32_t*)(ws + w.pref);
        int32_t* n_seed = (int32_t*)(ws + w.n_seed);
        hipLaunchKernelGGL(pref_kernel, dim3((P + kThreads / 64 - 1) / (kThreads / 64)), dim3(kThreads),
                           0, s, pair_bucket, idx->chunk_first, idx->chunk_centroid, idx->d_pad,
                           (const _Float16*)(ws + w.qbuf), pair_q, R, P, pref);
        LMI_LAUNCH_CHECK("pref_kernel");
        hipLaunchKernelGGL(pref_sort_kernel, dim3(C), dim3(kThreads), 0, s, counts, idx->chunk_first,
                           pair_q, pref, (int32_t*)(ws + w.pref_tmp), (int32_t*)(ws + w.pref_tmp2), QB,
                           n_seed);
        LMI_LAUNCH_CHECK("pref_sort_kernel");
        hipLaunchKernelGGL(tile3_fill_kernel, dim3(C), dim3(kThreads), 0, s, counts, idx->chunk_first,
                           pref, n_seed, C, QB, tiles, meta, work);
        LMI_LAUNCH_CHECK("tile3_fill_kernel");
    }
    if (nearest_first) ng = 1;  // one queue: seed tiles strictly first

    // tail split (scan v3; not after the nearest-chunk-first plan: its queue
    // has no seed count)
    uint32_t* split_mask = (uint32_t*)(ws + w.split_mask);
    const int64_t* scan_off = idx->bucket_off;
    if (split_k > 0) {
        if (do_plan)
            hipLaunchKernelGGL(tail_split_kernel, dim3(kGroups), dim3(256), 0, s, tiles, meta,
                               idx->bucket_off, (int64_t*)(ws + w.ext_off), C, idx->chunk_rows,
                               std::max(idx->max_chunks, 1), split_k, w.split_s, split_mask);
        LMI_LAUNCH_CHECK("tail_split_kernel");
        scan_off = (const int64_t*)(ws + w.ext_off);
    }

    // the collect scan: every grouped pair's fixed bound (0 = takes nothing)
    // and its candidate count
    if (wide && wide->mode == 2 && do_scan) {
        hipLaunchKernelGGL(set_bound_kernel, dim3((P + 255) / 256), dim3(256), 0, s, pair_q, P,
                           wide->bound_ord, (unsigned long long*)(ws + w.thr_g), wide->ccount, pair_bucket,
                           idx->bucket_off, wide->app_d, wide->app_row, wide->app_k, wide->cand, wide->cap);
        LMI_LAUNCH_CHECK("set_bound_kernel");
    }

    ScanArgs a{};
    a.corpus = idx->corpus;
    a.d_pad = idx->d_pad;
    a.inv_norm = idx->inv_norm;
    a.bucket_off = idx->bucket_off;
    a.chunk_rows = idx->chunk_rows;
    a.max_chunks = w.split_s * std::max(idx->max_chunks, 1);  // the partial-list stride (+ split parts)
    a.qbuf = ws + w.qbuf;
    a.invq = (const float*)(ws + w.invq);
    a.pair_q = pair_q;
    a.R = R;
    a.tiles = tiles;
    a.meta = meta;
    a.work = work;
    a.partial = (uint64_t*)(ws + w.partial);
    a.gpos = idx->gpos;
    a.lo_g = lo_g;

    int rc;
    if (phases != kPhaseAll && !(w.use_v2 || w.use_v3)) {
        set_error("phase flags need the fp16 scan (scan v2/v3: fp16 corpus and fp16-exact queries)");
        return LMI_E_UNSUPPORTED;
    }
    if (w.use_v2 || w.use_v3) {
        Scan2Args b{};
        b.corpus = reinterpret_cast<const _Float16*>(idx->corpus);
        b.inv_norm = idx->inv_norm;
        b.bucket_off = scan_off;
        b.chunk_rows = idx->chunk_rows;
        b.max_chunks = a.max_chunks;
        b.qbuf = reinterpret_cast<const _Float16*>(ws + w.qbuf);
        b.invq = a.invq;
        b.pair_q = pair_q;
        b.R = R;
        b.tiles = tiles;
        b.meta = meta;
        b.work = work;
        b.partial = a.partial;
        b.thr_g = reinterpret_cast<unsigned long long*>(ws + w.thr_g);
        b.gpos = idx->gpos;
        b.lo_g = lo_g;
        b.pair_pos = seed_pos;
        b.seed_margin = seed_margin;
        // (MODE 3: 2 eps = the seed margin of the float64 mode, rounded up,
        // + 2^-22 for the rounding of bound + band, distances being < 4)
        b.band = band ? seed_margin * (1.0f + 0x1p-20f) + 0x1p-22f : 0.0f;
        b.ng = ng;
        b.lag = std::max(0, std::min(3, env_config().scan_lag));
        // (thr_g was reset by prep)
        if (!do_scan) rc = LMI_OK;
        else
        if (wide) {
            if (!w.use_v3 || LOP || (wide->mode == 1 ? KL != 15 : KL != 10)) {
                set_error("internal: the wide scans take scan v3 with 15 (chunk lists) or 10 (collect) entries");
                return LMI_E_INVALID;
            }
            b.cand = wide->cand;
            b.ccount = wide->ccount;
            b.cap = wide->cap;
            b.bins = wide->bins;
            b.nbins = wide->nbins;
            b.sub_rows = wide->sub_rows;
            b.sub_take = wide->sub_take;
            rc = wide->mode == 1 ? launch_scan3_v<15, 0, false, 1>(b, s) : launch_scan3_v<10, 0, false, 2>(b, s);
        }
        else if (w.use_v3 && LOP) {
            // the passes' lists are 15 entries on v3 (passes_of)
            if (KL != 15) {
                set_error("lower-bound scan passes take 15-entry lists on scan v3");
                return LMI_E_UNSUPPORTED;
            }
            rc = launch_scan3_v<15, 0, true>(b, s);
        }
        else if (w.use_v3 && band)
            rc = launch_scan3_v<10, 0, false, 3>(b, s);
        else if (w.use_v3)
            rc = (KL == 10) ? launch_scan3<10>(b, s) : launch_scan3<15>(b, s);
        else
            rc = (KL == 10) ? launch_scan2<10>(b, s) : launch_scan2<16>(b, s);
    } else if (LOP) {
        // lower-bound passes off v3: the general kernel, 16-entry lists
        if (KL != 16) {
            set_error("lower-bound scan passes need 16-entry lists off scan v3");
            return LMI_E_UNSUPPORTED;
        }
        rc = f16math ? launch_scan<16, true, _Float16, true>(a, idx->d_pad, s)
           : (idx->dtype == LMI_F16) ? launch_scan<16, false, _Float16, true>(a, idx->d_pad, s)
                                     : launch_scan<16, false, float, true>(a, idx->d_pad, s);
    } else if (f16math) {
        rc = (KL == 10) ? launch_scan<10, true, _Float16>(a, idx->d_pad, s)
                        : launch_scan<16, true, _Float16>(a, idx->d_pad, s);
    } else if (idx->dtype == LMI_F16) {
        rc = (KL == 10) ? launch_scan<10, false, _Float16>(a, idx->d_pad, s)
                        : launch_scan<16, false, _Float16>(a, idx->d_pad, s);
    } else {
        rc = (KL == 10) ? launch_scan<10, false, float>(a, idx->d_pad, s)
                        : launch_scan<16, false, float>(a, idx->d_pad, s);
    }
    if (rc != LMI_OK) return rc;
    if (!do_merge) return LMI_OK;

    const int grid = (int)(((int64_t)P * kMergeLanes + kMergeBlock - 1) / kMergeBlock);
    if (band) {
        hipLaunchKernelGGL(chunk_merge_band_kernel, dim3(grid), dim3(kMergeBlock), 0, s, a.partial, a.max_chunks,
                           pair_q, pair_bucket, idx->chunk_first, idx->gpos, P, k, ldo, out_d, out_pos,
                           out_row, out_bound, idx->n_rows, status, split_mask, w.split_s, kth_out, kth_k,
                           classes, C);
        LMI_LAUNCH_CHECK("chunk_merge_band_kernel");
        return LMI_OK;
    }
#define LMI_CM(KLV, ROWSV)                                                                         \
    hipLaunchKernelGGL((chunk_merge_kernel<KLV, ROWSV>), dim3(grid), dim3(kMergeBlock), 0, s, a.partial, \
                       a.max_chunks, pair_q, pair_bucket, idx->chunk_first, idx->gpos, P, k, ldo,  \
                       out_d, out_pos, out_row, idx->n_rows, status, split_mask, w.split_s)
    if (KL == 10) {
        if (out_row) LMI_CM(10, true); else LMI_CM(10, false);
    } else if (KL == 15) {
        if (out_row) LMI_CM(15, true); else LMI_CM(15, false);
    } else {
        if (out_row) LMI_CM(16, true); else LMI_CM(16, false);
    }
#undef LMI_CM
    LMI_LAUNCH_CHECK("chunk_merge_kernel");
    return LMI_OK;
}

namespace lmi {
// |d~ - d| for every (query, row) of the split mode, d~ the fp16 scan's
// distance on the normalised, fp16-rounded vectors and d the exact one:
// rounding a unit vector to fp16 moves it by delta <= 2^-11 (relative, normal
// range; + 2^-22 for the float32 step before it) + sqrt(d) 2^-25 (absolute,
// the subnormal range), i.e. by an angle <= asin(delta); the angle between
// query and row moves by at most the two angles, and a cosine by at most the
// angle.  Plus the fp16 scan's own arithmetic on the rounded vectors
// (refine_eps of li/index.py, the fp16 path: gamma(2 (d_pad/16 + 16)) for the
// dot, the two norms, the scale and the final fma) and 2^-24 for rounding the
// exact value to float32 (ties of the rounded values then order by position).
double split_eps(int d_pad) {
    const double u = std::ldexp(1.0, -24);
    auto gamma = [&](double n) { return n * u / (1.0 - n * u); };
    const double delta = std::ldexp(1.0, -11) + std::ldexp(1.0, -22) + std::sqrt((double)d_pad) * std::ldexp(1.0, -25);
    const double h = 2.0 * (d_pad / 16 + 16), hq = 4.0 * ((d_pad + 255) / 256) + 6.0;
    const double scan = gamma(h) + gamma(2 * hq) / 2 + 4 * u + u + 2 * u + 2 * u;
    return 2.0 * std::asin(delta) + scan + u;
}

namespace {
struct XWs {
    size_t qr, ld, lpos, srow, bound, ccount, cand, failed, nfailed, wgl, sfl, spd, spg, fix, bins, sub_first, sub_rows, sub_take,
        off2, cf2, classes2, off2b, cf2b, classes2b, qn32, grp, tailq, goff, region, region_bytes, region_s,
        region_s_bytes, total;
    int32_t cap;
};
// k <= 10: the k-th of a per-bucket sample (the product scan over
// x_sample_desc); the device tables are filled by x_sample_desc_kernel
inline bool x_sample(int k) { return k <= 10; }
lmi_index_desc x_sample_desc(const lmi_index_desc* idx, const int64_t* off2, const int32_t* cf2) {
    lmi_index_desc d = *idx;
    d.n_buckets = 2 * idx->n_buckets;
    d.bucket_off = off2;
    d.chunk_first = cf2;
    // (host-side bounds for the workspace: a sample of at most n_c / 16 + 32
    // rows beyond one chunk)
    d.max_chunks = 2 + std::max(idx->max_chunks, 1) / kXSampleDiv;
    d.n_chunks = idx->n_buckets * d.max_chunks;
    d.chunk_centroid = nullptr;
    return d;
}
// the collect scan's: the rest of every bucket whose sample is skipped, the
// others whole (x_sample_desc_kernel)
lmi_index_desc x_collect_desc(const lmi_index_desc* idx, const int64_t* off2b, const int32_t* cf2b) {
    lmi_index_desc d = *idx;
    d.n_buckets = 2 * idx->n_buckets;
    d.bucket_off = off2b;
    d.chunk_first = cf2b;
    d.chunk_centroid = nullptr;
    return d;
}
// k <= 15: the k-th comes from a sampled bound scan (the wide path's chunk-list
// scan over two lists per bucket, each the first quarter of its rows), not a
// whole first scan
constexpr int kXLists = 2;
inline bool x_sampled(int k) { return k <= 15; }
lmi_index_desc bound_desc(const lmi_index_desc* idx, int lists, const int32_t* sub_first);

XWs x_ws(const lmi_index_desc* idx, int nq, int R, int k) {
    XWs w{};
    const size_t P = (size_t)nq * R;
    // collect slots per pair: 2048 (the rows within 2 eps of the k-th, ~20 on
    // the clip768-like mixture), fewer for huge batches (<= 2 GiB of slots)
    int cap = 2048;
    while (cap > 256 && P * (size_t)cap * 8 > (size_t(2) << 30)) cap >>= 1;
    w.cap = cap;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t at = off;
        off = align_up(off + bytes, 256);
        return at;
    };
    w.qr = take((size_t)nq * idx->d_pad * 4);
    w.ld = take(P * std::max(k, 15) * 4);
    w.lpos = take(P * std::max(k, 15) * 4);
    w.srow = take(P * std::max(k, 15) * 4);
    w.fix = take(P * 4);
    w.bins = take(P * 4);
    w.sub_first = take(((size_t)idx->n_buckets + 1) * 4);
    w.sub_rows = take((size_t)idx->n_buckets * 4);
    w.sub_take = take((size_t)idx->n_buckets * 4);
    w.off2 = take(((size_t)2 * idx->n_buckets + 1) * 8);
    w.cf2 = take(((size_t)2 * idx->n_buckets + 1) * 4);
    w.classes2 = take(P * 4);
    w.off2b = take(((size_t)2 * idx->n_buckets + 1) * 8);
    w.cf2b = take(((size_t)2 * idx->n_buckets + 1) * 4);
    w.classes2b = take(P * 4);
    w.qn32 = take((size_t)nq * idx->d_pad * 4);
    w.grp = take((size_t)R * idx->n_buckets * 4);
    w.tailq = take(P);
    w.goff = take(((size_t)idx->n_buckets + 1) * 8);
    w.bound = take(P * 4);
    w.ccount = take(P * 4);
    w.cand = take(P * (size_t)cap * 8);
    w.failed = take(P * 4);
    w.nfailed = take(256);  // (word 0: the failed pairs; word 8: the sfl pairs; word 16: the wgl pairs)
    w.wgl = take(P * 4);
    w.sfl = take(P * 4);
    // (the sliced sample fallback's lists)
    w.spd = take((size_t)kXSlicedPairs * kXSlices * k * 8);
    w.spg = take((size_t)kXSlicedPairs * kXSlices * k * 4);
    const lmi_index_desc bd = bound_desc(idx, kXLists, nullptr);
    const lmi_index_desc sd = x_sample_desc(idx, nullptr, nullptr);
    const lmi_index_desc cd = x_collect_desc(idx, nullptr, nullptr);
    w.region_bytes = std::max({ws_layout(idx, nq, R, k, LMI_Q_F16).total, ws_layout(idx, nq, R, 10, LMI_Q_F16).total,
                               ws_layout(&bd, nq, R, 15, LMI_Q_F16).total, ws_layout(&sd, nq, R, k, LMI_Q_F16).total,
                               ws_layout(&cd, nq, R, 10, LMI_Q_F16).total});
    w.region = take(w.region_bytes);
    // k <= 10: the sample scan's own region (ABI 11), so the plans of both
    // scans are laid down in one PLAN phase and the batch stream can run the
    // phases of one batch apart
    if (x_sample(k)) {
        w.region_s_bytes = ws_layout(&sd, nq, R, k, LMI_Q_F16).total;
        w.region_s = take(w.region_s_bytes);
    }
    w.total = off;
    return w;
}
}  // namespace

size_t x_ws_bytes(const lmi_index_desc* idx, int nq, int R, int k) { return x_ws(idx, nq, R, k).total; }
size_t x_nfailed_offset(const lmi_index_desc* idx, int nq, int R, int k) { return x_ws(idx, nq, R, k).nfailed; }

// The split mode: see lmi_index_desc.corpus32 (include/lmi_hip.h).  out_d is
// float (out_f64 = 0) or double [nq*R][k]; qmode is ignored (the queries are
// rounded here whatever their class).
int bucket_topk_x(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq, const double* q64,
                  int32_t ldq64, const int32_t* classes, int32_t R, int32_t k, void* out_d, int out_f64,
                  int32_t* out_pos, int32_t* status, void* workspace, size_t ws_bytes, hipStream_t s,
                  int phases) {
    LMI_CHECK_ARG(idx != nullptr, "null index");
    LMI_CHECK_ARG(idx->corpus32 != nullptr && idx->dtype == LMI_F16 && idx->d_pad == v2::D,
                  "split mode needs corpus32, an fp16 scan corpus and d_pad %d", v2::D);
    LMI_CHECK_ARG(k >= 1 && k <= LMI_MAX_K, "split mode: k=%d outside [1, %d]", k, LMI_MAX_K);
    LMI_CHECK_ARG(nq >= 0 && R >= 1 && (int64_t)nq * R < INT32_MAX, "bad nq/R");
    if (nq == 0) return LMI_OK;
    LMI_CHECK_ARG((q || q64) && classes && out_d && out_pos && status && workspace, "null pointer");
    LMI_CHECK_ARG(q64 ? ldq64 >= idx->d : ldq >= idx->d, "ldq < d");
    if (phases != kPhaseAll && !x_sample(k)) {
        set_error("split mode: phase flags need k <= 10 (the sample's bound)");
        return LMI_E_UNSUPPORTED;
    }
    const XWs w = x_ws(idx, nq, R, k);
    if (ws_bytes < w.total) {
        set_error("workspace %zu B < required %zu B", ws_bytes, w.total);
        return LMI_E_WORKSPACE;
    }
    const int P = nq * R;
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    float* qr = (float*)(ws + w.qr);
    float* ld = (float*)(ws + w.ld);
    int32_t* lpos = (int32_t*)(ws + w.lpos);
    auto* bound = (uint32_t*)(ws + w.bound);
    auto* ccount = (uint32_t*)(ws + w.ccount);
    auto* cand = (uint64_t*)(ws + w.cand);
    unsigned char* region = ws + w.region;
    const double two_eps = 2.0 * split_eps(idx->d_pad);
    const bool sampled = x_sampled(k);
    int32_t* fix = (int32_t*)(ws + w.fix);
    int rc;
    WideScan m2{2, bound, cand, ccount, w.cap, nullptr, 0, nullptr, nullptr};
    int32_t* srow = (int32_t*)(ws + w.srow);
    auto* off2b = (int64_t*)(ws + w.off2b);
    const lmi_index_desc cd = x_collect_desc(idx, off2b, (int32_t*)(ws + w.cf2b));
    if (x_sample(k)) {
        // (PLAN: the rounded queries and both scans' plans; SCAN: the sample
        // scan and its merge, the bound, the collect scan; MERGE: step 3)
        auto* off2 = (int64_t*)(ws + w.off2);
        auto* cf2 = (int32_t*)(ws + w.cf2);
        auto* classes2 = (int32_t*)(ws + w.classes2);
        const lmi_index_desc sd = x_sample_desc(idx, off2, cf2);
        unsigned char* region_s = ws + w.region_s;
        auto* classes2b = (int32_t*)(ws + w.classes2b);
        // (the collect skips the samples it can: their candidates are the
        // sample scan's lists, appended by set_bound_kernel)
        m2.app_d = ld;
        m2.app_row = srow;
        m2.app_k = k;
        if (phases & kPhasePlan) {
            hipLaunchKernelGGL(x_round_queries_kernel, dim3((nq + kThreads / 64 - 1) / (kThreads / 64)),
                               dim3(kThreads), 0, s, q, ldq, q64, ldq64, nq, idx->d, idx->d_pad, qr);
            LMI_LAUNCH_CHECK("x_round_queries_kernel");
            LMI_TRY(fill_u32(ws + w.nfailed, 0u, 32, s));
            hipLaunchKernelGGL(x_sample_desc_kernel, dim3((unsigned)std::min(1024, (P + 63) / 64)), dim3(64), 0, s,
                               idx->bucket_off, idx->n_buckets, (int64_t)idx->chunk_rows, classes, P, off2, cf2,
                               classes2, off2b, (int32_t*)(ws + w.cf2b), classes2b,
                               std::max(0, env_config().x_skip));
            LMI_LAUNCH_CHECK("x_sample_desc_kernel");
            rc = bucket_topk_impl(&sd, qr, nq, idx->d_pad, classes2, R, k, LMI_Q_F16, ld, lpos, srow, status,
                                  region_s, w.region_s_bytes, s, nullptr, 0, true, false, 0.0f, kPhasePlan);
            if (rc != LMI_OK) return rc;
            rc = bucket_topk_impl(&cd, qr, nq, idx->d_pad, classes2b, R, 10, LMI_Q_F16, ld, lpos, nullptr, status,
                                  region, w.region_bytes, s, nullptr, 0, false, false, 0.0f, kPhasePlan, &m2);
            if (rc != LMI_OK) return rc;
        }
        if (phases & kPhaseScan) {
            // 1. the k-th of every pair's bucket sample (its first chunk_rows
            //    rows): the product scan over the 2C-bucket sample descriptor,
            //    then that k-th + 2 eps as the collect bound
            rc = bucket_topk_impl(&sd, qr, nq, idx->d_pad, classes2, R, k, LMI_Q_F16, ld, lpos, srow, status,
                                  region_s, w.region_s_bytes, s, nullptr, 0, true, false, 0.0f,
                                  kPhaseScan | kPhaseMerge);
            if (rc != LMI_OK) return rc;
            hipLaunchKernelGGL(x_bound_kernel, dim3((P + 255) / 256), dim3(256), 0, s, (int64_t)P, k, ld, two_eps,
                               bound);
            LMI_LAUNCH_CHECK("x_bound_kernel");
            // 2. every row under the bound (the collect scan, as the wide path's,
            //    over the rest of the buckets whose sample it skips)
            rc = bucket_topk_impl(&cd, qr, nq, idx->d_pad, classes2b, R, 10, LMI_Q_F16, ld, lpos, nullptr, status,
                                  region, w.region_bytes, s, nullptr, 0, false, false, 0.0f, kPhaseScan, &m2);
            if (rc != LMI_OK) return rc;
        }
        if (!(phases & kPhaseMerge)) return LMI_OK;
    } else {
    hipLaunchKernelGGL(x_round_queries_kernel, dim3((nq + kThreads / 64 - 1) / (kThreads / 64)), dim3(kThreads),
                       0, s, q, ldq, q64, ldq64, nq, idx->d, idx->d_pad, qr);
    LMI_LAUNCH_CHECK("x_round_queries_kernel");
    LMI_TRY(fill_u32(ws + w.nfailed, 0u, 32, s));
    if (sampled) {
        // 1. a bound per pair from a sample: the wide path's chunk-list scan
        //    (two lists per bucket, each scanning the first quarter of its
        //    rows, every list its part's own top-15), the 15th smallest entry
        //    (>= the pair's 15th >= its k-th), + 2 eps
        hipLaunchKernelGGL(wide_init_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, (int64_t)P, 0,
                           nullptr, nullptr, nullptr, bound, fix);
        LMI_LAUNCH_CHECK("wide_init_kernel");
        auto* sub_first = (int32_t*)(ws + w.sub_first);
        auto* sub_rows = (int32_t*)(ws + w.sub_rows);
        auto* sub_take = (int32_t*)(ws + w.sub_take);
        hipLaunchKernelGGL(bound_lists_kernel, dim3(1), dim3(256), 0, s, idx->bucket_off, idx->n_buckets, kXLists,
                           sub_first, sub_rows, sub_take);
        LMI_LAUNCH_CHECK("bound_lists_kernel");
        const lmi_index_desc bd = bound_desc(idx, kXLists, sub_first);
        auto* bins = (uint32_t*)(ws + w.bins);
        LMI_TRY(fill_u32(bins, 0xffffffffu, (size_t)P, s));
        const WideScan m1{1, nullptr, nullptr, nullptr, 0, bins, 1, sub_rows, sub_take};
        rc = bucket_topk_impl(&bd, qr, nq, idx->d_pad, classes, R, 15, LMI_Q_F16, ld, lpos, nullptr, status, region,
                              w.region_bytes, s, nullptr, 0, false, false, 0.0f, kPhasePlan | kPhaseScan, &m1);
        if (rc != LMI_OK) return rc;
        const WsLayout lb = ws_layout(&bd, nq, R, 15, LMI_Q_F16);
        hipLaunchKernelGGL(kth_bound_kernel, dim3((unsigned)P), dim3(64), 0, s,
                           (const uint64_t*)(region + lb.partial), lb.split_s * bd.max_chunks, lb.split_s,
                           (const int32_t*)(region + lb.pair_q), (const int32_t*)(region + lb.pair_bucket), sub_first,
                           (const uint32_t*)(region + lb.split_mask), P, 15, idx->bucket_off, w.cap, bound, fix);
        LMI_LAUNCH_CHECK("kth_bound_kernel");
        hipLaunchKernelGGL(x_margin_kernel, dim3((P + 255) / 256), dim3(256), 0, s, (int64_t)P, two_eps, bound);
        LMI_LAUNCH_CHECK("x_margin_kernel");
    } else {
        // 1. the fp16 scan on the rounded vectors: every pair's approximate k-th
        rc = bucket_topk_impl(idx, qr, nq, idx->d_pad, classes, R, k, LMI_Q_F16, ld, lpos, nullptr, status,
                              region, w.region_bytes, s);
        if (rc != LMI_OK) return rc;
        hipLaunchKernelGGL(x_bound_kernel, dim3((P + 255) / 256), dim3(256), 0, s, (int64_t)P, k, ld, two_eps,
                           bound);
        LMI_LAUNCH_CHECK("x_bound_kernel");
    }
    // 2. every row under the bound (the collect scan, as the wide path's)
    rc = bucket_topk_impl(idx, qr, nq, idx->d_pad, classes, R, 10, LMI_Q_F16, ld, lpos, nullptr, status, region,
                          w.region_bytes, s, nullptr, 0, false, false, 0.0f, kPhasePlan | kPhaseScan, &m2);
    if (rc != LMI_OK) return rc;
    }
    // 3. the candidates' exact distances, sorted; overflowed pairs whole
    const WsLayout l = ws_layout(x_sample(k) ? &cd : idx, nq, R, 10, LMI_Q_F16);
    XArgs a{};
    a.rows32 = idx->corpus32;
    a.rows32n = idx->corpus32n;
    a.rows64 = out_f64 ? idx->corpus64 : nullptr;
    a.d = idx->d;
    a.d_pad = idx->d_pad;
    a.gpos = idx->gpos;
    a.bucket_off = idx->bucket_off;
    a.n_rows = idx->n_rows;
    a.q = q;
    a.ldq = ldq;
    a.q64 = out_f64 ? q64 : nullptr;
    a.ldq64 = ldq64;
    if (!a.q64 && !q) {
        set_error("split mode: float32 output needs the float32 queries");
        return LMI_E_INVALID;
    }
    a.classes = classes;
    a.nq = nq;
    a.R = R;
    a.k = k;
    a.pair_q = (const int32_t*)(region + l.pair_q);
    a.pair_bucket = (const int32_t*)(region + l.pair_bucket);
    a.cand = cand;
    a.ccount = ccount;
    a.cap = w.cap;
    a.out_d = out_d;
    a.out_f64 = out_f64;
    a.out_pos = out_pos;
    a.failed = (int32_t*)(ws + w.failed);
    a.n_failed = (int32_t*)(ws + w.nfailed);
    a.wgl = sampled ? (int32_t*)(ws + w.wgl) : nullptr;  // (two_eps > 0: the wave kernel runs)
    a.n_wgl = (int32_t*)(ws + w.nfailed) + 16;
    a.status = status;
    a.two_eps = sampled ? two_eps : 0.0;
    a.fix = sampled && !x_sample(k) ? fix : nullptr;
    // (ABI 10: the float32 output in the reference's own float32 order)
    a.qn32 = (!out_f64 && q) ? (const float*)(ws + w.qn32) : nullptr;
    a.grp = (const int32_t*)(ws + w.grp);
    a.nrows_c = idx->bucket_rows;
    a.C = idx->n_buckets;
    a.tailq = (const uint8_t*)(ws + w.tailq);
    a.goff = (const int64_t*)(ws + w.goff);
    a.plan_counts = (const int32_t*)(region + l.counts);
    a.plan_cm = x_sample(k) ? 2 : 1;
    if (x_sample(k)) {
        a.soff = off2b;
        a.skth = ld;
        a.sfailed = (int32_t*)(ws + w.sfl);
        a.n_sfailed = (int32_t*)(ws + w.nfailed) + 8;
        a.spd = (double*)(ws + w.spd);
        a.spg = (int32_t*)(ws + w.spg);
    }
    // (pairs whose class is out of range keep the prefill of step 1's prep:
    // the outputs are prefilled here, by pair id, in step 3's own buffers)
    hipLaunchKernelGGL(x_prefill_kernel, dim3((unsigned)(((int64_t)P * k + 255) / 256)), dim3(256), 0, s,
                       (int64_t)P * k, out_d, out_f64, out_pos);
    LMI_LAUNCH_CHECK("x_prefill_kernel");
    return launch_x_refine(a, P, s);
}
}  // namespace lmi

#ifdef LMI_DIAG
// Diagnostic (the `make ablation` library only): lower every pair's global
// bound before the SCAN phase, e.g. to the final k-th distance of the
// all-rank lists (tools/bound_study.py: how much of a stripe's scan the
// per-rank bound costs).  Call after the PLAN phase of lmi_bucket_topk with
// the same arguments; seed_ord[pair id] is a distance ordinal (f2ord), the
// bound keeps every row at or under it (ties survive).
namespace {
__global__ __launch_bounds__(256) void debug_seed_bounds_kernel(const int32_t* __restrict__ pair_q, int32_t P,
                                                                const uint32_t* __restrict__ seed_ord,
                                                                unsigned long long* __restrict__ thr_g) {
    const int pp = blockIdx.x * 256 + threadIdx.x;
    if (pp >= P) return;
    const int p = pair_q[pp];
    if (p < 0 || p >= P) return;
    const unsigned long long v = ((unsigned long long)seed_ord[p] << 32) | 0xffffffffull;
    if (v < thr_g[pp]) thr_g[pp] = v;
}
}  // namespace

extern "C" int lmi_debug_seed_bounds(const lmi_index_desc* idx, int32_t nq, int32_t R, int32_t k,
                                     int32_t qmode, const uint32_t* seed_ord, void* workspace,
                                     void* stream) {
    using namespace lmi;
    qmode &= ~LMI_Q_SEED_ROUND0;
    take_phases(qmode);
    const WsLayout w = ws_layout(idx, nq, R, k, qmode);
    if (!w.use_v3) {
        set_error("seeded bounds need scan v3");
        return LMI_E_UNSUPPORTED;
    }
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    const int P = nq * R;
    hipLaunchKernelGGL(debug_seed_bounds_kernel, dim3((P + 255) / 256), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), (const int32_t*)(ws + w.pair_q), P, seed_ord,
                       (unsigned long long*)(ws + w.thr_g));
    LMI_LAUNCH_CHECK("debug_seed_bounds_kernel");
    return LMI_OK;
}
#endif

namespace lmi {
// k > 16: ceil(k / kp) scan passes of kp-entry lists (kp = 15 on scan v3, else
// 16), each keeping the next kp entries of the (distance, position) order
// after the previous pass's last key.  Lists of ldo = passes * kp entries.
int passes_of(const lmi_index_desc* idx, int qmode, int k, int* kp_out) {
    const int kp = pick_kl(idx, qmode, 15) == 15 ? 15 : 16;
    if (kp_out) *kp_out = kp;
    return (k + kp - 1) / kp;
}

size_t passes_ws_bytes(const lmi_index_desc* idx, int nq, int R, int k, int qmode) {
    int kp;
    passes_of(idx, qmode, k, &kp);
    const size_t P = (size_t)nq * R;
    return align_up(P * 8, 256) + scan_workspace_bytes(idx, nq, R, kp, qmode, true);
}

int bucket_topk_passes(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                       const int32_t* classes, int32_t R, int32_t k, int32_t qmode, float* out_d,
                       int32_t* out_pos, int32_t* out_row, int32_t ldo, int32_t* status,
                       void* workspace, size_t ws_bytes, hipStream_t s) {
    int kp;
    const int np = passes_of(idx, qmode, k, &kp);
    if (ldo < np * kp) {
        set_error("pass lists of %d entries < %d passes x %d", ldo, np, kp);
        return LMI_E_INVALID;
    }
    const size_t P = (size_t)nq * R;
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    auto* lo = reinterpret_cast<unsigned long long*>(ws);
    const size_t lo_bytes = align_up(P * 8, 256);
    if (ws_bytes < lo_bytes) {
        set_error("workspace %zu B too small", ws_bytes);
        return LMI_E_WORKSPACE;
    }
    LMI_TRY(fill_u32(lo, 0u, P * 2, s));
    for (int j = 0; j < np; ++j) {
        const int rc = bucket_topk_impl(idx, q, nq, ldq, classes, R, kp, qmode, out_d + (size_t)j * kp,
                                        out_pos + (size_t)j * kp, out_row ? out_row + (size_t)j * kp : nullptr,
                                        status, ws + lo_bytes, ws_bytes - lo_bytes, s, lo, ldo, j == 0);
        if (rc != LMI_OK) return rc;
        if (j + 1 < np) {
            hipLaunchKernelGGL(next_lo_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, out_d,
                               out_pos, (int32_t)P, ldo, (j + 1) * kp - 1, lo);
            LMI_LAUNCH_CHECK("next_lo_kernel");
        }
    }
    return LMI_OK;
}

namespace {
struct WideWs {
    bool on;       // the bound + collect path (else bucket_topk_passes alone)
    int kw, cap;   // list entries produced (passes * kp); candidate slots per pair
    int lists;     // bound-scan lists per bucket (at most; bound_lists_kernel)
    int nbins;     // the bound scan's pruning bins per pair (Scan2Args::bins)
    size_t bound, fix, cls, ccount, cand, fd, fpos, frow, sub_first, sub_rows, sub_take, bins, region,
        region_bytes, total;
};

// The bound scan's index: the same rows and buckets, each bucket cut into at
// most `lists` lists (bound_lists_kernel; their rows per bucket in sub_rows),
// no chunk centroids (the nearest-chunk-first plan's units are the index's
// chunks).  Host-side values only: the workspace size must not read the device.
lmi_index_desc bound_desc(const lmi_index_desc* idx, int lists, const int32_t* sub_first) {
    lmi_index_desc b = *idx;
    b.max_chunks = lists;
    b.n_chunks = idx->n_buckets * lists;
    b.chunk_first = sub_first;
    b.chunk_centroid = nullptr;
    return b;
}

WideWs wide_ws(const lmi_index_desc* idx, int nq, int R, int k, int qmode, int ldo) {
    WideWs w{};
    int kp;
    const int np = passes_of(idx, qmode, k, &kp);
    w.kw = np * kp;
    w.on = v3_capable(idx, qmode) && kp == 15 && !env_config().wide_passes;
    const size_t P = (size_t)nq * R;
    if (!w.on) {
        w.region_bytes = w.total = passes_ws_bytes(idx, nq, R, k, qmode);
        return w;
    }
    // Bound scan: 2 kw / 15 lists per bucket, so a pair's lists hold 2 kw
    // entries, each the top-15 of the first quarter of its list's rows: their
    // kw-th smallest is about the pair's 4 kw-th distance, and the collect scan
    // finds about 4 kw rows within it; 8 kw (+ 64) slots before the fix-up
    // passes take over.  Buckets of fewer lists' entries than kw but no more
    // rows than the slots are collected whole.
    w.lists = 2 * np;
    w.nbins = np;  // (np * 15 = kw)
    int cap = 256;
    while (cap < 8 * w.kw + 64) cap <<= 1;
    w.cap = std::min(cap, 8192);
    // (candidate slots past 8 GiB -- huge batches at large k -- : the passes,
    // whose lists are 8x smaller)
    if (P * (size_t)w.cap * 8 > (size_t(8) << 30)) {
        w.on = false;
        w.region_bytes = w.total = passes_ws_bytes(idx, nq, R, k, qmode);
        return w;
    }
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t at = off;
        off = align_up(off + bytes, 256);
        return at;
    };
    w.bound = take(P * 4);
    w.fix = take(P * 4);
    w.cls = take(P * 4);
    w.ccount = take(P * 4);
    w.cand = take(P * (size_t)w.cap * 8);
    w.fd = take(P * (size_t)ldo * 4);
    w.fpos = take(P * (size_t)ldo * 4);
    w.frow = take(P * (size_t)ldo * 4);
    w.sub_first = take(((size_t)idx->n_buckets + 1) * 4);
    w.sub_rows = take((size_t)idx->n_buckets * 4);
    w.sub_take = take((size_t)idx->n_buckets * 4);
    w.bins = take(P * (size_t)w.nbins * 4);
    const lmi_index_desc bd = bound_desc(idx, w.lists, nullptr);
    w.region_bytes = std::max({scan_workspace_bytes(&bd, nq, R, 15, qmode),
                               scan_workspace_bytes(idx, nq, R, 10, qmode),
                               passes_ws_bytes(idx, nq, R, k, qmode)});
    w.region = take(w.region_bytes);
    w.total = off;
    return w;
}
}  // namespace

size_t wide_ws_bytes(const lmi_index_desc* idx, int nq, int R, int k, int qmode, int ldo) {
    return wide_ws(idx, nq, R, k, qmode, ldo).total;
}

int bucket_topk_wide(const lmi_index_desc* idx, const float* q, int32_t nq, int32_t ldq,
                     const int32_t* classes, int32_t R, int32_t k, int32_t qmode, float* out_d,
                     int32_t* out_pos, int32_t* out_row, int32_t ldo, int32_t* status,
                     void* workspace, size_t ws_bytes, hipStream_t s) {
    const WideWs w = wide_ws(idx, nq, R, k, qmode, ldo);
    if (!w.on || idx->n_rows == 0)
        return bucket_topk_passes(idx, q, nq, ldq, classes, R, k, qmode, out_d, out_pos, out_row, ldo,
                                  status, workspace, ws_bytes, s);
    if (ldo < w.kw) {
        set_error("lists of %d entries < %d", ldo, w.kw);
        return LMI_E_INVALID;
    }
    if (ws_bytes < w.total) {
        set_error("workspace %zu B < required %zu B", ws_bytes, w.total);
        return LMI_E_WORKSPACE;
    }
    if (nq == 0) return LMI_OK;
    const int P = nq * R;
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    auto* bound = (uint32_t*)(ws + w.bound);
    auto* fix = (int32_t*)(ws + w.fix);
    auto* ccount = (uint32_t*)(ws + w.ccount);
    auto* cand = (uint64_t*)(ws + w.cand);
    auto* fd = (float*)(ws + w.fd);
    auto* fpos = (int32_t*)(ws + w.fpos);
    auto* frow = out_row ? (int32_t*)(ws + w.frow) : nullptr;
    unsigned char* region = ws + w.region;
    const int64_t PL = (int64_t)P * ldo;
    hipLaunchKernelGGL(wide_init_kernel, dim3((unsigned)((PL + 255) / 256)), dim3(256), 0, s, (int64_t)P,
                       ldo, out_d, out_pos, out_row, bound, fix);
    LMI_LAUNCH_CHECK("wide_init_kernel");
    const int plan_scan = kPhasePlan | kPhaseScan;
    // 1. every (pair, bound-pass chunk part)'s own top-15 -> each pair's bound
    auto* sub_first = (int32_t*)(ws + w.sub_first);
    auto* sub_rows = (int32_t*)(ws + w.sub_rows);
    auto* sub_take = (int32_t*)(ws + w.sub_take);
    hipLaunchKernelGGL(bound_lists_kernel, dim3(1), dim3(256), 0, s, idx->bucket_off, idx->n_buckets,
                       w.lists, sub_first, sub_rows, sub_take);
    LMI_LAUNCH_CHECK("bound_lists_kernel");
    const lmi_index_desc bd = bound_desc(idx, w.lists, sub_first);
    auto* bins = (uint32_t*)(ws + w.bins);
    LMI_TRY(fill_u32(bins, 0xffffffffu, (size_t)P * w.nbins, s));
    const WideScan m1{1, nullptr, nullptr, nullptr, 0, bins, w.nbins, sub_rows, sub_take};
    int rc = bucket_topk_impl(&bd, q, nq, ldq, classes, R, 15, qmode, fd, fpos, nullptr, status, region,
                              w.region_bytes, s, nullptr, 0, false, false, 0.0f, plan_scan, &m1);
    if (rc != LMI_OK) return rc;
    {
        const WsLayout l = ws_layout(&bd, nq, R, 15, qmode);
        hipLaunchKernelGGL(kth_bound_kernel, dim3((unsigned)P), dim3(64), 0, s,
                           (const uint64_t*)(region + l.partial), l.split_s * bd.max_chunks, l.split_s,
                           (const int32_t*)(region + l.pair_q), (const int32_t*)(region + l.pair_bucket),
                           sub_first, (const uint32_t*)(region + l.split_mask), P, w.kw, idx->bucket_off,
                           w.cap, bound, fix);
        LMI_LAUNCH_CHECK("kth_bound_kernel");
    }
    // 2. every row within the bound -> sorted, the first kw
    const WideScan m2{2, bound, cand, ccount, w.cap, nullptr, 0, nullptr, nullptr};
    rc = bucket_topk_impl(idx, q, nq, ldq, classes, R, 10, qmode, fd, fpos, nullptr, status, region,
                          w.region_bytes, s, nullptr, 0, false, false, 0.0f, plan_scan, &m2);
    if (rc != LMI_OK) return rc;
    {
        const WsLayout l = ws_layout(idx, nq, R, 10, qmode);
        static std::once_flag once;
        static hipError_t attr_err = hipSuccess;
        std::call_once(once, [] {
            attr_err = hipFuncSetAttribute((const void*)collect_select_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 8192 * 8);
        });
        LMI_HIP_TRY(attr_err);
        hipLaunchKernelGGL(collect_select_kernel, dim3((unsigned)P), dim3(256), (size_t)w.cap * 8, s, cand,
                           ccount, w.cap, (const int32_t*)(region + l.pair_q),
                           (const int32_t*)(region + l.pair_bucket), idx->gpos, P, w.kw, ldo, bound, fix,
                           out_d, out_pos, out_row);
        LMI_LAUNCH_CHECK("collect_select_kernel");
    }
    // 3. the pairs without a bound or with too many candidates: the passes,
    //    over their buckets only (every other pair's class is -1)
    if (env_config().wide_no_fixup) return LMI_OK;
    int32_t* cls = (int32_t*)(ws + w.cls);
    hipLaunchKernelGGL(fix_classes_kernel, dim3((P + 255) / 256), dim3(256), 0, s, classes, fix, P, cls);
    LMI_LAUNCH_CHECK("fix_classes_kernel");
    rc = bucket_topk_passes(idx, q, nq, ldq, cls, R, k, qmode, fd, fpos, frow, ldo, status, region,
                            w.region_bytes, s);
    if (rc != LMI_OK) return rc;
    hipLaunchKernelGGL(fix_combine_kernel, dim3((unsigned)((PL + 255) / 256)), dim3(256), 0, s, fix,
                       (int64_t)P, ldo, fd, fpos, frow, out_d, out_pos, out_row);
    LMI_LAUNCH_CHECK("fix_combine_kernel");
    return LMI_OK;
}
}  // namespace lmi


extern "C" int32_t lmi_scan_set_workgroups(int32_t wgs) {
    const int prev = lmi::t_scan_wgs;
    lmi::t_scan_wgs = wgs > 0 ? wgs : 0;
    return prev;
}

extern "C" double lmi_split_eps(int32_t d_pad) { return d_pad > 0 ? lmi::split_eps(d_pad) : 0.0; }

extern "C" int lmi_timing_enable(int32_t on) {
    lmi::Timing& t = lmi::timing();
    std::lock_guard<std::mutex> g(t.mu);
    t.on = on != 0;
    return LMI_OK;
}

extern "C" int32_t lmi_timing_read(float* ms_out, int32_t max_n) {
    using namespace lmi;
    Timing& t = timing();
    std::lock_guard<std::mutex> g(t.mu);
    int32_t n = 0;
    for (auto& pr : t.pending) {
        if (hipEventSynchronize(pr.second) != hipSuccess) {
            set_error("hipEventSynchronize failed");
            return -LMI_E_HIP;
        }
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, pr.first, pr.second) != hipSuccess) {
            set_error("hipEventElapsedTime failed");
            return -LMI_E_HIP;
        }
        if (ms_out && n < max_n) ms_out[n] = ms;
        ++n;
        t.pool.push_back(pr);
    }
    t.pending.clear();
    return std::min(n, max_n);
}
