// A5 on the device — the reference's multi-round bucket merge replayed from the
// per-(query, probe) lists, without a host round trip.
//
// Same semantics as the host replay (lmi_replay.cpp), which restates
//   LearnedIndex.search        search/li/LearnedIndex.py:22-101
//     threshold = running k-th distance    :71-74  (dists_final.max(axis=1))
//     stable merge of rounds              :82-97  (argsort(kind='stable'))
//   LearnedIndex.search_single  search/li/LearnedIndex.py:103-195
//     groups: groupby('category') ascending, queries ascending  :143-147
//     threshold path                      :149-163 -> utils.py:14-43
//     the <k padding quirk                 :174-190
//     broadcast to the whole group         :192-193
// and is checked bit for bit against it (tests/test_gpu_replay.py).
//
// Before round 0 (the GROUPS phase: it needs the classes only, so a stream of
// batches runs it beside the scan), replay_groups_kernel (C x R workgroups)
// lays out every round's groups: the queries with classes[q, r] == c in
// ascending q; replay_thr_kernel resets round 0's rows and thresholds.
// Layout of one round r (R rounds run in order on one stream):
//   replay_group_kernel  per category c (one workgroup) over its group of
//                        round r; thresholded rounds
//                        need U = sorted unique union of the relevant
//                        positions, but only its smallest kr + kl members
//                        matter (fillers and the |U| < kr test), found by
//                        repeated block-wide minimum selection
//   replay_merge_kernel  per element of hstack(F, D_r): its stable rank; it
//                        also resets the next round's rows and writes its
//                        thresholds, and the last merge writes the answer
//                        (ids through pos_to_id, uint32).
#include "lmi_common.hpp"

#include <type_traits>

namespace lmi {
namespace {

constexpr int kT = 256;
constexpr double kFill = 10000.0;  // LearnedIndex.py:138, utils.py:35
constexpr int kMaxW = 64;          // widest merged row held per thread
constexpr int kMaxKr = 32;         // widest round row (k_round)

struct Ent {
    double d;
    int32_t pos;  // global position, -1 = none
};

__device__ inline int block_sum_i(int v, int* sh) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < kT / 64; ++w) t += sh[w];
    __syncthreads();
    return t;
}

__device__ inline int block_min_i(int v, int* sh) {
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    int t = sh[0];
    for (int w = 1; w < kT / 64; ++w) t = min(t, sh[w]);
    __syncthreads();
    return t;
}

extern "C" __device__ int __ockl_wfred_min_i32(int);
extern "C" __device__ int __ockl_wfred_add_i32(int);
// wave-wide minimum (DPP reduction)
__device__ inline int wave_min_i(int v) { return __ockl_wfred_min_i32(v); }

struct RoundArgs {
    const int32_t* classes;
    int32_t nq, R, r, kl, kr, C;
    const void* lists_d;     // [nq][R][kl] float, or double when lists_f64
    int32_t lists_f64;
    const int32_t* lists_p;  // [nq][R][kl]
    const int64_t* bucket_size;
    const int32_t* groups;   // [nq] this round's groups, category c at [g0(c), g1(c))
    const int32_t* gb;       // [C][2] this round's (g0, g1) per category
    int32_t thresholded;
    const double* thr;       // [nq]
    double* dr_d;            // [nq][kr]
    int32_t* dr_p;
    int32_t* uraw;           // [nq * kl] scratch (positions of relevant entries),
                             // category c at [g0 * kl, g1 * kl)
    int32_t* status;
};

// a list distance as the reference holds it: float32 widened, or float64
// (lmi_bucket_topk_f64 lists, the reference's arithmetic on fp16 data)
__device__ inline double list_d(const RoundArgs& a, size_t o) {
    return a.lists_f64 ? reinterpret_cast<const double*>(a.lists_d)[o]
                       : (double)reinterpret_cast<const float*>(a.lists_d)[o];
}

__device__ inline void list_at(const RoundArgs& a, int q, int j, double& d, int32_t& pos) {
    const size_t o = ((size_t)q * a.R + a.r) * a.kl + j;
    pos = a.lists_p[o];
    d = list_d(a, o);
}

// LearnedIndex.py:174-193 (quirk_row of lmi_replay.cpp): row (n_row values),
// u_pos (n_u positions), ann = stable argsort(row); out[kr]
__device__ void quirk_row_dev(const double* row, int n_row, const int32_t* u_pos, int n_u,
                              const int* ann, int n_ann, int kr, Ent* out) {
    const int p = (kr - n_u) / 2 + 1;
    double row_p[kMaxKr], orig[kMaxKr];
    int ann_p[kMaxKr];
    int32_t ids_p[kMaxKr];
    for (int j = 0; j < kr; ++j) {
        const int src = j - p;
        ids_p[j] = u_pos[min(max(src, 0), n_u - 1)];
        ann_p[j] = ann[min(max(src, 0), n_ann - 1)];
        row_p[j] = row[min(max(src, 0), n_row - 1)];
        orig[j] = row_p[j];
    }
    // np.unique(return_index) + setdiff: every repeated value becomes FILL
    for (int j = 0; j < kr; ++j)
        for (int i = 0; i < j; ++i)
            if (orig[i] == orig[j]) {
                row_p[j] = kFill;
                break;
            }
    for (int j = 0; j < kr; ++j) {
        out[j].pos = ids_p[ann_p[j]];
        out[j].d = row_p[ann_p[j]];
    }
}

__device__ void stable_argsort_dev(const double* row, int n, int* idx) {
    for (int i = 0; i < n; ++i) {
        int j = i;
        while (j > 0 && row[idx[j - 1]] > row[i]) {
            idx[j] = idx[j - 1];
            --j;
        }
        idx[j] = i;
    }
}

constexpr int kUCap = 8192;  // relevant positions of a group held in LDS
constexpr int kBmBits = 196608;  // selection bitmap: U's positions spanning < 192K (24 KiB)
constexpr int kTG = 1024;    // group kernel: one large workgroup per category

// sum, min and max over the workgroup in one pass (one barrier; sh3 is used
// once per workgroup, so no trailing barrier)
__device__ inline void block_sum_min_max_g(int& s, int& mn, int& mx, int (*sh3)[kTG / 64]) {
    s = __ockl_wfred_add_i32(s);
    mn = wave_min_i(mn);
    mx = -wave_min_i(-mx);
    if ((threadIdx.x & 63) == 0) {
        sh3[0][threadIdx.x >> 6] = s;
        sh3[1][threadIdx.x >> 6] = mn;
        sh3[2][threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    s = sh3[0][0];
    mn = sh3[1][0];
    mx = sh3[2][0];
    for (int w = 1; w < kTG / 64; ++w) {
        s += sh3[0][w];
        mn = min(mn, sh3[1][w]);
        mx = max(mx, sh3[2][w]);
    }
}

// The groups of every round at once (grid (C + 1) x R), before round 0:
// category c of round r = the queries with classes[q, r] == c in ascending q,
// placed at [g0, g1) of groups[r] with g0 = #{q : cat(q, r) < c}; category C
// collects the queries whose class is outside [0, C) (no group in the
// reference's groupby; they still take part in the merges).  gb is
// [R][C + 1][2].
__device__ inline int cat_of(int v, int C) { return (v >= 0 && v < C) ? v : C; }

__global__ __launch_bounds__(kTG) void replay_groups_kernel(const int32_t* __restrict__ classes,
                                                            int32_t nq, int32_t R, int32_t C,
                                                            int32_t* __restrict__ groups_all,
                                                            int32_t* __restrict__ gb_all) {
    const int c = blockIdx.x, r = blockIdx.y;
    const int tid = threadIdx.x;
    int32_t* groups = groups_all + (size_t)r * nq;
    int32_t* gb = gb_all + ((size_t)r * (C + 1) + c) * 2;
    // every wave takes a contiguous segment of the queries, read coalesced,
    // matches ranked by ballot
    __shared__ int wc[2][kTG / 64];
    const int lane = tid & 63, w = tid >> 6;
    const int seg = ((nq + kTG / 64 - 1) / (kTG / 64) + 63) & ~63;
    const int qa = min(nq, w * seg), qb = min(nq, qa + seg);
    constexpr int kU = 8;  // loads in flight per lane (each pass is latency-bound)
    int n_eq = 0, n_lt = 0;
    for (int q0 = qa; q0 < qb; q0 += kU * 64) {
        int v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int q = q0 + 64 * u + lane;
            v[u] = q < qb ? cat_of(classes[(size_t)q * R + r], C) : INT32_MAX;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            n_eq += __popcll(__ballot(v[u] == c));
            n_lt += __popcll(__ballot(v[u] < c));
        }
    }
    if (lane == 0) {
        wc[0][w] = n_eq;
        wc[1][w] = n_lt;
    }
    __syncthreads();
    int before = 0, n_g = 0, lt = 0;
    for (int i = 0; i < kTG / 64; ++i) {
        before += (i < w) ? wc[0][i] : 0;
        n_g += wc[0][i];
        lt += wc[1][i];
    }
    if (tid == 0) {
        gb[0] = lt;
        gb[1] = lt + n_g;
    }
    if (n_g == 0) return;
    int o = lt + before;
    const uint64_t lanes_lt = (1ull << lane) - 1ull;
    for (int q0 = qa; q0 < qb; q0 += kU * 64) {
        int v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int q = q0 + 64 * u + lane;
            v[u] = q < qb ? cat_of(classes[(size_t)q * R + r], C) : INT32_MAX;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint64_t m = __ballot(v[u] == c);
            if (v[u] == c) groups[o + __popcll(m & lanes_lt)] = q0 + 64 * u + lane;
            o += __popcll(m);
        }
    }
}

__device__ void replay_group_body(const RoundArgs& a, const int c) {
    __shared__ int32_t S[2 * kMaxKr + 16];  // smallest members of U, ascending
    __shared__ Ent qrow[kMaxKr];            // the quirk row of the group
    __shared__ int32_t Ul[kUCap];
    __shared__ int32_t Sw[kTG / 64][2 * kMaxKr];  // per wave: smallest members of its share
    __shared__ int nsw[kTG / 64 + 1];
    __shared__ int wsum[kTG / 64];
    __shared__ uint32_t bm[kBmBits / 32];  // U as a bitmap (positions - umin)
    __shared__ int sh3[3][kTG / 64];
    const int tid = threadIdx.x;
    if (c >= a.C) return;               // out-of-range classes: no group
    if (a.bucket_size[c] <= 0) return;  // groupby visits non-empty categories only
    // the group: queries with classes[q, r] == c in ascending q, placed at
    // [g0, g1) with g0 = #{q : classes[q, r] < c} (disjoint across categories)
    const int g0 = a.gb[2 * c], g1 = a.gb[2 * c + 1];  // (replay_groups_kernel)
    if (g1 <= g0) return;
    const int32_t* G = a.groups;
    const int kr = a.kr;
    const int kl_use = min(kr, a.kl);
    if (a.thresholded) {
        // B_q = leading list entries with d < thr[q] (utils.py:22-23, strict);
        // U = unique positions over the group; only its smallest members matter
        const int nU = (g1 - g0) * kl_use;
        int32_t* U = nU <= kUCap ? Ul : a.uraw + (size_t)g0 * kl_use;
        // entry-parallel: a list is sorted by distance with its empty entries
        // last, so "leading entries with d < thr" is a per-entry test
        // (a popular category's group holds ~10^3 queries: kUL entries per
        // lane with their dependent loads in flight together, not one
        // latency chain per entry)
        constexpr int kUL = 8;
        int nb_tot = 0;
        int umin = INT32_MAX, umax = -1;  // range of U's relevant positions
        // (this thread's first kUL entries stay in registers for the B_q
        // writes below: no second round of dependent global loads)
        int32_t p0v[kUL];
        int q0v[kUL];
        double d0v[kUL];
        for (int e0 = tid; e0 < nU; e0 += kUL * kTG) {
            int qv[kUL];
            size_t ov[kUL];
#pragma unroll
            for (int u = 0; u < kUL; ++u) {
                const int e = e0 + u * kTG;
                const int gi = g0 + e / kl_use, j = e - (e / kl_use) * kl_use;
                qv[u] = e < nU ? G[gi] : 0;
                ov[u] = ((size_t)qv[u] * a.R + a.r) * a.kl + j;
            }
            int32_t pv[kUL];
            double dv[kUL], tv[kUL];
#pragma unroll
            for (int u = 0; u < kUL; ++u) {
                const bool in = e0 + u * kTG < nU;
                pv[u] = in ? a.lists_p[ov[u]] : -1;
                dv[u] = in ? list_d(a, ov[u]) : 0.0;
                tv[u] = in ? a.thr[qv[u]] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < kUL; ++u) {
                const int e = e0 + u * kTG;
                const bool rel = pv[u] >= 0 && dv[u] < tv[u];
                if (e < nU) U[e] = rel ? pv[u] : INT32_MAX;
                nb_tot += rel ? 1 : 0;
                if (rel) {
                    umin = min(umin, pv[u]);
                    umax = max(umax, pv[u]);
                }
                if (e0 == tid) {
                    p0v[u] = (e < nU && rel) ? pv[u] : INT32_MAX;
                    q0v[u] = qv[u];
                    d0v[u] = dv[u];
                }
            }
        }
        block_sum_min_max_g(nb_tot, umin, umax, sh3);  // (its barrier publishes U)
        if (nb_tot == 0) return;  // LearnedIndex.py:157-159
        const int want = kr + kl_use;
        const int lane = tid & 63, wv = tid >> 6;
        if (umax - umin < kBmBits) {
            // U's positions as a bitmap over [umin, umax] (unique by
            // construction), then the `want` lowest set bits by one block-wide
            // prefix count: a few barriers instead of `want` dependent
            // wave-minimum rounds twice over (the bench's groups: ~28 -> a few us)
            const int nw = ((umax - umin) >> 5) + 1;
            for (int i = tid; i < nw; i += kTG) bm[i] = 0u;
            __syncthreads();
            for (int e = tid; e < nU; e += kTG) {
                const int32_t p = U[e];
                if (p != INT32_MAX) atomicOr(&bm[(p - umin) >> 5], 1u << ((p - umin) & 31));
            }
            __syncthreads();
            const int wpt = (nw + kTG - 1) / kTG;
            const int w0 = min(nw, tid * wpt), w1 = min(nw, w0 + wpt);
            int cnt_t = 0;
            for (int i = w0; i < w1; ++i) cnt_t += __popc(bm[i]);
            int incl = cnt_t;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(incl, off);
                if (lane >= off) incl += y;
            }
            if (lane == 63) wsum[wv] = incl;
            __syncthreads();
            int pre = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < kTG / 64; ++w) {
                pre += (w < wv) ? wsum[w] : 0;
                tot += wsum[w];
            }
            int o = pre + incl - cnt_t;  // set bits before this thread's words
            for (int i = w0; i < w1 && o < want; ++i) {
                uint32_t m = bm[i];
                while (m != 0u && o < want) {
                    const int b = __builtin_ctz(m);
                    m &= m - 1u;
                    S[o++] = umin + 32 * i + b;
                }
            }
            if (tid == 0) nsw[kTG / 64] = min(tot, want);
        } else {
        // the smallest `want` members of U: each wave finds those of its
        // share (every 4th 64-entry run), then wave 0 merges the four lists
        // (a global member among the smallest `want` is among its share's)
        int prev = -1, cnt = 0;
        // the lane's share (<= NR entries) read once into registers, then the
        // `want` rounds run on them; NR by the group's size (the compares of
        // a round scale with it: 2 at the bench's groups of <= 253 queries,
        // up to 16 for a popular category's 10^3 queries past the LDS staging)
        auto sel = [&](auto nr) {
            constexpr int NR = decltype(nr)::value;
            int uc[NR];
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                const int e = wv * 64 + lane + i * kTG;
                uc[i] = e < nU ? U[e] : INT32_MAX;
            }
            for (; cnt < want; ++cnt) {
                int m = INT32_MAX;
#pragma unroll
                for (int i = 0; i < NR; ++i)
                    if (uc[i] > prev && uc[i] < m) m = uc[i];
                m = wave_min_i(m);
                if (m == INT32_MAX) break;
                if (lane == 0) Sw[wv][cnt] = m;
                prev = m;
            }
        };
        if (nU <= 2 * kTG) {
            sel(std::integral_constant<int, 2>{});
        } else if (nU <= 4 * kTG) {
            sel(std::integral_constant<int, 4>{});
        } else if (nU <= 8 * kTG) {
            sel(std::integral_constant<int, 8>{});
        } else if (nU <= 16 * kTG) {
            sel(std::integral_constant<int, 16>{});
        } else {
            for (; cnt < want; ++cnt) {
                int m = INT32_MAX;
                for (int e = wv * 64 + lane; e < nU; e += kTG) {
                    const int32_t p = U[e];
                    if (p > prev && p < m) m = p;
                }
                m = wave_min_i(m);
                if (m == INT32_MAX) break;
                if (lane == 0) Sw[wv][cnt] = m;
                prev = m;
            }
        }
        if (lane == 0) nsw[wv] = cnt;
        __syncthreads();
        if (wv == 0) {
            // the 16 wave lists (<= want entries each) packed want-major over
            // the lanes: NV registers per lane for 16 * want entries
            auto mrg = [&](auto nv) {
                constexpr int NV = decltype(nv)::value;
                int v[NV];
#pragma unroll
                for (int t = 0; t < NV; ++t) {
                    const int e = lane + 64 * t, w = e / want, i = e - w * want;
                    v[t] = (w < kTG / 64 && i < nsw[w]) ? Sw[w][i] : INT32_MAX;
                }
                int pv = -1, n = 0;
                for (; n < want; ++n) {
                    int m = INT32_MAX;
#pragma unroll
                    for (int t = 0; t < NV; ++t)
                        if (v[t] > pv && v[t] < m) m = v[t];
                    m = wave_min_i(m);
                    if (m == INT32_MAX) break;
                    if (lane == 0) S[n] = m;
                    pv = m;
                }
                if (lane == 0) nsw[kTG / 64] = n;
            };
            static_assert((kTG / 64) * (2 * kMaxKr) <= 16 * 64, "merge registers");
            if ((kTG / 64) * want <= 4 * 64)
                mrg(std::integral_constant<int, 4>{});
            else if ((kTG / 64) * want <= 8 * 64)
                mrg(std::integral_constant<int, 8>{});
            else
                mrg(std::integral_constant<int, 16>{});
        }
        }  // (register selection)
        __syncthreads();
        const int ns = nsw[kTG / 64];
        __syncthreads();
        if (ns >= kr) {
            // normal case: B_q then the smallest members of U not in B_q;
            // B_q entry-parallel (U holds its positions), then per query the
            // fillers, membership tested against its U row
            for (int e0 = tid; e0 < nU; e0 += kUL * kTG) {
                int32_t pv[kUL];
                int qv[kUL];
                double dv[kUL];
                if (e0 == tid) {
#pragma unroll
                    for (int u = 0; u < kUL; ++u) {
                        pv[u] = p0v[u];
                        qv[u] = q0v[u];
                        dv[u] = d0v[u];
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < kUL; ++u) {
                        const int e = e0 + u * kTG;
                        pv[u] = e < nU ? U[e] : INT32_MAX;
                        const int gi = g0 + e / kl_use;
                        qv[u] = pv[u] != INT32_MAX ? G[gi] : 0;
                    }
#pragma unroll
                    for (int u = 0; u < kUL; ++u) {
                        const int e = e0 + u * kTG;
                        const int j = e - (e / kl_use) * kl_use;
                        dv[u] = pv[u] != INT32_MAX ? list_d(a, ((size_t)qv[u] * a.R + a.r) * a.kl + j) : 0.0;
                    }
                }
#pragma unroll
                for (int u = 0; u < kUL; ++u) {
                    if (pv[u] == INT32_MAX) continue;
                    const int e = e0 + u * kTG;
                    const int j = e - (e / kl_use) * kl_use;
                    a.dr_d[(size_t)qv[u] * kr + j] = dv[u];
                    a.dr_p[(size_t)qv[u] * kr + j] = pv[u];
                }
            }
            // the query's relevant positions in NL registers (NL >= kl_use:
            // 10 at the bench's k, so the membership test of each of the ns
            // smallest members of U is 10 compares, not kMaxKr)
            auto fill = [&](auto nl) {
                constexpr int NL = decltype(nl)::value;
                for (int gi = g0 + tid; gi < g1; gi += kTG) {
                    const int q = G[gi];
                    const int32_t* u = U + (size_t)(gi - g0) * kl_use;
                    int32_t lp[NL];
                    int n_rel = 0;
#pragma unroll
                    for (int j = 0; j < NL; ++j) {
                        lp[j] = j < kl_use ? u[j] : INT32_MAX;
                        n_rel += lp[j] != INT32_MAX ? 1 : 0;
                    }
                    double* od = a.dr_d + (size_t)q * kr;
                    int32_t* op = a.dr_p + (size_t)q * kr;
                    int n = n_rel;
                    for (int v = 0; v < ns && n < kr; ++v) {
                        const int32_t sv = S[v];
                        bool mine = false;
#pragma unroll
                        for (int j = 0; j < NL; ++j) mine |= lp[j] == sv;
                        if (!mine) {
                            od[n] = kFill;
                            op[n] = sv;
                            ++n;
                        }
                    }
                    if (n < kr) atomicOr(a.status, 1);  // cannot happen: |U| >= kr
                }
            };
            static_assert(kMaxKr == 32, "membership widths");
            if (kl_use <= 10)
                fill(std::integral_constant<int, 10>{});
            else if (kl_use <= 16)
                fill(std::integral_constant<int, 16>{});
            else
                fill(std::integral_constant<int, 32>{});
        } else {
            // |U| < kr: the quirk on row 0 (q0 = first query of the group)
            if (tid == 0) {
                const int q0 = G[g0];
                double row[kMaxKr];
                int ann[kMaxKr];
                for (int j = 0; j < kr; ++j) row[j] = kFill;
                for (int j = 0; j < kl_use; ++j) {
                    double d;
                    int32_t pos;
                    list_at(a, q0, j, d, pos);
                    if (pos < 0 || !(d < a.thr[q0])) break;
                    int at = 0;
                    while (at < ns && S[at] < pos) ++at;
                    row[at] = d;
                }
                stable_argsort_dev(row, kr, ann);
                quirk_row_dev(row, kr, S, ns, ann, kr, kr, qrow);
            }
            __syncthreads();
            for (int gi = g0 + tid; gi < g1; gi += kTG) {
                const int q = G[gi];
                for (int j = 0; j < kr; ++j) {
                    a.dr_d[(size_t)q * kr + j] = qrow[j].d;
                    a.dr_p[(size_t)q * kr + j] = qrow[j].pos;
                }
            }
        }
    } else {
        const int64_t n = a.bucket_size[c];
        if (n >= kr) {
            for (int gi = g0 + tid; gi < g1; gi += kTG) {
                const int q = G[gi];
                // 8 entries' loads in flight before their stores (the stores
                // may alias the lists for the compiler: one chain per entry)
                for (int j0 = 0; j0 < kr; j0 += 8) {
                    double dv[8];
                    int32_t pv[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (j0 + u < kr) list_at(a, q, j0 + u, dv[u], pv[u]);
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (j0 + u < kr) {
                            a.dr_d[(size_t)q * kr + j0 + u] = dv[u];
                            a.dr_p[(size_t)q * kr + j0 + u] = pv[u];
                        }
                    }
                }
            }
        } else {
            // bucket smaller than kr: row 0 = q0's distances to the whole
            // bucket in position order, then the quirk
            if (tid == 0) {
                const int q0 = G[g0];
                double row[kMaxKr];
                int32_t upos[kMaxKr];
                int ann[kMaxKr];
                int m = 0;
                for (int j = 0; j < kl_use && j < (int)n; ++j) {
                    double d;
                    int32_t pos;
                    list_at(a, q0, j, d, pos);
                    if (pos < 0) break;
                    int at = m++;
                    while (at > 0 && upos[at - 1] > pos) {  // insertion by position
                        upos[at] = upos[at - 1];
                        row[at] = row[at - 1];
                        --at;
                    }
                    upos[at] = pos;
                    row[at] = d;
                }
                if (m != (int)n) atomicOr(a.status, 2);
                if (m > 0) {
                    stable_argsort_dev(row, m, ann);
                    quirk_row_dev(row, m, upos, m, ann, m, kr, qrow);
                }
            }
            __syncthreads();
            for (int gi = g0 + tid; gi < g1; gi += kTG) {
                const int q = G[gi];
                for (int j = 0; j < kr; ++j) {
                    a.dr_d[(size_t)q * kr + j] = qrow[j].d;
                    a.dr_p[(size_t)q * kr + j] = qrow[j].pos;
                }
            }
        }
    }
}

__global__ __launch_bounds__(kTG) void replay_group_kernel(RoundArgs a) {
    replay_group_body(a, blockIdx.x);
}

__global__ __launch_bounds__(kT) void replay_thr_kernel(int32_t nq, int32_t kr, int32_t fs,
                                                        int32_t wF, int32_t mode,
                                                        const double* __restrict__ Fd,
                                                        const double* __restrict__ thr0,
                                                        double* __restrict__ thr,
                                                        double* __restrict__ dr_d,
                                                        int32_t* __restrict__ dr_p,
                                                        int32_t* __restrict__ zero_status) {
    const int q = blockIdx.x * kT + threadIdx.x;
    if (zero_status && q == 0) *zero_status = 0;  // (the phased replay's GROUPS phase)
    if (q >= nq) return;
    for (int j = 0; j < kr; ++j) {
        dr_d[(size_t)q * kr + j] = kFill;
        dr_p[(size_t)q * kr + j] = -1;
    }
    if (mode == 1) {
        thr[q] = thr0[q];
    } else if (mode == 2) {
        double m = Fd[(size_t)q * fs];
        for (int j = 1; j < wF; ++j) m = fmax(m, Fd[(size_t)q * fs + j]);
        thr[q] = m;
    }
}

// LearnedIndex.py:82-97: the first wn of argsort(hstack(F, D_r), kind='stable'),
// one thread per element of the concatenation: its stable rank is
// #{i : d_i < d_j} + #{i < j : d_i == d_j}.  F is read from one buffer and the
// merged row written to the other (ping-pong across rounds).
__global__ __launch_bounds__(kT) void replay_merge_kernel(int32_t nq, int32_t kr, int32_t fs,
                                                          int32_t wF, int32_t wn, int32_t first,
                                                          const double* __restrict__ Fd,
                                                          const int32_t* __restrict__ Fp,
                                                          double* __restrict__ Fd_out,
                                                          int32_t* __restrict__ Fp_out,
                                                          const double* __restrict__ dr_d,
                                                          const int32_t* __restrict__ dr_p,
                                                          double* __restrict__ thr_next,
                                                          double* __restrict__ drd_next,
                                                          int32_t* __restrict__ drp_next,
                                                          const int64_t* __restrict__ pos_to_id,
                                                          int64_t n_total, double* __restrict__ dists,
                                                          uint32_t* __restrict__ anns,
                                                          int32_t* __restrict__ status) {
    // fused prologue of the next round (replay_thr_kernel's mode 2): its row
    // buffers (the other pair) reset to (10000, -1), and its threshold
    // max(F_q) written by the thread that places F's last element
    const int n = first ? kr : wF + kr;
    const int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (t >= (int64_t)nq * n) return;
    const int q = (int)(t / n), j = (int)(t - (int64_t)q * n);
    const double* fd = Fd + (size_t)q * fs;
    const double* dd = dr_d + (size_t)q * kr;
    if (drd_next && j < kr) {
        drd_next[(size_t)q * kr + j] = kFill;
        drp_next[(size_t)q * kr + j] = -1;
    }
    // the last merge (dists non-null) writes the answer itself: positions ->
    // ids through pos_to_id, uint32 (one launch less than a separate output
    // pass).  (A lambda capturing by reference kept its captures on the
    // stack: 40 B of scratch per thread.)
#define LMI_PUT(AT, V, P)                                                              \
    do {                                                                               \
        const int at_ = (AT);                                                          \
        const double v_ = (V);                                                         \
        const int32_t p_ = (P);                                                        \
        if (dists) {                                                                   \
            int64_t id = 0;                                                            \
            if (p_ >= 0) {                                                             \
                if (p_ < n_total) id = pos_to_id[p_];                                  \
                else atomicOr(status, 4);                                              \
            }                                                                          \
            dists[(size_t)q * wn + at_] = v_;                                          \
            anns[(size_t)q * wn + at_] = (uint32_t)id; /* numpy int64 -> uint32 */     \
        } else {                                                                       \
            Fd_out[(size_t)q * fs + at_] = v_;                                         \
            Fp_out[(size_t)q * fs + at_] = p_;                                         \
        }                                                                              \
    } while (0)
    if (first) {
        LMI_PUT(j, dd[j], dr_p[(size_t)q * kr + j]);
        if (thr_next && j == 0) {  // round 0's row need not be ascending (the <k quirk)
            double m = dd[0];
            for (int i = 1; i < kr; ++i) m = fmax(m, dd[i]);
            thr_next[q] = m;
        }
        return;
    }
    const double dj = j < wF ? fd[j] : dd[j - wF];
    int rank = 0;
    for (int i = 0; i < wF; ++i) {
        const double di = fd[i];
        rank += (di < dj || (di == dj && i < j)) ? 1 : 0;
    }
    for (int i = 0; i < kr; ++i) {
        const double di = dd[i];
        rank += (di < dj || (di == dj && wF + i < j)) ? 1 : 0;
    }
    if (rank < wn) LMI_PUT(rank, dj, j < wF ? Fp[(size_t)q * fs + j] : dr_p[(size_t)q * kr + j - wF]);
    if (thr_next && rank == wn - 1) thr_next[q] = dj;  // the merged row is ascending
#undef LMI_PUT
}

struct ReplayWs {
    size_t groups, gb, Fd[2], Fp[2], drd[2], drp[2], thr, uraw, total;
};

ReplayWs replay_ws(int nq, int R, int kl, int kr, int w, int C) {
    ReplayWs s{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t at = off;
        off = align_up(off + bytes, 256);
        return at;
    };
    const int fs = std::max(kr, w);
    s.groups = take((size_t)R * nq * 4);
    s.gb = take((size_t)R * (C + 1) * 2 * 4);
    for (int b = 0; b < 2; ++b) {
        s.Fd[b] = take((size_t)nq * fs * 8);
        s.Fp[b] = take((size_t)nq * fs * 4);
    }
    for (int b = 0; b < 2; ++b) {  // round r's rows live in buffer r & 1
        s.drd[b] = take((size_t)nq * kr * 8);
        s.drp[b] = take((size_t)nq * kr * 4);
    }
    s.thr = take((size_t)nq * 8);
    s.uraw = take((size_t)nq * kl * 4);  // one round's (the rounds run one after another)
    s.total = off;
    return s;
}

}  // namespace
}  // namespace lmi

extern "C" size_t lmi_replay_device_workspace_bytes(int32_t nq, int32_t R, int32_t k_list,
                                                    int32_t k_round, int32_t k_final,
                                                    int32_t n_buckets) {
    if (nq < 0 || R < 1 || k_list < 1 || k_round < 1 || k_final < 1 || n_buckets < 1) return 0;
    const int w = R == 1 ? k_round : k_final;
    return lmi::replay_ws(nq, R, k_list, k_round, w, n_buckets).total;
}

namespace lmi {
int replay_device_impl(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                       const void* lists_d, int lists_f64, const int32_t* lists_pos,
                       int32_t k_round, int32_t k_final, const int64_t* bucket_size,
                       int32_t n_buckets, const int64_t* pos_to_id, int64_t n_total,
                       int32_t use_threshold, const double* thr_round0, double* dists_out,
                       uint32_t* anns_out, int32_t* status, void* workspace, size_t ws_bytes,
                       void* stream, int32_t phases = LMI_REPLAY_PHASE_GROUPS | LMI_REPLAY_PHASE_ROUNDS);
}  // namespace lmi

extern "C" int lmi_replay_device(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                                 const float* lists_d, const int32_t* lists_pos, int32_t k_round,
                                 int32_t k_final, const int64_t* bucket_size, int32_t n_buckets,
                                 const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
                                 const double* thr_round0, double* dists_out, uint32_t* anns_out,
                                 int32_t* status, void* workspace, size_t ws_bytes, void* stream) {
    return lmi::replay_device_impl(classes, nq, R, k_list, lists_d, 0, lists_pos, k_round, k_final,
                                   bucket_size, n_buckets, pos_to_id, n_total, use_threshold,
                                   thr_round0, dists_out, anns_out, status, workspace, ws_bytes,
                                   stream);
}

extern "C" int lmi_replay_device_f64(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                                     const double* lists_d, const int32_t* lists_pos,
                                     int32_t k_round, int32_t k_final, const int64_t* bucket_size,
                                     int32_t n_buckets, const int64_t* pos_to_id, int64_t n_total,
                                     int32_t use_threshold, const double* thr_round0,
                                     double* dists_out, uint32_t* anns_out, int32_t* status,
                                     void* workspace, size_t ws_bytes, void* stream) {
    return lmi::replay_device_impl(classes, nq, R, k_list, lists_d, 1, lists_pos, k_round, k_final,
                                   bucket_size, n_buckets, pos_to_id, n_total, use_threshold,
                                   thr_round0, dists_out, anns_out, status, workspace, ws_bytes,
                                   stream);
}

extern "C" int lmi_replay_device_phase(int32_t phases, int32_t lists_f64, const int32_t* classes, int32_t nq,
                                       int32_t R, int32_t k_list, const void* lists_d,
                                       const int32_t* lists_pos, int32_t k_round, int32_t k_final,
                                       const int64_t* bucket_size, int32_t n_buckets,
                                       const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
                                       const double* thr_round0, double* dists_out, uint32_t* anns_out,
                                       int32_t* status, void* workspace, size_t ws_bytes, void* stream) {
    return lmi::replay_device_impl(classes, nq, R, k_list, lists_d, lists_f64 ? 1 : 0, lists_pos, k_round,
                                   k_final, bucket_size, n_buckets, pos_to_id, n_total, use_threshold,
                                   thr_round0, dists_out, anns_out, status, workspace, ws_bytes, stream,
                                   phases);
}

int lmi::replay_device_impl(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                            const void* lists_d, int lists_f64, const int32_t* lists_pos,
                            int32_t k_round, int32_t k_final, const int64_t* bucket_size,
                            int32_t n_buckets, const int64_t* pos_to_id, int64_t n_total,
                            int32_t use_threshold, const double* thr_round0, double* dists_out,
                            uint32_t* anns_out, int32_t* status, void* workspace, size_t ws_bytes,
                            void* stream, int32_t phases) {
    using namespace lmi;
    LMI_CHECK_ARG(nq >= 0 && R >= 1 && k_round >= 1 && k_final >= 1 && k_list >= 1 && n_buckets >= 1,
                  "lmi_replay_device: bad sizes");
    LMI_CHECK_ARG(k_round <= kMaxKr, "lmi_replay_device: k_round=%d > %d", k_round, kMaxKr);
    LMI_CHECK_ARG(k_final <= kMaxW, "lmi_replay_device: k=%d > %d", k_final, kMaxW);
    LMI_CHECK_ARG(k_list >= k_round, "lmi_replay_device: lists of %d < k_round=%d", k_list, k_round);
    LMI_CHECK_ARG(phases >= 1 && phases <= 3, "lmi_replay_device: bad phases %d", phases);
    int w = k_round;
    for (int r = 1; r < R; ++r) {
        w = std::min(k_final, w + k_round);
        if (w != k_final) {
            set_error("lmi_replay_device: k=%d exceeds the merged width %d (reference assert, "
                      "LearnedIndex.py:99)", k_final, w);
            return LMI_E_INVALID;
        }
    }
    if (nq == 0) return LMI_OK;
    const bool do_groups = phases & LMI_REPLAY_PHASE_GROUPS, do_rounds = phases & LMI_REPLAY_PHASE_ROUNDS;
    LMI_CHECK_ARG(classes && bucket_size && status && workspace, "lmi_replay_device: null pointer");
    LMI_CHECK_ARG(!do_rounds || (lists_d && lists_pos && pos_to_id && dists_out && anns_out),
                  "lmi_replay_device: null pointer");
    const ReplayWs s = replay_ws(nq, R, k_list, k_round, w, n_buckets);
    if (ws_bytes < s.total) {
        set_error("workspace %zu B < required %zu B", ws_bytes, s.total);
        return LMI_E_WORKSPACE;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    const int C = n_buckets;
    const int fs = std::max(k_round, w);
    int32_t* groups = (int32_t*)(ws + s.groups);
    int32_t* gb = (int32_t*)(ws + s.gb);
    const dim3 qgrid((unsigned)((nq + kT - 1) / kT));
    auto thresholded_at = [&](int r) { return ((r > 0) && use_threshold) || (r == 0 && thr_round0); };
    if (do_groups) {
        // every round's groups ((C + 1) x R workgroups) and round 0's prologue:
        // its rows reset, its thresholds (the caller's, or none); the phased
        // call (GROUPS alone) also zeroes the status word.  They depend on the
        // classes only: a stream of batches runs them beside the scan.
        hipLaunchKernelGGL(replay_groups_kernel, dim3(C + 1, R), dim3(kTG), 0, st, classes, nq, R, C, groups, gb);
        LMI_LAUNCH_CHECK("replay_groups_kernel");
        const int mode = thr_round0 ? 1 : 0;
        hipLaunchKernelGGL(replay_thr_kernel, qgrid, dim3(kT), 0, st, nq, k_round, fs, 0, mode,
                           (const double*)(ws + s.Fd[0]), thr_round0, (double*)(ws + s.thr),
                           (double*)(ws + s.drd[0]), (int32_t*)(ws + s.drp[0]),
                           do_rounds ? nullptr : status);
        LMI_LAUNCH_CHECK("replay_thr_kernel");
    }
    if (!do_rounds) return LMI_OK;
    auto round_args = [&](int r) {
        RoundArgs a{};
        a.classes = classes;
        a.nq = nq;
        a.R = R;
        a.r = r;
        a.kl = k_list;
        a.kr = k_round;
        a.C = C;
        a.lists_d = lists_d;
        a.lists_f64 = lists_f64;
        a.lists_p = lists_pos;
        a.bucket_size = bucket_size;
        a.groups = groups + (size_t)r * nq;
        a.gb = gb + (size_t)r * (C + 1) * 2;
        a.thresholded = thresholded_at(r) ? 1 : 0;
        a.thr = (const double*)(ws + s.thr);
        a.dr_d = (double*)(ws + s.drd[r & 1]);
        a.dr_p = (int32_t*)(ws + s.drp[r & 1]);
        a.uraw = (int32_t*)(ws + s.uraw);
        a.status = status;
        return a;
    };
    int cur = 0;  // F lives in buffer cur; a merge writes the other one
    int wF = 0;
    for (int r = 0; r < R; ++r) {
        double* Fd = (double*)(ws + s.Fd[cur]);
        int32_t* Fp = (int32_t*)(ws + s.Fp[cur]);
        double* drd = (double*)(ws + s.drd[r & 1]);
        int32_t* drp = (int32_t*)(ws + s.drp[r & 1]);
        const bool last = r + 1 == R;
        const int wn = (r == 0) ? k_round : std::min(k_final, wF + k_round);
        hipLaunchKernelGGL(replay_group_kernel, dim3(C), dim3(kTG), 0, st, round_args(r));
        LMI_LAUNCH_CHECK("replay_group_kernel");
        const int n = (r == 0) ? k_round : wF + k_round;
        const dim3 mgrid((unsigned)(((int64_t)nq * n + kT - 1) / kT));
        // (the last merge writes the answer: w == wn there)
        hipLaunchKernelGGL(replay_merge_kernel, mgrid, dim3(kT), 0, st, nq, k_round, fs, wF, wn,
                           r == 0 ? 1 : 0, Fd, Fp, (double*)(ws + s.Fd[cur ^ 1]),
                           (int32_t*)(ws + s.Fp[cur ^ 1]), drd, drp,
                           last ? nullptr : (double*)(ws + s.thr),
                           last ? nullptr : (double*)(ws + s.drd[(r + 1) & 1]),
                           last ? nullptr : (int32_t*)(ws + s.drp[(r + 1) & 1]), pos_to_id, n_total,
                           last ? dists_out : nullptr, anns_out, status);
        LMI_LAUNCH_CHECK("replay_merge_kernel");
        cur ^= 1;
        wF = wn;
    }
    return LMI_OK;
}
