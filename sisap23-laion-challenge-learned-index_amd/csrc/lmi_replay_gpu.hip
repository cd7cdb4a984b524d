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
// Layout of one round r (R rounds run in order on one stream):
//   replay_thr_kernel    per query: thr = max of the merged row; D_r <- (FILL, -1)
//   replay_group_kernel  per category c (one workgroup): the queries with
//                        classes[q, r] == c in ascending q; thresholded rounds
//                        need U = sorted unique union of the relevant
//                        positions, but only its smallest kr + kl members
//                        matter (fillers and the |U| < kr test), found by
//                        repeated block-wide minimum selection
//   replay_merge_kernel  per query: stable insertion sort of hstack(F, D_r)
// followed by replay_out_kernel (ids through pos_to_id, uint32).
#include "lmi_common.hpp"

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

// counts[r][c] = #{q : classes[q, r] == c}
__global__ __launch_bounds__(kT) void replay_count_kernel(const int32_t* __restrict__ classes,
                                                          int32_t nq, int32_t R, int32_t C,
                                                          int32_t* __restrict__ counts) {
    __shared__ int sh[kT / 64];
    const int c = blockIdx.x;
    for (int r = 0; r < R; ++r) {
        int n = 0;
        for (int q = threadIdx.x; q < nq; q += kT) n += (classes[(size_t)q * R + r] == c) ? 1 : 0;
        n = block_sum_i(n, sh);
        if (threadIdx.x == 0) counts[r * C + c] = n;
    }
}

// groups[r][goff(r, c) + i] = i-th query (ascending) with classes[q, r] == c
__global__ __launch_bounds__(kT) void replay_group_fill_kernel(const int32_t* __restrict__ classes,
                                                               int32_t nq, int32_t R, int32_t C,
                                                               const int32_t* __restrict__ counts,
                                                               int32_t* __restrict__ goff,
                                                               int32_t* __restrict__ groups) {
    __shared__ int sh[kT / 64];
    __shared__ int wcnt[kT / 64];
    const int c = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int r = 0; r < R; ++r) {
        int off = 0;
        for (int b = tid; b < c; b += kT) off += counts[r * C + b];
        off = block_sum_i(off, sh);
        if (tid == 0) {
            goff[r * (C + 1) + c] = off;
            if (c == C - 1) goff[r * (C + 1) + C] = off + counts[r * C + c];
        }
        int run = 0;
        for (int base = 0; base < nq; base += kT) {
            const int q = base + tid;
            const bool pred = (q < nq) && (classes[(size_t)q * R + r] == c);
            const uint64_t m = __ballot(pred);
            const int rank = __popcll(m & ((1ull << lane) - 1ull));
            __syncthreads();
            if (lane == 0) wcnt[w] = __popcll(m);
            __syncthreads();
            int wpre = 0, tot = 0;
            for (int i = 0; i < kT / 64; ++i) {
                wpre += (i < w) ? wcnt[i] : 0;
                tot += wcnt[i];
            }
            if (pred) groups[(size_t)r * nq + off + run + wpre + rank] = q;
            run += tot;
        }
        __syncthreads();
    }
}

struct RoundArgs {
    const int32_t* classes;
    int32_t nq, R, r, kl, kr, C;
    const float* lists_d;    // [nq][R][kl]
    const int32_t* lists_p;  // [nq][R][kl]
    const int64_t* bucket_size;
    const int32_t* groups;   // [R][nq]
    const int32_t* goff;     // [R][C+1]
    int32_t thresholded;
    const double* thr;       // [nq]
    double* dr_d;            // [nq][kr]
    int32_t* dr_p;
    int32_t* uraw;           // [nq * kl] scratch (positions of relevant entries)
    int32_t* status;
};

__device__ inline void list_at(const RoundArgs& a, int q, int j, double& d, int32_t& pos) {
    const size_t o = ((size_t)q * a.R + a.r) * a.kl + j;
    pos = a.lists_p[o];
    d = (double)a.lists_d[o];
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

__global__ __launch_bounds__(kT) void replay_group_kernel(RoundArgs a) {
    __shared__ int sh[kT / 64];
    __shared__ int32_t S[2 * kMaxKr + 16];  // smallest members of U, ascending
    __shared__ Ent qrow[kMaxKr];            // the quirk row of the group
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    const int g0 = a.goff[a.r * (a.C + 1) + c], g1 = a.goff[a.r * (a.C + 1) + c + 1];
    if (g0 == g1 || a.bucket_size[c] <= 0) return;  // groupby visits non-empty categories only
    const int32_t* G = a.groups + (size_t)a.r * a.nq;
    const int kr = a.kr;
    const int kl_use = min(kr, a.kl);
    if (a.thresholded) {
        // B_q = leading list entries with d < thr[q] (utils.py:22-23, strict);
        // U = unique positions over the group; only its smallest members matter
        int nb_tot = 0;
        for (int gi = g0 + tid; gi < g1; gi += kT) {
            const int q = G[gi];
            int n = 0;
            for (int j = 0; j < kl_use; ++j) {
                double d;
                int32_t pos;
                list_at(a, q, j, d, pos);
                if (pos < 0 || !(d < a.thr[q])) break;
                a.uraw[(size_t)q * a.kl + j] = pos;
                ++n;
            }
            for (int j = n; j < a.kl; ++j) a.uraw[(size_t)q * a.kl + j] = INT32_MAX;
            nb_tot += n;
        }
        nb_tot = block_sum_i(nb_tot, sh);
        if (nb_tot == 0) return;  // LearnedIndex.py:157-159
        const int want = kr + kl_use;
        int ns = 0, prev = -1;
        for (; ns < want; ++ns) {
            int m = INT32_MAX;
            for (int gi = g0 + tid; gi < g1; gi += kT) {
                const int q = G[gi];
                for (int j = 0; j < kl_use; ++j) {
                    const int32_t p = a.uraw[(size_t)q * a.kl + j];
                    if (p == INT32_MAX) break;
                    if (p > prev && p < m) m = p;
                }
            }
            m = block_min_i(m, sh);
            if (m == INT32_MAX) break;
            if (tid == 0) S[ns] = m;
            prev = m;
        }
        __syncthreads();
        if (ns >= kr) {
            // normal case: B_q then the smallest members of U not in B_q
            for (int gi = g0 + tid; gi < g1; gi += kT) {
                const int q = G[gi];
                double* od = a.dr_d + (size_t)q * kr;
                int32_t* op = a.dr_p + (size_t)q * kr;
                int n = 0, n_rel;
                for (int j = 0; j < kl_use && n < kr; ++j) {
                    double d;
                    int32_t pos;
                    list_at(a, q, j, d, pos);
                    if (pos < 0 || !(d < a.thr[q])) break;
                    od[n] = d;
                    op[n] = pos;
                    ++n;
                }
                n_rel = n;
                for (int u = 0; u < ns && n < kr; ++u) {
                    bool mine = false;
                    for (int j = 0; j < n_rel; ++j) mine |= (op[j] == S[u]);
                    if (!mine) {
                        od[n] = kFill;
                        op[n] = S[u];
                        ++n;
                    }
                }
                if (n < kr) atomicOr(a.status, 1);  // cannot happen: |U| >= kr
            }
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
            for (int gi = g0 + tid; gi < g1; gi += kT) {
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
            for (int gi = g0 + tid; gi < g1; gi += kT) {
                const int q = G[gi];
                for (int j = 0; j < kr; ++j) {
                    double d;
                    int32_t pos;
                    list_at(a, q, j, d, pos);
                    a.dr_d[(size_t)q * kr + j] = d;
                    a.dr_p[(size_t)q * kr + j] = pos;
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
            for (int gi = g0 + tid; gi < g1; gi += kT) {
                const int q = G[gi];
                for (int j = 0; j < kr; ++j) {
                    a.dr_d[(size_t)q * kr + j] = qrow[j].d;
                    a.dr_p[(size_t)q * kr + j] = qrow[j].pos;
                }
            }
        }
    }
}

__global__ __launch_bounds__(kT) void replay_thr_kernel(int32_t nq, int32_t kr, int32_t fs,
                                                        int32_t wF, int32_t mode,
                                                        const double* __restrict__ Fd,
                                                        const double* __restrict__ thr0,
                                                        double* __restrict__ thr,
                                                        double* __restrict__ dr_d,
                                                        int32_t* __restrict__ dr_p) {
    const int q = blockIdx.x * kT + threadIdx.x;
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

__global__ __launch_bounds__(kT) void replay_merge_kernel(int32_t nq, int32_t kr, int32_t fs,
                                                          int32_t wF, int32_t wn, int32_t first,
                                                          double* __restrict__ Fd,
                                                          int32_t* __restrict__ Fp,
                                                          const double* __restrict__ dr_d,
                                                          const int32_t* __restrict__ dr_p) {
    const int q = blockIdx.x * kT + threadIdx.x;
    if (q >= nq) return;
    if (first) {
        for (int j = 0; j < kr; ++j) {
            Fd[(size_t)q * fs + j] = dr_d[(size_t)q * kr + j];
            Fp[(size_t)q * fs + j] = dr_p[(size_t)q * kr + j];
        }
        return;
    }
    // stable sort of hstack(F, D_r) by distance (argsort(kind='stable')), first wn
    Ent cat[kMaxW + kMaxKr];
    int len = 0;
    for (int j = 0; j < wF + kr; ++j) {
        const Ent e = j < wF ? Ent{Fd[(size_t)q * fs + j], Fp[(size_t)q * fs + j]}
                             : Ent{dr_d[(size_t)q * kr + (j - wF)], dr_p[(size_t)q * kr + (j - wF)]};
        int i = len++;
        while (i > 0 && cat[i - 1].d > e.d) {
            cat[i] = cat[i - 1];
            --i;
        }
        cat[i] = e;
    }
    for (int j = 0; j < wn; ++j) {
        Fd[(size_t)q * fs + j] = cat[j].d;
        Fp[(size_t)q * fs + j] = cat[j].pos;
    }
}

__global__ __launch_bounds__(kT) void replay_out_kernel(int32_t nq, int32_t w, int32_t fs,
                                                        const double* __restrict__ Fd,
                                                        const int32_t* __restrict__ Fp,
                                                        const int64_t* __restrict__ pos_to_id,
                                                        int64_t n_total, double* __restrict__ dists,
                                                        uint32_t* __restrict__ anns,
                                                        int32_t* __restrict__ status) {
    const int q = blockIdx.x * kT + threadIdx.x;
    if (q >= nq) return;
    for (int j = 0; j < w; ++j) {
        const int32_t p = Fp[(size_t)q * fs + j];
        int64_t id = 0;
        if (p >= 0) {
            if (p < n_total)
                id = pos_to_id[p];
            else
                atomicOr(status, 4);
        }
        dists[(size_t)q * w + j] = Fd[(size_t)q * fs + j];
        anns[(size_t)q * w + j] = (uint32_t)id;  // numpy int64 -> uint32 assignment
    }
}

struct ReplayWs {
    size_t counts, goff, groups, Fd, Fp, drd, drp, thr, uraw, total;
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
    s.counts = take((size_t)R * C * 4);
    s.goff = take((size_t)R * (C + 1) * 4);
    s.groups = take((size_t)R * nq * 4);
    s.Fd = take((size_t)nq * fs * 8);
    s.Fp = take((size_t)nq * fs * 4);
    s.drd = take((size_t)nq * kr * 8);
    s.drp = take((size_t)nq * kr * 4);
    s.thr = take((size_t)nq * 8);
    s.uraw = take((size_t)nq * kl * 4);
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

extern "C" int lmi_replay_device(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                                 const float* lists_d, const int32_t* lists_pos, int32_t k_round,
                                 int32_t k_final, const int64_t* bucket_size, int32_t n_buckets,
                                 const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
                                 const double* thr_round0, double* dists_out, uint32_t* anns_out,
                                 int32_t* status, void* workspace, size_t ws_bytes, void* stream) {
    using namespace lmi;
    LMI_CHECK_ARG(nq >= 0 && R >= 1 && k_round >= 1 && k_final >= 1 && k_list >= 1 && n_buckets >= 1,
                  "lmi_replay_device: bad sizes");
    LMI_CHECK_ARG(k_round <= kMaxKr, "lmi_replay_device: k_round=%d > %d", k_round, kMaxKr);
    LMI_CHECK_ARG(k_final <= kMaxW, "lmi_replay_device: k=%d > %d", k_final, kMaxW);
    LMI_CHECK_ARG(k_list >= k_round, "lmi_replay_device: lists of %d < k_round=%d", k_list, k_round);
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
    LMI_CHECK_ARG(classes && lists_d && lists_pos && bucket_size && pos_to_id && dists_out &&
                  anns_out && status && workspace, "lmi_replay_device: null pointer");
    const ReplayWs s = replay_ws(nq, R, k_list, k_round, w, n_buckets);
    if (ws_bytes < s.total) {
        set_error("workspace %zu B < required %zu B", ws_bytes, s.total);
        return LMI_E_WORKSPACE;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    auto* ws = reinterpret_cast<unsigned char*>(workspace);
    const int C = n_buckets;
    const int fs = std::max(k_round, w);
    int32_t* counts = (int32_t*)(ws + s.counts);
    int32_t* goff = (int32_t*)(ws + s.goff);
    int32_t* groups = (int32_t*)(ws + s.groups);
    double* Fd = (double*)(ws + s.Fd);
    int32_t* Fp = (int32_t*)(ws + s.Fp);
    const dim3 qgrid((unsigned)((nq + kT - 1) / kT));
    hipLaunchKernelGGL(replay_count_kernel, dim3(C), dim3(kT), 0, st, classes, nq, R, C, counts);
    LMI_LAUNCH_CHECK("replay_count_kernel");
    hipLaunchKernelGGL(replay_group_fill_kernel, dim3(C), dim3(kT), 0, st, classes, nq, R, C, counts,
                       goff, groups);
    LMI_LAUNCH_CHECK("replay_group_fill_kernel");
    int wF = 0;
    for (int r = 0; r < R; ++r) {
        const bool thresholded = ((r > 0) && use_threshold) || (r == 0 && thr_round0);
        const int mode = (r == 0 && thr_round0) ? 1 : (thresholded ? 2 : 0);
        hipLaunchKernelGGL(replay_thr_kernel, qgrid, dim3(kT), 0, st, nq, k_round, fs, wF, mode, Fd,
                           thr_round0, (double*)(ws + s.thr), (double*)(ws + s.drd),
                           (int32_t*)(ws + s.drp));
        LMI_LAUNCH_CHECK("replay_thr_kernel");
        RoundArgs a{};
        a.classes = classes;
        a.nq = nq;
        a.R = R;
        a.r = r;
        a.kl = k_list;
        a.kr = k_round;
        a.C = C;
        a.lists_d = lists_d;
        a.lists_p = lists_pos;
        a.bucket_size = bucket_size;
        a.groups = groups;
        a.goff = goff;
        a.thresholded = thresholded ? 1 : 0;
        a.thr = (const double*)(ws + s.thr);
        a.dr_d = (double*)(ws + s.drd);
        a.dr_p = (int32_t*)(ws + s.drp);
        a.uraw = (int32_t*)(ws + s.uraw);
        a.status = status;
        hipLaunchKernelGGL(replay_group_kernel, dim3(C), dim3(kT), 0, st, a);
        LMI_LAUNCH_CHECK("replay_group_kernel");
        const int wn = (r == 0) ? k_round : std::min(k_final, wF + k_round);
        hipLaunchKernelGGL(replay_merge_kernel, qgrid, dim3(kT), 0, st, nq, k_round, fs, wF, wn,
                           r == 0 ? 1 : 0, Fd, Fp, (const double*)(ws + s.drd),
                           (const int32_t*)(ws + s.drp));
        LMI_LAUNCH_CHECK("replay_merge_kernel");
        wF = wn;
    }
    hipLaunchKernelGGL(replay_out_kernel, qgrid, dim3(kT), 0, st, nq, w, fs, Fd, Fp, pos_to_id, n_total,
                       dists_out, anns_out, status);
    LMI_LAUNCH_CHECK("replay_out_kernel");
    return LMI_OK;
}
