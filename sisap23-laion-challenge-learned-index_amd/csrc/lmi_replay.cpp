// A5 — host replay of the reference's multi-round bucket merge.
//
// The reference interleaves distance computation with a per-round,
// per-category procedure whose data-dependent quirks decide the answer
// (SURVEY.md §0.3).  Given the exact per-(query, probe) top-k lists from the
// device scan (lmi_bucket_topk), this file replays that procedure exactly:
//
//   LearnedIndex.search        search/li/LearnedIndex.py:22-101
//     threshold = running k-th distance    :71-74  (dists_final.max(axis=1))
//     stable merge of rounds              :82-97  (argsort(kind='stable'))
//   LearnedIndex.search_single  search/li/LearnedIndex.py:103-195
//     groups: groupby('category') ascending, queries np.where ascending :143-147
//     threshold path                      :149-163 -> utils.py:14-43
//     first-k of each row                  :170-172
//     the <k padding quirk                 :174-190 (row 0 only, edge pad,
//                                                     np.unique dedup)
//     broadcast to the whole group         :192-193
//
// Ordering conventions: every sort the reference does on rows of <= 16
// values (numpy <= 1.24 introsort = insertion sort there) is stable, and the
// scan's lists are ordered by (distance, position) — identical on tie-free
// inputs.  The order of the 10000-valued fillers of a normal threshold row
// (utils.py:35-42, `U \ B_q`) is unspecified in the reference (introsort
// over ties); here they are taken in ascending position.  They can reach the
// output only when k_final > k_round.
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/lmi_hip.h"

namespace lmi {
void set_error(const char* fmt, ...);
}

namespace {

constexpr double kFill = 10000.0;  // LearnedIndex.py:138, utils.py:35

struct Entry {
    double d;
    int64_t pos;  // -1 = no object (id 0)
};

// numpy: np.pad(a, p, 'edge')[:k]
template <typename T>
void edge_pad_take(const std::vector<T>& a, int p, int k, std::vector<T>& out) {
    out.clear();
    const int n = (int)a.size();
    for (int j = 0; j < k; ++j) {
        const int src = j - p;  // index into a, clamped to the edges
        out.push_back(a[std::min(std::max(src, 0), n - 1)]);
    }
}

// stable argsort of a short row
void stable_argsort(const std::vector<double>& row, std::vector<int>& idx) {
    idx.resize(row.size());
    for (size_t i = 0; i < row.size(); ++i) idx[i] = (int)i;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return row[a] < row[b]; });
}

// LearnedIndex.py:174-193: the quirk for a group whose candidate set U has
// fewer than k_round members.  `row` is row 0 (query q0) in U order, `u_pos`
// the positions of U, `ann` the (stable) argsort of the row.
void quirk_row(const std::vector<double>& row, const std::vector<int64_t>& u_pos,
               const std::vector<int>& ann, int kr, std::vector<Entry>& out) {
    const int n = (int)u_pos.size();
    const int p = (kr - n) / 2 + 1;
    std::vector<int64_t> ids_p;
    std::vector<int> ann_p;
    std::vector<double> row_p;
    edge_pad_take(u_pos, p, kr, ids_p);
    edge_pad_take(ann, p, kr, ann_p);
    edge_pad_take(row, p, kr, row_p);
    // _, i = np.unique(seq, return_index=True); seq[0][setdiff(arange(k), i)] = 10000:
    // every value that is not the first occurrence of itself (decided on the
    // values before any rewrite) becomes 10000.
    const std::vector<double> orig = row_p;
    for (int j = 0; j < kr; ++j) {
        for (int i = 0; i < j; ++i) {
            if (orig[i] == orig[j]) {
                row_p[j] = kFill;
                break;
            }
        }
    }
    out.resize(kr);
    for (int j = 0; j < kr; ++j) {
        out[j].pos = ids_p[ann_p[j]];
        out[j].d = row_p[ann_p[j]];
    }
}

}  // namespace

namespace {
int replay_impl(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list, const void* lists_dv,
                bool lists_f64, const int32_t* lists_pos, int32_t k_round, int32_t k_final,
                const int64_t* bucket_size, int32_t n_buckets, const int64_t* pos_to_id,
                int64_t n_total, int32_t use_threshold, const double* thr_round0,
                double* dists_out, uint32_t* anns_out, int32_t* w_out);
}  // namespace

extern "C" int lmi_replay(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                          const float* lists_d, const int32_t* lists_pos, int32_t k_round,
                          int32_t k_final, const int64_t* bucket_size, int32_t n_buckets,
                          const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
                          const double* thr_round0, double* dists_out, uint32_t* anns_out,
                          int32_t* w_out) {
    return replay_impl(classes, nq, R, k_list, lists_d, false, lists_pos, k_round, k_final,
                       bucket_size, n_buckets, pos_to_id, n_total, use_threshold, thr_round0,
                       dists_out, anns_out, w_out);
}

extern "C" int lmi_replay_f64(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list,
                              const double* lists_d, const int32_t* lists_pos, int32_t k_round,
                              int32_t k_final, const int64_t* bucket_size, int32_t n_buckets,
                              const int64_t* pos_to_id, int64_t n_total, int32_t use_threshold,
                              const double* thr_round0, double* dists_out, uint32_t* anns_out,
                              int32_t* w_out) {
    return replay_impl(classes, nq, R, k_list, lists_d, true, lists_pos, k_round, k_final,
                       bucket_size, n_buckets, pos_to_id, n_total, use_threshold, thr_round0,
                       dists_out, anns_out, w_out);
}

namespace {
int replay_impl(const int32_t* classes, int32_t nq, int32_t R, int32_t k_list, const void* lists_dv,
                bool lists_f64, const int32_t* lists_pos, int32_t k_round, int32_t k_final,
                const int64_t* bucket_size, int32_t n_buckets, const int64_t* pos_to_id,
                int64_t n_total, int32_t use_threshold, const double* thr_round0,
                double* dists_out, uint32_t* anns_out, int32_t* w_out) {
    using lmi::set_error;
    const void* lists_d = lists_dv;
    if (nq < 0 || R < 1 || k_round < 1 || k_final < 1 || k_list < 1 || n_buckets < 1) {
        set_error("lmi_replay: bad sizes");
        return LMI_E_INVALID;
    }
    if (nq > 0 && (!classes || !lists_d || !lists_pos || !bucket_size || !pos_to_id ||
                   !dists_out || !anns_out)) {
        set_error("lmi_replay: null pointer");
        return LMI_E_INVALID;
    }
    const int kr = k_round;
    // widths of the merged result: w0 = kr, w_r = min(k_final, w_{r-1} + kr);
    // the reference asserts w_r == k_final at every merge (LearnedIndex.py:99)
    int w = kr;
    for (int r = 1; r < R; ++r) {
        w = std::min(k_final, w + kr);
        if (w != k_final) {
            set_error("lmi_replay: k=%d exceeds the merged width %d (reference assert, LearnedIndex.py:99)",
                      k_final, w);
            return LMI_E_INVALID;
        }
    }
    if (w_out) *w_out = w;
    if (nq == 0) return LMI_OK;

    // The scan's lists must hold what one round can show: min(k_round, n_c).
    const int kl_use = std::min(kr, k_list);
    if (k_list < kr) {
        for (int c = 0; c < n_buckets; ++c) {
            if (bucket_size[c] > k_list) {
                set_error("lmi_replay: lists of %d entries cannot replay k_round=%d", k_list, kr);
                return LMI_E_INVALID;
            }
        }
    }

    // F holds round 0 (k_round wide) and every merge (k_final wide)
    const int fs = std::max(kr, w);
    std::vector<Entry> F((size_t)nq * fs), Dr((size_t)nq * kr);
    int wF = 0;
    std::vector<int> order(nq), start(n_buckets + 1);
    std::vector<double> thr(nq);
    // Rounds are sequential; inside a round, queries (threshold, merge,
    // output) and bucket groups (each writes only its own queries' D_r rows)
    // are independent and split over OpenMP threads.  Results do not depend
    // on the thread count.
    std::atomic<int> err{0};
    std::vector<int> fillp(n_buckets);

    for (int r = 0; r < R; ++r) {
        const bool thresholded = ((r > 0) && use_threshold) || (r == 0 && thr_round0);
#pragma omp parallel for schedule(static)
        for (int q = 0; q < nq; ++q) {
            for (int j = 0; j < kr; ++j) Dr[(size_t)q * kr + j] = Entry{kFill, -1};
            if (r == 0 && thr_round0) {
                thr[q] = thr_round0[q];
            } else if (thresholded) {
                double m = F[(size_t)q * fs].d;
                for (int j = 1; j < wF; ++j) m = std::max(m, F[(size_t)q * fs + j].d);
                thr[q] = m;
            }
        }
        // groups: queries with classes[q, r] == c, ascending q (counting sort)
        std::fill(start.begin(), start.end(), 0);
        for (int q = 0; q < nq; ++q) {
            const int c = classes[(size_t)q * R + r];
            if (c >= 0 && c < n_buckets) ++start[c + 1];
        }
        for (int c = 0; c < n_buckets; ++c) start[c + 1] += start[c];
        std::copy(start.begin(), start.end() - 1, fillp.begin());
        for (int q = 0; q < nq; ++q) {
            const int c = classes[(size_t)q * R + r];
            if (c >= 0 && c < n_buckets) order[fillp[c]++] = q;
        }
        auto list_at = [&](int q, int j, double& d, int64_t& pos) {
            const size_t o = ((size_t)q * R + r) * k_list + j;
            pos = lists_pos[o];
            d = lists_f64 ? static_cast<const double*>(lists_dv)[o]
                          : (double)static_cast<const float*>(lists_dv)[o];
        };
#pragma omp parallel for schedule(dynamic, 1)
        for (int c = 0; c < n_buckets; ++c) {
            std::vector<Entry> tmp;
            const int g0 = start[c], g1 = start[c + 1];
            if (g0 == g1 || bucket_size[c] <= 0) continue;  // groupby visits non-empty categories only
            if (thresholded) {
                // utils.py:22-32: relevant = d < thr[q] (strict); U = unique columns
                std::vector<int64_t> U;
                for (int gi = g0; gi < g1; ++gi) {
                    const int q = order[gi];
                    for (int j = 0; j < kl_use; ++j) {
                        double d;
                        int64_t pos;
                        list_at(q, j, d, pos);
                        if (pos < 0 || !(d < thr[q])) break;  // list is ascending
                        U.push_back(pos);
                    }
                }
                std::sort(U.begin(), U.end());
                U.erase(std::unique(U.begin(), U.end()), U.end());
                if (U.empty()) continue;  // LearnedIndex.py:157-159
                if ((int)U.size() >= kr) {
                    for (int gi = g0; gi < g1; ++gi) {
                        const int q = order[gi];
                        Entry* out = &Dr[(size_t)q * kr];
                        int n = 0;
                        for (int j = 0; j < kl_use && n < kr; ++j) {
                            double d;
                            int64_t pos;
                            list_at(q, j, d, pos);
                            if (pos < 0 || !(d < thr[q])) break;
                            out[n++] = Entry{d, pos};
                        }
                        // fillers: objects of U not relevant to q, distance 10000
                        // (the first n entries of `out` are q's relevant ones)
                        const int n_rel = n;
                        for (size_t u = 0; u < U.size() && n < kr; ++u) {
                            bool mine = false;
                            for (int j = 0; j < n_rel; ++j) mine |= (out[j].pos == U[u]);
                            if (!mine) out[n++] = Entry{kFill, U[u]};
                        }
                    }
                } else {
                    const int q0 = order[g0];
                    std::vector<double> row(kr, kFill);
                    for (int j = 0; j < kl_use; ++j) {
                        double d;
                        int64_t pos;
                        list_at(q0, j, d, pos);
                        if (pos < 0 || !(d < thr[q0])) break;
                        const size_t at = std::lower_bound(U.begin(), U.end(), pos) - U.begin();
                        row[at] = d;
                    }
                    std::vector<int> ann;
                    stable_argsort(row, ann);  // length kr = the row's full length
                    quirk_row(row, U, ann, kr, tmp);
                    for (int gi = g0; gi < g1; ++gi)
                        std::copy(tmp.begin(), tmp.end(), &Dr[(size_t)order[gi] * kr]);
                }
            } else {
                const int64_t n = bucket_size[c];
                if (n >= kr) {
                    for (int gi = g0; gi < g1; ++gi) {
                        const int q = order[gi];
                        for (int j = 0; j < kr; ++j) {
                            double d;
                            int64_t pos;
                            list_at(q, j, d, pos);
                            Dr[(size_t)q * kr + j] = Entry{d, pos};
                        }
                    }
                } else {
                    // row 0 = q0's distances to the whole bucket in position order
                    const int q0 = order[g0];
                    std::vector<std::pair<int64_t, double>> objs;
                    for (int j = 0; j < kl_use && j < (int)n; ++j) {
                        double d;
                        int64_t pos;
                        list_at(q0, j, d, pos);
                        if (pos < 0) break;
                        objs.emplace_back(pos, d);
                    }
                    if ((int64_t)objs.size() != n) {
                        err.store(c + 1);  // reported after the loop
                        continue;
                    }
                    std::sort(objs.begin(), objs.end());
                    std::vector<double> row;
                    std::vector<int64_t> u_pos;
                    for (auto& o : objs) {
                        u_pos.push_back(o.first);
                        row.push_back(o.second);
                    }
                    std::vector<int> ann;
                    stable_argsort(row, ann);  // [:min(k, n)] = all n
                    quirk_row(row, u_pos, ann, kr, tmp);
                    for (int gi = g0; gi < g1; ++gi)
                        std::copy(tmp.begin(), tmp.end(), &Dr[(size_t)order[gi] * kr]);
                }
            }
        }
        // merge (LearnedIndex.py:82-97)
        if (r == 0) {
            for (int q = 0; q < nq; ++q)
                for (int j = 0; j < kr; ++j) F[(size_t)q * fs + j] = Dr[(size_t)q * kr + j];
            wF = kr;
        } else {
            const int wn = std::min(k_final, wF + kr);
#pragma omp parallel
            {
                std::vector<Entry> cat(wF + kr);
#pragma omp for schedule(static)
                for (int q = 0; q < nq; ++q) {
                    // stable sort of hstack(F, D_r) by distance (argsort(kind='stable')):
                    // insertion sort, strict > so equal distances keep hstack order.
                    // (F need not be sorted: quirk rows of round 0 are not.)
                    int len = 0;
                    for (int j = 0; j < wF + kr; ++j) {
                        const Entry e = j < wF ? F[(size_t)q * fs + j] : Dr[(size_t)q * kr + (j - wF)];
                        int i = len++;
                        while (i > 0 && cat[i - 1].d > e.d) {
                            cat[i] = cat[i - 1];
                            --i;
                        }
                        cat[i] = e;
                    }
                    for (int j = 0; j < wn; ++j) F[(size_t)q * fs + j] = cat[j];
                }
            }
            wF = wn;
        }
        if (err.load()) {
            const int c = err.load() - 1;
            set_error("lmi_replay: the list of bucket %d does not hold all its %lld objects", c,
                      (long long)bucket_size[c]);
            return LMI_E_INVALID;
        }
    }
    std::atomic<int64_t> bad{-1};
#pragma omp parallel for schedule(static)
    for (int q = 0; q < nq; ++q) {
        for (int j = 0; j < w; ++j) {
            const Entry& e = F[(size_t)q * fs + j];
            dists_out[(size_t)q * w + j] = e.d;
            int64_t id = 0;
            if (e.pos >= 0) {
                if (e.pos >= n_total) {
                    bad.store(e.pos);
                    continue;
                }
                id = pos_to_id[e.pos];
            }
            anns_out[(size_t)q * w + j] = (uint32_t)id;  // numpy int64 -> uint32 assignment
        }
    }
    if (bad.load() >= 0) {
        set_error("lmi_replay: position %lld out of range", (long long)bad.load());
        return LMI_E_INVALID;
    }
    return LMI_OK;
}
}  // namespace
