// artificial_matrix.cpp -- synthetic CSR generator (the reference's artificial-matrix-generator submodule is empty
// in the reference tree, .gitmodules:5-8; this is a from-scratch design against its 11-parameter contract,
// spmv_bench.cpp:842-869, and the feature definitions that measure it, csr_util_gen.c:269-610,964-983).
//
// Model, per row i (degree d_i):
//   * d_i ~ |N(avg, std)| ("normal", lib/random.h random_normal: Box-Muller) or Gamma(k=(avg/std)^2,
//     theta=std^2/avg) ("gamma", Marsaglia-Tsang), rounded, capped at nr_cols.
//   * crs >= 0.8 with std/avg >= 0.5: degrees sorted ascending inside aligned 64-row windows (see row_degrees).
//   * skew > 0: one row (seeded choice) gets degree avg*(1+skew) (capped at nr_cols); the other rows are scaled so
//     that the total stays avg*nr_rows and clamped at that degree -- the feature skew = (max - avg)/avg then equals
//     the parameter even when it lies below the natural tail of the degree distribution.
//   * neighbours: the row is laid out as R = d*(1 - nu/2) runs of consecutive columns separated by >= 1 free column;
//     a run of length L contributes 2(L-1) to the row-neighbour count, so the mean over the row's nonzeros is nu.
//   * columns live in a window of width W_i = bw*nr_cols*(R_t+1)/(R_t-1) centred on the diagonal, R_t = the row's
//     runs (copied + new, each placed independently): the expected span of R_t uniform points in the window is then
//     bw*nr_cols.  A row keeps >= 2 runs when the requested span is wider than the row (else one run spans nothing).
//     "random" placement = uniform positions inside the window, "diagonal" = positions from its central half.
//   * cross-row similarity: row i copies runs of row i-1 until crs*d_{i-1} of row i-1's columns have a column
//     within +-1 in row i (the feature's definition, csr_util_gen.c:553-610); a run is copied whole while that
//     stays within the target, else its first L' columns (they match L'+1 of row i-1's columns).  New runs avoid
//     +-1 contact with row i-1 where they can (a few random retries), so accidental matches do not inflate it.
//   * values: seeded uniform [0.5, 1.5) (positive, cancellation-free, so 1e-10 checks are meaningful).
// Determinism: every random stream is keyed by (seed, row, purpose); the copy chain restarts every SEG rows so
// segments can be generated independently (any thread count, any row range) with identical output.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/spmm_host.h"

namespace {

constexpr int64_t SEG = 4096;  // copy-chain restart period (rows)

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

struct Rng {  // xoshiro256**
    uint64_t s[4];
    Rng(uint64_t seed, uint64_t a, uint64_t b) {
        uint64_t x = splitmix64(seed ^ splitmix64(a * 0x100000001B3ULL + b));
        for (auto &v : s) v = x = splitmix64(x);
    }
    static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    double uniform() { return (next() >> 11) * 0x1.0p-53; }  // [0,1)
    int64_t below(int64_t n) { return n <= 1 ? 0 : (int64_t)(uniform() * (double)n); }
    double normal() {  // Box-Muller
        double u1 = uniform(), u2 = uniform();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
    }
    double gamma(double k) {  // Marsaglia-Tsang, k > 0
        if (k < 1.0) return gamma(k + 1.0) * std::pow(uniform() + 1e-300, 1.0 / k);
        const double d = k - 1.0 / 3.0, c = 1.0 / std::sqrt(9.0 * d);
        for (;;) {
            double x, v;
            do {
                x = normal();
                v = 1.0 + c * x;
            } while (v <= 0);
            v = v * v * v;
            const double u = uniform();
            if (u < 1.0 - 0.0331 * x * x * x * x) return d * v;
            if (std::log(u) < 0.5 * x * x + d * (1.0 - v + std::log(v))) return d * v;
        }
    }
};

enum Stream : uint64_t { S_DEG = 1, S_SKEW = 2, S_COLS = 3, S_VALS = 4 };

bool valid(const spmm_gen_params_t *p) {
    return p && p->nr_rows > 0 && p->nr_cols > 0 && p->avg_nnz_per_row >= 0 && p->std_nnz_per_row >= 0 &&
           p->bw >= 0 && p->skew >= 0 && p->avg_num_neighbours >= 0 && p->cross_row_similarity >= 0;
}

// Twin-style lines (high cross-row similarity, widely varying degrees): degrees sorted in windows, and a short row
// after a much longer one copies the long row's runs nearest its own diagonal first (see row_degrees, RowGen::gen).
bool smooth_degrees(const spmm_gen_params_t *p) {
    return p->cross_row_similarity >= 0.8 && p->avg_nnz_per_row > 0 &&
           p->std_nnz_per_row / p->avg_nnz_per_row >= 0.5;
}

// Row degrees of the whole matrix (deterministic, thread-count independent).
int row_degrees(const spmm_gen_params_t *p, std::vector<int64_t> &deg) {
    const int64_t m = p->nr_rows, n = p->nr_cols;
    const double avg = p->avg_nnz_per_row, sd = p->std_nnz_per_row;
    const bool gam = (strcmp(p->distribution, "gamma") == 0);
    std::vector<double> raw(m);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < m; ++i) {
        Rng r((uint64_t)p->seed, (uint64_t)i, S_DEG);
        double x;
        if (gam && avg > 0 && sd > 0) {
            const double k = (avg / sd) * (avg / sd), theta = sd * sd / avg;
            x = r.gamma(k) * theta;
        } else {
            x = std::fabs(avg + sd * r.normal());
        }
        raw[i] = x;
    }
    deg.assign(m, 0);
    int64_t giant = -1, giant_deg = 0;
    double scale = 1.0;
    if (p->skew > 0 && m > 1) {
        Rng r((uint64_t)p->seed, 0, S_SKEW);
        giant = r.below(m);
        giant_deg = std::min<int64_t>(n, (int64_t)std::llround(avg * (1.0 + p->skew)));
        double rest = 0;
#pragma omp parallel for reduction(+ : rest)
        for (int64_t i = 0; i < m; ++i)
            if (i != giant) rest += raw[i];
        const double want = std::max(0.0, avg * (double)m - (double)giant_deg);
        scale = rest > 0 ? want / rest : 0.0;
        // the clamp at giant_deg removes mass from the tail: re-solve the scale (bisection, deterministic) so the
        // clamped rows still sum to the wanted total
        auto clamped_sum = [&](double sc) {
            double t = 0;
#pragma omp parallel for reduction(+ : t)
            for (int64_t i = 0; i < m; ++i)
                if (i != giant) t += (double)std::min<int64_t>((int64_t)std::llround(raw[i] * sc), giant_deg);
            return t;
        };
        if (scale > 0 && clamped_sum(scale) < 0.999 * want) {
            double lo = scale, hi = scale;
            for (int it = 0; it < 8 && clamped_sum(hi) < want; ++it) hi *= 2.0;
            for (int it = 0; it < 24; ++it) {
                const double mid = 0.5 * (lo + hi);
                (clamped_sum(mid) < want ? lo : hi) = mid;
            }
            scale = hi;
        }
    }
    int64_t total = 0;
#pragma omp parallel for reduction(+ : total)
    for (int64_t i = 0; i < m; ++i) {
        int64_t d = (i == giant) ? giant_deg : (int64_t)std::llround(raw[i] * scale);
        if (giant >= 0) d = std::min(d, giant_deg);   // the heavy row IS the maximum (small skews: below the tail)
        d = std::max<int64_t>(0, std::min<int64_t>(d, n));
        deg[i] = d;
        total += d;
    }
    if (total >= INT32_MAX) return SPMM_HOST_ERR_OVERFLOW;
    // High cross-row similarity with widely varying degrees (the validation twins of real matrices): the feature
    // counts row i's columns matched in row i+1, so a long row followed by a short one cannot reach it with
    // independently drawn degrees (measured shortfall up to 0.27).  Real matrices vary their row lengths smoothly;
    // sorting the degrees ascending inside aligned windows of DEG_WIN rows keeps the degree multiset (avg, std,
    // skew unchanged) and makes row i+1 at least as long as row i except at window boundaries.  Off for the
    // synthetic datasets' own lines (std/avg = 1/3).
    if (smooth_degrees(p)) {
        constexpr int64_t DEG_WIN = 64;   // divides SEG: row-range generation stays identical
#pragma omp parallel for schedule(static)
        for (int64_t w0 = 0; w0 < m; w0 += DEG_WIN)
            std::sort(deg.begin() + w0, deg.begin() + std::min(m, w0 + DEG_WIN));
    }
    return SPMM_HOST_OK;
}

struct RowGen {
    const spmm_gen_params_t *p;
    double bw_scale = 1.0;   // 1 / fraction of rows with >= 2 nonzeros (1-nonzero rows span nothing)
    std::vector<int32_t> prev, cur, tmp;
    std::vector<std::pair<int32_t, int32_t>> runs_prev, runs_cur;  // (start, length)

    // window [lo, lo+W) for row i with degree d laid out as rt independently placed runs
    void window(int64_t i, int64_t d, int64_t rt, int64_t &lo, int64_t &W) const {
        const int64_t n = p->nr_cols, m = p->nr_rows;
        double w = p->bw * bw_scale * (double)n;
        if (rt >= 2) w *= (double)(rt + 1) / (double)(rt - 1);
        W = std::max<int64_t>(std::llround(w), std::max<int64_t>(1, d));
        // room for the runs and their separating gaps
        W = std::min<int64_t>(n, std::max<int64_t>(W, 2 * d));
        const double center = ((double)i + 0.5) * (double)n / (double)m;
        lo = (int64_t)std::llround(center - 0.5 * (double)W);
        lo = std::max<int64_t>(0, std::min<int64_t>(lo, n - W));
        if (strcmp(p->placement, "diagonal") == 0 && W >= 4 * std::max<int64_t>(d, 1)) {
            lo += W / 4;
            W /= 2;
        }
    }

    static bool taken(const std::vector<int32_t> &sorted, int64_t c) {
        return std::binary_search(sorted.begin(), sorted.end(), (int32_t)c);
    }

    // Generate row i (degree d) given the previous row of the chain (prev/runs_prev, possibly empty).
    void gen(int64_t i, int64_t d) {
        cur.clear();
        runs_cur.clear();
        if (d == 0) return;
        const int64_t n = p->nr_cols;
        Rng r((uint64_t)p->seed, (uint64_t)i, S_COLS);
        const double nu = std::min(2.0, p->avg_num_neighbours);

        // 1. copy runs of the previous row: matched = row i-1 columns that get a column within +-1 in row i
        int64_t copied_runs = 0;
        if (!runs_prev.empty() && p->cross_row_similarity > 0) {
            const int64_t target = std::llround(p->cross_row_similarity * (double)prev.size());
            std::vector<int> order(runs_prev.size());
            for (size_t q = 0; q < order.size(); ++q) order[q] = (int)q;
            for (size_t q = order.size(); q > 1; --q) std::swap(order[q - 1], order[r.below((int64_t)q)]);
            if (smooth_degrees(p) && (int64_t)prev.size() > 2 * d) {
                // runs nearest this row's diagonal first: a short row following a long one keeps its span
                const double center = ((double)i + 0.5) * (double)n / (double)p->nr_rows;
                std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
                    return std::fabs(runs_prev[a].first - center) < std::fabs(runs_prev[b].first - center);
                });
            }
            int64_t matched = 0;
            for (int q : order) {
                const int64_t need = target - matched, room = d - (int64_t)cur.size();
                if (need <= 0 || room <= 0) break;
                const auto run = runs_prev[q];
                int64_t len = run.second;
                if (len > need) len = std::max<int64_t>(1, need - 1);   // first len columns match len + 1
                len = std::min(len, room);
                for (int64_t t = 0; t < len; ++t) cur.push_back(run.first + (int32_t)t);
                matched += (len < run.second) ? len + 1 : len;
                ++copied_runs;
            }
        }
        std::sort(cur.begin(), cur.end());

        // 2. the rest of the row.  The row should hold R_t runs: d*(1 - nu/2) for the neighbour count, and at least
        // (1+bw)/(1-bw) when the requested span is wider than the row (R_t uniform runs span (R_t-1)/(R_t+1) of a
        // window that cannot exceed n).  Copied runs count; if they already are R_t, the new columns grow them at
        // their ends, otherwise R_t - copied new runs are placed in the row's own window.
        int64_t rest = d - (int64_t)cur.size();
        int64_t Rt = std::max<int64_t>(1, std::llround((double)d * (1.0 - nu / 2.0)));
        if (p->bw * bw_scale * (double)n >= 2.0 * (double)d) {
            const double bwf = std::min(0.95, p->bw * bw_scale);
            Rt = std::max<int64_t>(Rt, (int64_t)std::ceil((1.0 + bwf) / (1.0 - bwf) - 1e-9));
        }
        Rt = std::min<int64_t>(Rt, d);
        if (rest > 0 && copied_runs >= Rt) {
            std::vector<std::pair<int32_t, int32_t>> cr;   // copied runs as they stand in cur
            for (size_t q = 0; q < cur.size();) {
                size_t t = q + 1;
                while (t < cur.size() && cur[t] == cur[t - 1] + 1) ++t;
                cr.push_back({cur[q], (int32_t)(t - q)});
                q = t;
            }
            for (int64_t tries = 0; rest > 0 && tries < 4 * d + 16; ++tries) {
                auto &run = cr[r.below((int64_t)cr.size())];
                const int64_t c = run.first + run.second;            // grow the run at its end
                if (c < n && !taken(cur, c) && !taken(cur, c + 1)) {
                    cur.insert(std::upper_bound(cur.begin(), cur.end(), (int32_t)c), (int32_t)c);
                    ++run.second;
                    --rest;
                }
            }
        }
        if (rest > 0) {
            const int64_t R = std::min<int64_t>(rest, std::max<int64_t>(1, Rt - copied_runs));
            int64_t lo, W;
            window(i, d, R + copied_runs, lo, W);
            // run lengths: all 1, then the remaining units dealt at random
            std::vector<int64_t> L(R, 1);
            for (int64_t u = R; u < rest; ++u) L[r.below(R)]++;
            const int64_t free_cells = W - rest - (R - 1);
            std::vector<int64_t> g(R);
            if (free_cells >= 0) {
                for (auto &x : g) x = r.below(free_cells + 1);
                std::sort(g.begin(), g.end());
            }
            int64_t off = 0;
            tmp.clear();
            for (int64_t q = 0; q < R; ++q) {
                int64_t start = (free_cells >= 0) ? lo + g[q] + off + q : lo + r.below(std::max<int64_t>(1, W - L[q]));
                off += L[q];
                // keep the run clear of copied columns (exact hits or adjacency) and of +-1 contact with the
                // previous row (accidental similarity); retry a few random starts
                for (int tries = 0; tries < 8; ++tries) {
                    bool clash = false;
                    for (int64_t t = -1; t <= L[q] && !clash; ++t) clash = taken(cur, start + t) || taken(prev, start + t);
                    if (!clash) break;
                    start = lo + r.below(std::max<int64_t>(1, W - L[q]));
                }
                for (int64_t t = 0; t < L[q]; ++t) {
                    const int64_t c = start + t;
                    if (c >= 0 && c < n) tmp.push_back((int32_t)c);
                }
                runs_cur.push_back({(int32_t)start, (int32_t)L[q]});
            }
            cur.insert(cur.end(), tmp.begin(), tmp.end());
            std::sort(cur.begin(), cur.end());
            cur.erase(std::unique(cur.begin(), cur.end()), cur.end());
            // 3. top up after collisions: random free columns, window first, then the whole row
            if (d - (int64_t)cur.size() > 4096) {
                // many missing columns (a huge or dense row): a bitmap of the row instead of sorted inserts
                // (quadratic); random free columns while the window is sparse, then free columns in window order
                // from a random offset, then the rest of the row
                std::vector<uint8_t> bm((size_t)n, 0);
                for (int32_t c : cur) bm[(size_t)c] = 1;
                int64_t have = (int64_t)cur.size();
                for (int64_t guard = 0; have < d && guard < 8 * d; ++guard) {
                    const int64_t c = lo + r.below(W);
                    if (!bm[(size_t)c]) bm[(size_t)c] = 1, ++have;
                }
                const int64_t off = r.below(std::max<int64_t>(1, W));
                for (int64_t t = 0; t < W && have < d; ++t) {
                    const int64_t c = lo + (off + t) % W;
                    if (!bm[(size_t)c]) bm[(size_t)c] = 1, ++have;
                }
                for (int64_t c = 0; c < n && have < d; ++c)
                    if (!bm[(size_t)c]) bm[(size_t)c] = 1, ++have;
                cur.clear();
                for (int64_t c = 0; c < n; ++c)
                    if (bm[(size_t)c]) cur.push_back((int32_t)c);
            }
            int64_t guard = 0;
            while ((int64_t)cur.size() < d) {
                const bool wide = guard++ > 64 * d;
                const int64_t c = wide ? r.below(n) : lo + r.below(W);
                if (!taken(cur, c)) cur.insert(std::upper_bound(cur.begin(), cur.end(), (int32_t)c), (int32_t)c);
                if (guard > 4096 * d + 1000000) {  // dense row: take the first free columns
                    for (int64_t c2 = 0; c2 < n && (int64_t)cur.size() < d; ++c2)
                        if (!taken(cur, c2)) cur.insert(std::upper_bound(cur.begin(), cur.end(), (int32_t)c2), (int32_t)c2);
                }
            }
        } else if ((int64_t)cur.size() > d) {
            cur.resize(d);
        }
        // rebuild the run list from the final sorted columns (what the next row copies)
        runs_cur.clear();
        for (size_t q = 0; q < cur.size();) {
            size_t t = q + 1;
            while (t < cur.size() && cur[t] == cur[t - 1] + 1) ++t;
            runs_cur.push_back({cur[q], (int32_t)(t - q)});
            q = t;
        }
    }
};

int alloc_csr(spmm_csr_t *out, int64_t m, int64_t ncols, int64_t nnz) {
    out->m = m;
    out->ncols = ncols;
    out->nnz = nnz;
    out->row_ptr = (int32_t *)malloc((size_t)(m + 1) * sizeof(int32_t));
    out->col_idx = (int32_t *)malloc((size_t)std::max<int64_t>(nnz, 1) * sizeof(int32_t));
    out->values = (double *)malloc((size_t)std::max<int64_t>(nnz, 1) * sizeof(double));
    if (!out->row_ptr || !out->col_idx || !out->values) {
        spmm_host_csr_free(out);
        return SPMM_HOST_ERR_NOMEM;
    }
    return SPMM_HOST_OK;
}

// Fill rows [r0, r1) (row_ptr already holds the rebased offsets of that range).
void fill_rows(const spmm_gen_params_t *p, const std::vector<int64_t> &deg, int64_t r0, int64_t r1,
               spmm_csr_t *out) {
    const int64_t seg0 = r0 / SEG, seg1 = (r1 + SEG - 1) / SEG;
    int64_t multi = 0;   // rows with >= 2 nonzeros, over the WHOLE matrix (same for every row range)
    for (int64_t d : deg) multi += (d >= 2);
    const double bw_scale = 1.0 / std::max(0.05, (double)multi / (double)std::max<size_t>(deg.size(), 1));
#pragma omp parallel
    {
        RowGen g;
        g.p = p;
        g.bw_scale = bw_scale;
#pragma omp for schedule(dynamic, 1)
        for (int64_t s = seg0; s < seg1; ++s) {
            g.prev.clear();
            g.runs_prev.clear();
            const int64_t a = s * SEG, b = std::min<int64_t>((s + 1) * SEG, p->nr_rows);
            for (int64_t i = a; i < b; ++i) {
                g.gen(i, deg[i]);
                if (i >= r0 && i < r1) {
                    const int64_t base = out->row_ptr[i - r0];
                    Rng rv((uint64_t)p->seed, (uint64_t)i, S_VALS);
                    for (size_t t = 0; t < g.cur.size(); ++t) {
                        out->col_idx[base + t] = g.cur[t];
                        out->values[base + t] = 0.5 + rv.uniform();
                    }
                }
                if (!g.cur.empty()) {  // the chain links non-empty rows (csr_util_gen.c:570-572)
                    std::swap(g.prev, g.cur);
                    std::swap(g.runs_prev, g.runs_cur);
                }
            }
        }
    }
}

}  // namespace

extern "C" {

int spmm_host_parse_gen_line(const char *line, spmm_gen_params_t *p) {
    if (!line || !p) return SPMM_HOST_ERR_ARG;
    memset(p, 0, sizeof(*p));
    long long rows, cols, seed;
    char dist[16], place[16];
    int n = sscanf(line, "%lld %lld %lf %lf %15s %15s %lf %lf %lf %lf %lld", &rows, &cols, &p->avg_nnz_per_row,
                   &p->std_nnz_per_row, dist, place, &p->bw, &p->skew, &p->avg_num_neighbours,
                   &p->cross_row_similarity, &seed);
    if (n != 11) return SPMM_HOST_ERR_PARSE;
    p->nr_rows = rows;
    p->nr_cols = cols;
    p->seed = seed;
    snprintf(p->distribution, sizeof(p->distribution), "%s", dist);
    snprintf(p->placement, sizeof(p->placement), "%s", place);
    return SPMM_HOST_OK;
}

int spmm_host_generate_row_ptr(const spmm_gen_params_t *p, int32_t *row_ptr) {
    if (!valid(p) || !row_ptr) return SPMM_HOST_ERR_ARG;
    std::vector<int64_t> deg;
    int st = row_degrees(p, deg);
    if (st) return st;
    row_ptr[0] = 0;
    for (int64_t i = 0; i < p->nr_rows; ++i) row_ptr[i + 1] = (int32_t)(row_ptr[i] + deg[i]);
    return SPMM_HOST_OK;
}

int spmm_host_generate_rows(const spmm_gen_params_t *p, int64_t r0, int64_t r1, spmm_csr_t *out) {
    if (!valid(p) || !out || r0 < 0 || r1 < r0 || r1 > p->nr_rows) return SPMM_HOST_ERR_ARG;
    memset(out, 0, sizeof(*out));
    std::vector<int64_t> deg;
    int st = row_degrees(p, deg);
    if (st) return st;
    int64_t nnz = 0;
    for (int64_t i = r0; i < r1; ++i) nnz += deg[i];
    st = alloc_csr(out, r1 - r0, p->nr_cols, nnz);
    if (st) return st;
    out->row_ptr[0] = 0;
    for (int64_t i = r0; i < r1; ++i) out->row_ptr[i - r0 + 1] = (int32_t)(out->row_ptr[i - r0] + deg[i]);
    fill_rows(p, deg, r0, r1, out);
    return SPMM_HOST_OK;
}

// The whole matrix's row_ptr with the columns (and values) of the rows where mask[i] != 0 only -- the other rows'
// entries are left zero (column 0).  Only the 4096-row copy-chain segments that hold a masked row are generated, up
// to their last masked row, so a row sample of a large matrix costs a fraction of the full generation
// (tools/plan_census.py: the matrix-core gate reads its sampled 16-row tiles only).  The masked rows are identical to
// the same rows of spmm_host_generate.
int spmm_host_generate_masked(const spmm_gen_params_t *p, const uint8_t *mask, spmm_csr_t *out) {
    if (!valid(p) || !out || !mask) return SPMM_HOST_ERR_ARG;
    memset(out, 0, sizeof(*out));
    std::vector<int64_t> deg;
    int st = row_degrees(p, deg);
    if (st) return st;
    const int64_t m = p->nr_rows;
    int64_t nnz = 0;
    for (int64_t i = 0; i < m; ++i) nnz += deg[i];
    out->m = m;
    out->ncols = p->nr_cols;
    out->nnz = nnz;
    out->row_ptr = (int32_t *)malloc((size_t)(m + 1) * sizeof(int32_t));
    out->col_idx = (int32_t *)calloc((size_t)std::max<int64_t>(nnz, 1), sizeof(int32_t));   // untouched pages stay
    out->values = (double *)calloc((size_t)std::max<int64_t>(nnz, 1), sizeof(double));     // unmapped
    if (!out->row_ptr || !out->col_idx || !out->values) {
        spmm_host_csr_free(out);
        return SPMM_HOST_ERR_NOMEM;
    }
    out->row_ptr[0] = 0;
    for (int64_t i = 0; i < m; ++i) out->row_ptr[i + 1] = (int32_t)(out->row_ptr[i] + deg[i]);
    int64_t multi = 0;   // as fill_rows: rows with >= 2 nonzeros over the whole matrix
    for (int64_t d : deg) multi += (d >= 2);
    const double bw_scale = 1.0 / std::max(0.05, (double)multi / (double)std::max<size_t>(deg.size(), 1));
    std::vector<int64_t> segs;
    for (int64_t s = 0; s * SEG < m; ++s) {
        const int64_t a = s * SEG, b = std::min<int64_t>((s + 1) * SEG, m);
        for (int64_t i = a; i < b; ++i)
            if (mask[i]) {
                segs.push_back(s);
                break;
            }
    }
#pragma omp parallel
    {
        RowGen g;
        g.p = p;
        g.bw_scale = bw_scale;
#pragma omp for schedule(dynamic, 1)
        for (size_t q = 0; q < segs.size(); ++q) {
            g.prev.clear();
            g.runs_prev.clear();
            const int64_t a = segs[q] * SEG, b = std::min<int64_t>((segs[q] + 1) * SEG, m);
            int64_t last = a;
            for (int64_t i = a; i < b; ++i)
                if (mask[i]) last = i + 1;
            for (int64_t i = a; i < last; ++i) {
                g.gen(i, deg[i]);
                if (mask[i]) {
                    const int64_t base = out->row_ptr[i];
                    Rng rv((uint64_t)p->seed, (uint64_t)i, S_VALS);
                    for (size_t t = 0; t < g.cur.size(); ++t) {
                        out->col_idx[base + t] = g.cur[t];
                        out->values[base + t] = 0.5 + rv.uniform();
                    }
                }
                if (!g.cur.empty()) {
                    std::swap(g.prev, g.cur);
                    std::swap(g.runs_prev, g.runs_cur);
                }
            }
        }
    }
    return SPMM_HOST_OK;
}

int spmm_host_generate(const spmm_gen_params_t *p, spmm_csr_t *out) {
    if (!valid(p)) return SPMM_HOST_ERR_ARG;
    return spmm_host_generate_rows(p, 0, p->nr_rows, out);
}

int spmm_host_features(const spmm_csr_t *a, spmm_features_t *f) {
    if (!a || !f || a->m < 1 || a->ncols < 1) return SPMM_HOST_ERR_ARG;
    const int64_t m = a->m, n = a->ncols, nnz = a->nnz;
    const int32_t *rp = a->row_ptr, *ci = a->col_idx;
    double s_deg = 0, s_deg2 = 0, s_bw = 0, s_bw2 = 0, s_sc = 0, s_sc2 = 0, s_neigh = 0, s_sim = 0;
    int64_t max_deg = 0, nonempty = 0;
#pragma omp parallel for schedule(static) reduction(+ : s_deg, s_deg2, s_bw, s_bw2, s_sc, s_sc2, s_neigh, s_sim, \
                                                        nonempty) reduction(max : max_deg)
    for (int64_t i = 0; i < m; ++i) {
        const int64_t js = rp[i], je = rp[i + 1], d = je - js;
        s_deg += (double)d;
        s_deg2 += (double)d * (double)d;
        if (d > max_deg) max_deg = d;
        if (d == 0) continue;
        // bandwidth / scatter (csr_util_gen.c:296-309)
        int64_t cmin = ci[js], cmax = ci[js];
        for (int64_t j = js; j < je; ++j) {
            cmin = std::min<int64_t>(cmin, ci[j]);
            cmax = std::max<int64_t>(cmax, ci[j]);
        }
        const double b = (double)(cmax - cmin), sc = b > 0 ? (double)d / b : 0.0;
        s_bw += b;
        s_bw2 += b * b;
        s_sc += sc;
        s_sc2 += sc * sc;
        // row neighbours, window 1 (csr_util_gen.c:459-490): pairs j<k with col[k]-col[j] <= 1, counted twice
        for (int64_t j = js; j < je; ++j)
            for (int64_t k = j + 1; k < je; ++k) {
                if (ci[k] - ci[j] > 1) break;
                s_neigh += 2.0;
            }
        // cross-row similarity, window 1 (csr_util_gen.c:553-610): next non-empty row
        ++nonempty;
        int64_t l = i + 1;
        while (l < m && rp[l + 1] - rp[l] == 0) ++l;
        if (l < m) {
            int64_t k = rp[l];
            const int64_t ke = rp[l + 1];
            int64_t sim = 0;
            for (int64_t j = js; j < je; ++j) {
                while (k < ke) {
                    const int64_t diff = (int64_t)ci[k] - ci[j];
                    if (std::llabs(diff) <= 1) {
                        ++sim;
                        break;
                    }
                    if (diff <= 0)
                        ++k;
                    else
                        break;
                }
            }
            s_sim += (double)sim / (double)d;
        }
    }
    memset(f, 0, sizeof(*f));
    f->nr_rows = m;
    f->nr_cols = n;
    f->nr_nzeros = nnz;
    f->density = (double)nnz / ((double)m * (double)n);
    f->mem_footprint = ((double)nnz * 12.0 + (double)(m + 1) * 4.0) / (1024.0 * 1024.0);
    const double mf = f->mem_footprint;
    snprintf(f->mem_range, sizeof(f->mem_range), "%s",
             mf < 4 ? "[0-4]" : mf < 32 ? "[4-32]" : mf < 512 ? "[32-512]" : mf < 2048 ? "[512-2048]" : "[2048-]");
    const double dm = (double)m;
    f->avg_nnz_per_row = s_deg / dm;
    f->std_nnz_per_row = std::sqrt(std::max(0.0, s_deg2 / dm - f->avg_nnz_per_row * f->avg_nnz_per_row));
    f->avg_bw = s_bw / dm;  // mean over all rows, empty rows count 0 (array_mean(bandwidths, m))
    f->std_bw = std::sqrt(std::max(0.0, s_bw2 / dm - f->avg_bw * f->avg_bw));
    f->avg_bw_scaled = f->avg_bw / (double)n;
    f->std_bw_scaled = f->std_bw / (double)n;
    f->avg_sc = s_sc / dm;
    f->std_sc = std::sqrt(std::max(0.0, s_sc2 / dm - f->avg_sc * f->avg_sc));
    f->avg_sc_scaled = f->avg_sc;  // scatter is already a ratio
    f->std_sc_scaled = f->std_sc;
    f->max_nnz_per_row = max_deg;
    f->skew = f->avg_nnz_per_row > 0 ? ((double)max_deg - f->avg_nnz_per_row) / f->avg_nnz_per_row : 0.0;
    f->avg_num_neighbours = nnz > 0 ? s_neigh / (double)nnz : 0.0;
    f->cross_row_similarity = nonempty > 0 ? s_sim / (double)nonempty : 0.0;
    return SPMM_HOST_OK;
}

void spmm_host_csr_free(spmm_csr_t *a) {
    if (!a) return;
    free(a->row_ptr);
    free(a->col_idx);
    free(a->values);
    a->row_ptr = nullptr;
    a->col_idx = nullptr;
    a->values = nullptr;
}

void spmm_host_drand48_fill(int64_t seed, double *out, int64_t n) {
    uint64_t X = (((uint64_t)seed) << 16) | 0x330EULL;
    for (int64_t i = 0; i < n; ++i) {
        X = (0x5DEECE66DULL * X + 0xBULL) & ((1ULL << 48) - 1);
        out[i] = std::ldexp((double)X, -48);
    }
}

void spmm_host_uniform_fill(int64_t seed, double lo, double hi, double *out, int64_t n) {
    const int64_t CH = 1 << 16;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (n + CH - 1) / CH; ++c) {
        Rng r((uint64_t)seed, (uint64_t)c, 99);
        const int64_t e = std::min<int64_t>(n, (c + 1) * CH);
        for (int64_t i = c * CH; i < e; ++i) out[i] = lo + (hi - lo) * r.uniform();
    }
}

}  // extern "C"
