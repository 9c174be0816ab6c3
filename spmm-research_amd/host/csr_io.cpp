// csr_io.cpp -- Matrix Market reader and COO->CSR conversion (the input path in front of the SpMM kernel).
//
// Behaviour follows the reference exactly where it defines the CSR the kernel sees:
//   header          matrix_market.c:149-239 ("%%MatrixMarket matrix <coordinate|array> <field> <symmetry>"; a file
//                   without the banner is read as coordinate/real/general; '%' comment lines skipped)
//   coordinate data matrix_market_gen.c:70-158: 1-based -> 0-based; for symmetric / skew-symmetric / Hermitian
//                   the mirrored off-diagonal entries are APPENDED after all file entries, in file order, with
//                   value v (symmetric), -v (skew), conj(v) (Hermitian)
//   field values    spmv_bench.cpp:730-763: integer -> double, complex -> |z|, pattern -> 1.0
//   coo_to_csr      csr_gen.c:163-217: rows bucketed, then each row's entries sorted by column; duplicates kept.
//                   The order of DUPLICATE (row, col) values follows the reference run by one OpenMP thread: its row
//                   bucketing (bucketsort_gen.c:163-199) hands slots out from the end of each row with an atomic
//                   decrement, so with several threads the order among duplicates depends on thread timing (not
//                   reproducible even by the reference); with one thread a row holds its file entries reversed, and
//                   the per-row column sort (stable bucket sort for rows longer than n/5, the reference quicksort
//                   otherwise) is restated exactly, so duplicate values come out in the reference's order.
// "array" format (dense, column-major) is read as a full coordinate listing (the reference would dereference a
// NULL row array there).
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/spmm_host.h"

namespace {

struct Lines {
    std::string buf;
    std::vector<size_t> start;  // offsets of non-empty lines
};

int read_lines(const char *path, Lines &L) {
    FILE *f = fopen(path, "rb");
    if (!f) return SPMM_HOST_ERR_IO;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (sz < 0) {
        fclose(f);
        return SPMM_HOST_ERR_IO;
    }
    L.buf.resize((size_t)sz + 1);
    size_t got = fread(&L.buf[0], 1, (size_t)sz, f);
    fclose(f);
    L.buf.resize(got);
    L.buf.push_back('\n');
    size_t p = 0;
    while (p < L.buf.size()) {
        size_t e = L.buf.find('\n', p);
        if (e == std::string::npos) e = L.buf.size();
        // skip blank lines (file_to_lines splits on newlines and drops empty atoms)
        size_t q = p;
        while (q < e && (L.buf[q] == ' ' || L.buf[q] == '\t' || L.buf[q] == '\r')) ++q;
        if (q < e) L.start.push_back(p);
        L.buf[e] = '\0';
        p = e + 1;
    }
    return SPMM_HOST_OK;
}

// csr_sort_columns' per-row sorts (csr_gen.c:120-140), restated.  Rows of more than n/5 entries: a stable bucket
// sort by column (bucketsort_stable_serial, bucketsort_gen.c:127-160).  Shorter rows: the reference quicksort of
// the entries' indices keyed by column (quicksort_gen.c:93-127 with partition_auto_serial / partition_serial_base,
// partition_gen.c:146-193,269-294 and the comparator csr_gen.c:33-37) -- deterministic (its srandom_r state is
// never read) but not stable, so the order it leaves among duplicate columns is its own; restated step by step.
void ref_bucket_stable(const int32_t *cols, int64_t deg, int32_t *src_of_slot) {
    std::vector<int64_t> idx((size_t)deg);
    for (int64_t q = 0; q < deg; ++q) idx[(size_t)q] = q;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return cols[a] < cols[b]; });
    for (int64_t q = 0; q < deg; ++q) src_of_slot[q] = (int32_t)idx[(size_t)q];
}

inline int qcmp(int32_t a, int32_t b, const int32_t *keys) {
    return keys[a] > keys[b] ? 1 : keys[a] < keys[b] ? -1 : 0;
}

// entries [lo, hi] (inclusive) around `pivot`: returns the first index of the right part
int64_t part_base(int32_t pivot, int32_t *A, int64_t lo, int64_t hi, const int32_t *keys) {
    for (;;) {
        while (lo < hi && qcmp(A[lo], pivot, keys) < 0) ++lo;
        while (lo < hi && qcmp(A[hi], pivot, keys) > 0) --hi;
        if (lo >= hi) break;
        std::swap(A[lo], A[hi]);
        ++lo;
        --hi;
    }
    if (qcmp(A[lo], pivot, keys) < 0) ++lo;
    return lo;
}

// [s, e) with a median-of-three pivot at the middle
int64_t part_auto(int32_t *A, int64_t s, int64_t e, const int32_t *keys) {
    if (e - s == 1) return s;
    if (e - s == 2) {
        if (qcmp(A[s], A[s + 1], keys) > 0) std::swap(A[s], A[s + 1]);
        return s + 1;
    }
    const int64_t last = e - 1, mid = (s + last) / 2;
    if (qcmp(A[s], A[last], keys) > 0) std::swap(A[s], A[last]);
    if (qcmp(A[s], A[mid], keys) > 0) std::swap(A[s], A[mid]);
    if (qcmp(A[mid], A[last], keys) > 0) std::swap(A[mid], A[last]);
    return part_base(A[mid], A, s + 1, last - 1, keys);
}

// the reference's iterative driver: partition [s, e], remember s, continue with the right part; when a part is
// down to one element, step e back by one and resume from the remembered start
void ref_quicksort(int32_t *A, int64_t N, const int32_t *keys, std::vector<int64_t> &stack) {
    if (N < 2) return;
    stack.assign((size_t)N + 1, 0);
    int64_t s = 0, e = N - 1, i = 0;
    for (;;) {
        while (s >= e) {
            if (s == 0) return;
            --i;
            --e;
            s = stack[(size_t)i];
        }
        const int64_t m = part_auto(A, s, e + 1, keys);
        stack[(size_t)i++] = s;
        s = m;
    }
}

}  // namespace

extern "C" {

int spmm_host_coo_to_csr(const int32_t *R, const int32_t *C, const double *V, int64_t m, int64_t n, int64_t nnz,
                         int32_t *row_ptr, int32_t *col_idx, double *values) {
    if (m < 0 || n < 0 || nnz < 0 || !row_ptr || (nnz > 0 && (!R || !C || !col_idx))) return SPMM_HOST_ERR_ARG;
    if (nnz >= INT32_MAX) return SPMM_HOST_ERR_OVERFLOW;
    std::vector<int64_t> end((size_t)m + 1, 0);
    for (int64_t i = 0; i < nnz; ++i) {
        if (R[i] < 0 || R[i] >= m || C[i] < 0 || C[i] >= n) return SPMM_HOST_ERR_ARG;
        end[R[i] + 1]++;
    }
    for (int64_t i = 0; i < m; ++i) end[i + 1] += end[i];
    for (int64_t i = 0; i <= m; ++i) row_ptr[i] = (int32_t)end[i];
    // 1. rows bucketed like the reference's bucketsort (bucketsort_gen.c:163-199) run by ONE thread: each entry
    //    takes the next free slot from the END of its row, so a row holds its file entries in reverse order
    std::vector<int32_t> Cb((size_t)nnz);
    std::vector<double> Vb((size_t)nnz);
    {
        std::vector<int64_t> top(end.begin() + 1, end.end());
        for (int64_t i = 0; i < nnz; ++i) {
            const int64_t pos = --top[R[i]];
            Cb[(size_t)pos] = C[i];
            Vb[(size_t)pos] = V ? V[i] : 1.0;
        }
    }
    // 2. each row sorted by column (csr_sort_columns, csr_gen.c:83-156)
#pragma omp parallel
    {
        std::vector<int32_t> perm;
        std::vector<int64_t> stack;
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < m; ++i) {
            const int64_t s = end[i], deg = end[i + 1] - s;
            if (deg == 0) continue;
            perm.resize((size_t)deg);
            if (deg > n / 5) {
                ref_bucket_stable(Cb.data() + s, deg, perm.data());      // perm[q] = source of slot q
            } else {
                for (int64_t q = 0; q < deg; ++q) perm[(size_t)q] = (int32_t)q;
                ref_quicksort(perm.data(), deg, Cb.data() + s, stack);
            }
            for (int64_t q = 0; q < deg; ++q) {
                col_idx[s + q] = Cb[(size_t)(s + perm[(size_t)q])];
                if (values) values[s + q] = Vb[(size_t)(s + perm[(size_t)q])];
            }
        }
    }
    return SPMM_HOST_OK;
}

int spmm_host_mtx_read(const char *path, spmm_csr_t *out, char *field_out, int field_n, int32_t *symmetric_out) {
    if (!path || !out) return SPMM_HOST_ERR_ARG;
    memset(out, 0, sizeof(*out));
    Lines L;
    int st = read_lines(path, L);
    if (st) return st;
    if (L.start.empty()) return SPMM_HOST_ERR_PARSE;
    size_t li = 0;
    std::string format = "coordinate", field = "real";
    int sym = 0;  // 0 general, 1 symmetric/Hermitian, 2 skew
    bool hermitian = false;
    {
        const char *h = &L.buf[L.start[0]];
        char t0[64] = {0}, t1[64] = {0}, t2[64] = {0}, t3[64] = {0}, t4[64] = {0};
        int n = sscanf(h, "%63s %63s %63s %63s %63s", t0, t1, t2, t3, t4);
        if (n >= 1 && strcmp(t0, "%%MatrixMarket") == 0) {
            if (n < 5 || strcmp(t1, "matrix") != 0 || (strcmp(t2, "coordinate") && strcmp(t2, "array")))
                return SPMM_HOST_ERR_PARSE;
            format = t2;
            field = t3;
            if (!strcmp(t4, "symmetric"))
                sym = 1;
            else if (!strcmp(t4, "Hermitian")) {
                sym = 1;
                hermitian = true;
            } else if (!strcmp(t4, "skew-symmetric"))
                sym = 2;
            else if (strcmp(t4, "general"))
                return SPMM_HOST_ERR_PARSE;
            li = 1;
        }
    }
    while (li < L.start.size() && L.buf[L.start[li]] == '%') ++li;
    if (li >= L.start.size()) return SPMM_HOST_ERR_PARSE;
    const bool complex_w = (field == "complex");
    const bool pattern = (field == "pattern");
    const bool integer = (field == "integer");
    if (!complex_w && !pattern && !integer && field != "real") return SPMM_HOST_ERR_PARSE;
    long long M = 0, N = 0, NZ = 0;
    const bool coord = (format == "coordinate");
    if (coord) {
        if (sscanf(&L.buf[L.start[li]], "%lld %lld %lld", &M, &N, &NZ) != 3) return SPMM_HOST_ERR_PARSE;
    } else {
        if (sscanf(&L.buf[L.start[li]], "%lld %lld", &M, &N) != 2) return SPMM_HOST_ERR_PARSE;
        NZ = M * N;
    }
    ++li;
    if ((long long)(L.start.size() - li) != NZ) return SPMM_HOST_ERR_PARSE;  // matrix_market.c:228-229
    if (M < 0 || N < 0 || M >= INT32_MAX || N >= INT32_MAX || 2 * NZ >= INT32_MAX) return SPMM_HOST_ERR_OVERFLOW;

    std::vector<int32_t> R, C;
    std::vector<double> V;
    R.resize((size_t)NZ);
    C.resize((size_t)NZ);
    V.resize((size_t)NZ);
    std::vector<std::complex<double>> Z;
    if (complex_w) Z.resize((size_t)NZ);
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (long long e = 0; e < NZ; ++e) {
        char *s = &L.buf[L.start[li + (size_t)e]];
        char *end;
        if (coord) {
            long r = strtol(s, &end, 10);
            long c = strtol(end, &end, 10);
            if (r < 1 || c < 1 || r > M || c > N) bad |= 1;
            R[e] = (int32_t)(r - 1);
            C[e] = (int32_t)(c - 1);
            s = end;
        } else {  // array: column-major listing
            R[e] = (int32_t)(e % M);
            C[e] = (int32_t)(e / M);
        }
        if (pattern) {
            V[e] = 1.0;
        } else if (integer) {
            V[e] = (double)(int)strtol(s, &end, 10);
        } else if (complex_w) {
            double re = strtod(s, &end);
            double im = strtod(end, &end);
            Z[e] = std::complex<double>(re, im);
        } else {
            V[e] = strtod(s, &end);
        }
    }
    if (bad) return SPMM_HOST_ERR_PARSE;
    int64_t nnz = NZ;
    if (sym) {  // append the mirrored off-diagonal entries in file order
        for (long long e = 0; e < NZ; ++e) {
            if (R[e] == C[e]) continue;
            R.push_back(C[e]);
            C.push_back(R[e]);
            if (complex_w) {
                std::complex<double> z = Z[e];
                Z.push_back(sym == 2 ? -std::conj(z) : (hermitian ? std::conj(z) : std::conj(z)));
            } else {
                V.push_back(sym == 2 ? -V[e] : V[e]);
            }
        }
        nnz = (int64_t)R.size();
        if (!complex_w) V.resize((size_t)nnz);
    }
    if (complex_w) {
        V.resize((size_t)nnz);
        for (int64_t e = 0; e < nnz; ++e) V[e] = std::abs(Z[e]);
    }
    out->m = M;
    out->ncols = N;
    out->nnz = nnz;
    out->row_ptr = (int32_t *)malloc((size_t)(M + 1) * sizeof(int32_t));
    out->col_idx = (int32_t *)malloc((size_t)std::max<int64_t>(nnz, 1) * sizeof(int32_t));
    out->values = (double *)malloc((size_t)std::max<int64_t>(nnz, 1) * sizeof(double));
    if (!out->row_ptr || !out->col_idx || !out->values) {
        spmm_host_csr_free(out);
        return SPMM_HOST_ERR_NOMEM;
    }
    st = spmm_host_coo_to_csr(R.data(), C.data(), V.data(), M, N, nnz, out->row_ptr, out->col_idx, out->values);
    if (st) {
        spmm_host_csr_free(out);
        return st;
    }
    if (field_out && field_n > 0) snprintf(field_out, (size_t)field_n, "%s", field.c_str());
    if (symmetric_out) *symmetric_out = sym;
    return SPMM_HOST_OK;
}

// DLMC .smtx (lib/storage_formats/dlcm_matrices/dlcm_matrix.c:152-255 header, dlcm_matrix_gen.c:56-123 body):
//   line 1  "M, K, nnz"            (sscanf "%ld,%ld,%ld")
//   line 2  M+1 row offsets        (whitespace-separated; the CSR row_ptr, used as is)
//   line 3  nnz column indices     (0-based, used as is: the harness copies them without coo_to_csr,
//                                   spmv_bench.cpp:769-801, so rows keep the file's column order)
// The format carries no values: the reference draws U(-1, 1) from rand() re-seeded with time(NULL) + j + thread
// (dlcm_matrix_gen.c:111-122), i.e. not reproducible; here they are a seeded uniform [-1, 1) stream
// (spmm_host_uniform_fill(value_seed, -1, 1)).  The reference parses without checks; malformed offsets or
// out-of-range columns are rejected here (SPMM_HOST_ERR_PARSE).
int spmm_host_smtx_read(const char *path, int64_t value_seed, spmm_csr_t *out) {
    if (!path || !out) return SPMM_HOST_ERR_ARG;
    memset(out, 0, sizeof(*out));
    Lines L;
    int st = read_lines(path, L);
    if (st) return st;
    if (L.start.empty()) return SPMM_HOST_ERR_PARSE;
    long long M = 0, K = 0, NZ = 0;
    if (sscanf(&L.buf[L.start[0]], "%lld,%lld,%lld", &M, &K, &NZ) != 3) return SPMM_HOST_ERR_PARSE;
    if (M < 0 || K < 0 || NZ < 0) return SPMM_HOST_ERR_PARSE;
    if (M >= INT32_MAX || K >= INT32_MAX || NZ >= INT32_MAX) return SPMM_HOST_ERR_OVERFLOW;
    if (L.start.size() < (NZ > 0 ? 3u : 2u)) return SPMM_HOST_ERR_PARSE;
    out->row_ptr = (int32_t *)malloc((size_t)(M + 1) * sizeof(int32_t));
    out->col_idx = (int32_t *)malloc((size_t)std::max<long long>(NZ, 1) * sizeof(int32_t));
    out->values = (double *)malloc((size_t)std::max<long long>(NZ, 1) * sizeof(double));
    if (!out->row_ptr || !out->col_idx || !out->values) {
        spmm_host_csr_free(out);
        return SPMM_HOST_ERR_NOMEM;
    }
    // n integers from one line; fails on a short line or a token that is not a number
    auto parse_ints = [](char *s, long long n, long long lo, long long hi, int32_t *dst) -> bool {
        for (long long j = 0; j < n; ++j) {
            char *end;
            const long long v = strtoll(s, &end, 10);
            if (end == s || v < lo || v > hi) return false;
            dst[j] = (int32_t)v;
            s = end;
        }
        return true;
    };
    bool ok = parse_ints(&L.buf[L.start[1]], M + 1, 0, NZ, out->row_ptr) && out->row_ptr[0] == 0 &&
              out->row_ptr[M] == NZ;
    for (long long i = 0; ok && i < M; ++i) ok = out->row_ptr[i] <= out->row_ptr[i + 1];
    if (ok && NZ > 0) ok = parse_ints(&L.buf[L.start[2]], NZ, 0, K - 1, out->col_idx);
    if (!ok) {
        spmm_host_csr_free(out);
        return SPMM_HOST_ERR_PARSE;
    }
    out->m = M;
    out->ncols = K;
    out->nnz = NZ;
    spmm_host_uniform_fill(value_seed, -1.0, 1.0, out->values, NZ);
    return SPMM_HOST_OK;
}

}  // extern "C"
