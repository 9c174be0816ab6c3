// csr_io.cpp -- Matrix Market reader and COO->CSR conversion (the input path in front of the SpMM kernel).
//
// Behaviour follows the reference exactly where it defines the CSR the kernel sees:
//   header          matrix_market.c:149-239 ("%%MatrixMarket matrix <coordinate|array> <field> <symmetry>"; a file
//                   without the banner is read as coordinate/real/general; '%' comment lines skipped)
//   coordinate data matrix_market_gen.c:70-158: 1-based -> 0-based; for symmetric / skew-symmetric / Hermitian
//                   the mirrored off-diagonal entries are APPENDED after all file entries, in file order, with
//                   value v (symmetric), -v (skew), conj(v) (Hermitian)
//   field values    spmv_bench.cpp:730-763: integer -> double, complex -> |z|, pattern -> 1.0
//   coo_to_csr      csr_gen.c:163-217: rows bucketed, then each row's entries sorted by column; duplicates kept
// The one deliberate difference: among duplicate (row, col) entries the reference's per-row quicksort is not
// stable; we keep file order (stable), so duplicate VALUES may sit in a different order (indexing is identical).
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

}  // namespace

extern "C" {

int spmm_host_coo_to_csr(const int32_t *R, const int32_t *C, const double *V, int64_t m, int64_t nnz,
                         int32_t *row_ptr, int32_t *col_idx, double *values) {
    if (m < 0 || nnz < 0 || !row_ptr || (nnz > 0 && (!R || !C || !col_idx))) return SPMM_HOST_ERR_ARG;
    if (nnz >= INT32_MAX) return SPMM_HOST_ERR_OVERFLOW;
    std::vector<int64_t> cnt((size_t)m + 1, 0);
    for (int64_t i = 0; i < nnz; ++i) {
        if (R[i] < 0 || R[i] >= m) return SPMM_HOST_ERR_ARG;
        cnt[R[i] + 1]++;
    }
    for (int64_t i = 0; i < m; ++i) cnt[i + 1] += cnt[i];
    for (int64_t i = 0; i <= m; ++i) row_ptr[i] = (int32_t)cnt[i];
    std::vector<int64_t> perm((size_t)nnz);
    {
        std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
        for (int64_t i = 0; i < nnz; ++i) perm[fill[R[i]]++] = i;  // stable bucket by row
    }
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t i = 0; i < m; ++i)
        std::stable_sort(perm.begin() + cnt[i], perm.begin() + cnt[i + 1],
                         [&](int64_t a, int64_t b) { return C[a] < C[b]; });
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < nnz; ++p) {
        col_idx[p] = C[perm[p]];
        if (values) values[p] = V ? V[perm[p]] : 1.0;
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
    st = spmm_host_coo_to_csr(R.data(), C.data(), V.data(), M, nnz, out->row_ptr, out->col_idx, out->values);
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
