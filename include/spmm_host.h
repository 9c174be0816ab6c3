/*
 * spmm_host.h -- C ABI of the host-side input path of the SpMM engine (libspmm_host.so, no GPU needed).
 *
 * These replace the reference's host inputs to the hot path:
 *   spmm_host_mtx_read      mtx_read(file, expand_symmetry=1, pattern_dummy_vals=1) + the harness's value
 *                           conversion + coo_to_csr(..., sort_columns=1, transpose=0)
 *                           (lib/storage_formats/matrix_market/matrix_market.c:249-314,
 *                            matrix_market_gen.c:70-158; spmv_bench.cpp:724-763,805-826; csr_gen.c:163-217)
 *   spmm_host_smtx_read     smtx_read (DLMC .smtx: lib/storage_formats/dlcm_matrices/dlcm_matrix.c:152-324) + the
 *                           harness's USE_DLCM_MATRICES copy (spmv_bench.cpp:667-696,769-801)
 *   spmm_host_coo_to_csr    coo_to_csr (lib/storage_formats/csr/csr_gen.c:163-217)
 *   spmm_host_generate      artificial_matrix_generation(nr_rows, nr_cols, avg, std, distribution, seed,
 *                           placement, bw, skew, avg_num_neighbours, cross_row_similarity)
 *                           (call sites spmv_bench.cpp:842-869; the generator submodule itself is absent from
 *                            the reference tree -- this is a from-scratch design)
 *   spmm_host_features      the structural features the harness prints for synthetic matrices
 *                           (spmv_bench.cpp:522-545; definitions lib/storage_formats/csr_util/csr_util_gen.c:
 *                            269-329 degrees/bandwidths/scatters, 459-490 row neighbours, 553-610 cross-row
 *                            similarity, 964-983 twin line)
 *   spmm_host_check_accuracy CheckAccuracy (spmv_bench.cpp:121-206) plus a normwise cancellation-robust check
 */
#ifndef SPMM_HOST_H
#define SPMM_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int64_t m, ncols, nnz;
    int32_t *row_ptr; /* [m+1]   */
    int32_t *col_idx; /* [nnz]   */
    double *values;   /* [nnz]   double, as the harness's csr_a_ref */
} spmm_csr_t;

/* Fields of the reference's csr_matrix that the harness prints (spmv_bench.cpp:522-545). */
typedef struct {
    char distribution[16];
    char placement[16];
    int64_t seed;
    int64_t nr_rows, nr_cols, nr_nzeros;
    double density;
    double mem_footprint; /* MB: (nnz*(4+8) + (m+1)*4) / 2^20 */
    char mem_range[32];
    double avg_nnz_per_row, std_nnz_per_row;
    double avg_bw, std_bw, avg_bw_scaled, std_bw_scaled;
    double avg_sc, std_sc, avg_sc_scaled, std_sc_scaled;
    double skew;
    double avg_num_neighbours;
    double cross_row_similarity;
    int64_t max_nnz_per_row;
} spmm_features_t;

/* Generator parameters, in the reference's argv order (spmv_bench.cpp:852-862). */
typedef struct {
    int64_t nr_rows, nr_cols;
    double avg_nnz_per_row, std_nnz_per_row;
    char distribution[16]; /* "normal" | "gamma" */
    char placement[16];    /* "random" | "diagonal" */
    double bw;             /* target mean(max col - min col) / nr_cols */
    double skew;           /* target (max row degree - avg) / avg */
    double avg_num_neighbours;   /* target mean #same-row nonzeros at |dcol| <= 1 */
    double cross_row_similarity; /* target mean fraction of a row's nonzeros with one at |dcol| <= 1 in the next row */
    int64_t seed;
} spmm_gen_params_t;

#define SPMM_HOST_OK 0
#define SPMM_HOST_ERR_ARG -1
#define SPMM_HOST_ERR_IO -2
#define SPMM_HOST_ERR_PARSE -3
#define SPMM_HOST_ERR_NOMEM -4
#define SPMM_HOST_ERR_OVERFLOW -5

/* Parse one 11-field generator line ("rows cols avg std distribution placement bw skew neigh crs seed"). */
int spmm_host_parse_gen_line(const char *line, spmm_gen_params_t *p);

/* Whole matrix.  Deterministic for a given parameter set, independent of the thread count. */
int spmm_host_generate(const spmm_gen_params_t *p, spmm_csr_t *out);

/* Row lengths of the whole matrix only (cheap: lets ranks partition before generating their shard). */
int spmm_host_generate_row_ptr(const spmm_gen_params_t *p, int32_t *row_ptr /* [nr_rows+1] */);

/* Rows [r0, r1) of the same matrix: out->row_ptr is rebased to start at 0; column ids stay global. */
int spmm_host_generate_rows(const spmm_gen_params_t *p, int64_t r0, int64_t r1, spmm_csr_t *out);
/* The whole matrix's row_ptr, with the columns and values of the rows where mask[i] != 0 only (the other rows'
 * entries are zero); the masked rows equal those of spmm_host_generate.  Only the generator segments holding a
 * masked row are generated (a row sample of a large matrix: tools/plan_census.py). */
int spmm_host_generate_masked(const spmm_gen_params_t *p, const uint8_t *mask, spmm_csr_t *out);

int spmm_host_features(const spmm_csr_t *a, spmm_features_t *f);

/* .mtx -> CSR (indexing identical to mtx_read + coo_to_csr).  field_out receives the header field
 * ("real", "integer", "complex", "pattern"), symmetric_out 0/1/2 (general/symmetric-or-Hermitian/skew). */
int spmm_host_mtx_read(const char *path, spmm_csr_t *out, char *field_out, int field_n, int32_t *symmetric_out);

/* DLMC .smtx -> CSR (smtx_read + the harness copy, lib/storage_formats/dlcm_matrices/dlcm_matrix.c:152-324,
 * spmv_bench.cpp:667-696,769-801): row offsets and column indices used as stored (no sort); the format has no
 * values, so they are a seeded uniform [-1, 1) stream (the reference's are time-seeded rand(), unreproducible). */
int spmm_host_smtx_read(const char *path, int64_t value_seed, spmm_csr_t *out);

/* coo_to_csr(R, C, V, m, n, nnz, row_ptr, col_idx, values, sort_columns=1, transpose=0) (csr_gen.c:163-217):
 * rows bucketed, each row sorted by column, duplicates kept.  Duplicate (row, col) values keep the order the
 * reference leaves when run by one OpenMP thread (file entries reversed by the row bucketing, then its per-row
 * sort: stable bucket sort for rows of more than n/5 entries, its quicksort otherwise); with several threads the
 * reference's own order among duplicates depends on thread timing (atomic slot hand-out, bucketsort_gen.c:186-194).
 * V may be NULL (values 1.0). */
int spmm_host_coo_to_csr(const int32_t *R, const int32_t *C, const double *V, int64_t m, int64_t n, int64_t nnz,
                         int32_t *row_ptr, int32_t *col_idx, double *values);

void spmm_host_csr_free(spmm_csr_t *a);

/* Fill helpers: drand48 stream (srand48(seed)), seeded uniform [lo, hi). */
void spmm_host_drand48_fill(int64_t seed, double *out, int64_t n);
void spmm_host_uniform_fill(int64_t seed, double lo, double hi, double *out, int64_t n);

/* CheckAccuracy (spmv_bench.cpp:121-206).  values_ref / x_ref are double (x column-major [k][ncols]); y_test is
 * row-major [m][k] of dtype (0 = double, 1 = float).  eps = 1e-10 (fp64) / 1e-7 (fp32) as :125-129.
 * out[0] max relative diff over y_gold > eps (the reference's pass/fail number)
 * out[1..8] mae, max_ae, mse, mape, smape, lnQ_error, mlare, gmare
 * out[9] entries failing |y - gold| <= eps * max(|gold|, sum_j |a_ij b_jn|)  (SURVEY §8a normwise criterion)
 * out[10] max over entries of |y - gold| / max(|gold|, sum_j |a_ij b_jn|) */
int spmm_host_check_accuracy(const int32_t *row_ptr, const int32_t *col_idx, const double *values_ref, int64_t m,
                             int64_t ncols, const double *x_ref, int32_t k, const void *y_test, int32_t dtype,
                             double eps, double *out);

#ifdef __cplusplus
}
#endif

#endif /* SPMM_HOST_H */
