/*
 * spmm_pbv.h -- C ABI of the perfect-balance CSR format (libspmm_pbv.so): K = 1 SpMV with every lane given the
 * same number of merge items, the GPU form of the reference's "Custom_CSR_PBV" format.
 *
 * Reference interface it replaces: the CUSTOM_VECTOR_PERFECT_NNZ_BALANCE build of the CSR plugin
 * (benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel_csr.cpp:68-80 partition, :183-184 dispatch, :196-201
 * format name, :626-680 compute_csr_vector_perfect_nnz_balance), behind the same plugin surface as the engine
 * (spmv_kernel.h:9-30: csr_to_format / spmm(x, y, k) / statistics).  The reference splits the nonzeros evenly over
 * OpenMP threads; a thread's first and last rows may be partial, and the partial sums are added in a serial fix-up.
 * Here the unit is a lane: the m row ends and nnz nonzeros form one merged sequence of m + nnz items (merge path),
 * cut into blocks of 256 x E items (one workgroup) and lanes of E items, so every lane does the same work however
 * the row lengths are distributed (empty rows cost one item).
 *
 * Numerics: a row whose items all fall in one lane is one left-to-right FMA chain from 0 in CSR order -- bit-identical
 * to the reference's serial compute_csr row (spmm_pbv_exact_rows reports these rows).  A row cut by lane boundaries is
 * the sum of its lane pieces in lane order (each piece a chain), plus, for rows cut by block boundaries, the block
 * pieces added first in block order: deterministic, within 1e-10 relative normwise of the exact sum (fp64).  The
 * reference's PBV format also splits rows (at its thread boundaries), so its bits depend on its thread count; the
 * oracle pins split rows by the normwise bound against a float128 gold, not by bits.
 *
 * Status codes, dtypes and B layouts are the engine's (spmm_hip.h).
 */
#ifndef SPMM_PBV_H
#define SPMM_PBV_H

#include <stdint.h>

#include "spmm_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spmm_pbv_handle spmm_pbv_t;

/* items (row ends + nonzeros) per lane the factory accepts; a workgroup holds 256 x E items */
#define SPMM_PBV_E_MIN  4
#define SPMM_PBV_E_MAX  16

/* Host-only plan (no device needed): the merge-path coordinates of every block start and the exact-row mask.
 *   blk_out    int32 [2 * (nblk + 1)]: {row, nonzero} of the first item of block b (b = nblk: {m, nnz})
 *   exact_out  uint8 [m] (may be NULL): 1 = the row's items lie in one lane (bit-identical row)
 * nblk = ceil((m + nnz) / (256 * items_per_lane)) (0 when m = 0); spmm_pbv_nblk() returns it. */
int64_t spmm_pbv_nblk(int64_t m, int64_t nnz, int32_t items_per_lane);
int spmm_pbv_plan_host(const int32_t *row_ptr, int64_t m, int64_t nnz, int32_t items_per_lane, int32_t *blk_out,
                       uint8_t *exact_out);

/* Factory: replaces csr_to_format (spmv_kernel.h:29) of the PBV build.  Borrows the host arrays for the call:
 * validates A, copies it and the block table to `device`.  items_per_lane: E in [SPMM_PBV_E_MIN, SPMM_PBV_E_MAX]
 * (0 = the default, 8). */
int spmm_pbv_create(const int32_t *row_ptr, const int32_t *col_idx, const void *values, int64_t m, int64_t ncols,
                    int64_t nnz, int32_t dtype, int32_t device, int32_t items_per_lane, spmm_pbv_t **out);

/* Execute, host buffers: replaces Matrix_Format::spmm(x, y, k) (spmv_kernel.h:18).  x column-major [k][ncols],
 * y row-major [m][k] (the reference layouts); K > 1 runs the SpMV once per column of x (the format is a K = 1
 * format, as the reference's is an SpMV format).  Synchronous. */
int spmm_pbv_run(spmm_pbv_t *h, const void *x, void *y, int32_t k);

/* Execute, device buffers: y[i * ldy] = sum_j A[i][j] x[j] for one vector x (device, ncols entries); stream is a
 * hipStream_t (NULL = the null stream).  Two launches: the block kernel and the cross-block fix-up. */
int spmm_pbv_run_device(spmm_pbv_t *h, const void *d_x, void *d_y, int64_t ldy, void *stream);

/* Kernel time (ms, HIP events around both launches) of the last run_device / run call (last column for K > 1). */
int spmm_pbv_last_ms(spmm_pbv_t *h, double *ms);

/* out[0..m): 1 = the row is bit-identical to the reference's serial row */
int spmm_pbv_exact_rows(spmm_pbv_t *h, uint8_t *out);

/* out[0] blocks, [1] items per lane, [2] exact rows, [3] rows cut by a block boundary, [4] device bytes held */
int spmm_pbv_info(spmm_pbv_t *h, int64_t *out, int32_t n);

/* Statistics: statistics_print_labels / statistics_print_data counterparts (spmv_kernel.h:20,30), as the engine's
 * spmm_hip_stats_labels / spmm_hip_stats: append CSV columns, return the characters written.  Columns:
 *   kernel_ms,bytes_alg,hbm_gbs_alg,roofline_frac,blocks,items_per_lane,exact_rows,device */
int spmm_pbv_stats_labels(char *buf, long buf_n);
int spmm_pbv_stats(spmm_pbv_t *h, char *buf, long buf_n);

int spmm_pbv_destroy(spmm_pbv_t *h);
const char *spmm_pbv_last_error_detail(void);

#ifdef __cplusplus
}
#endif

#endif /* SPMM_PBV_H */
