/*
 * spmm_pipeline.h -- C ABI of the sparse-attention pipeline consumer (libspmm_hip.so), SURVEY.md §8f-4.
 *
 * The reference's pipeline bench (benchmark_code/CPU/AMD/pipeline_code_bench/) drives one plugin per executable
 * through a second Matrix_Format variant (sddmm_kernel.h:9-31):
 *     csr_to_format(mask row_ptr, col_ind, values, m, nnz, n)                 -- holds the attention mask
 *     MF->spmm(type, m, k, n, ia, ja, a, x, y, threads)   type 'K','Q','V'     -- K/Q/V = W_{K,Q,V} x (row-major x)
 *     MF->sddmm(y, threads)                                                    -- y = SDDMM(mask, Q, K)
 *     MF->spmm('final', m, m, n, mask ia, mask ja, y, V, y_final, threads)     -- y_final = mask(y) V
 * (sddmm_bench.cpp:918-937).  The SpMMs map onto the engine (spmm_hip.h: spmm_hip_run_rowmajor / run_device with
 * SPMM_HIP_B_ROW_MAJOR, spmm_hip_update_values[_device] for the final SpMM's values); the SDDMM is below.
 */
#ifndef SPMM_PIPELINE_H
#define SPMM_PIPELINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spmm_sddmm spmm_sddmm_t;

/* SDDMM variants (flags).  Q is [m][n] row-major (m = mask rows), K is [k_rows][n] row-major.
 *   SPMM_SDDMM_REF_ROWDIAG  what the reference computes (sddmm_taco_naive.cpp:98-140, and its own gold,
 *                           sddmm_bench.cpp:260-276): for a mask nonzero p in row i,
 *                           y[p] = a[p] * sum_n Q[i][n] * K[i][n] (row i of K for every column of the row) --
 *                           one FMA chain over n from 0 in order, then one multiply: bit-identical to the reference.
 *   SPMM_SDDMM_QKT          the attention SDDMM: y[p] = a[p] * sum_n Q[i][n] * K[col(p)][n], same chain order.
 *   SPMM_SDDMM_SOFTMAX      (or'ed in) then y = softmax over all nonzeros -- the reference's softmax()
 *                           (sddmm_taco_naive.cpp:191-209; commented out in its pipeline and gold); deterministic
 *                           tree reductions, within tolerance of the serial order, not bit-identical. */
#define SPMM_SDDMM_REF_ROWDIAG  0
#define SPMM_SDDMM_QKT          1
#define SPMM_SDDMM_SOFTMAX      2

/* Mask: CSR [m][ncols] with values a (the reference's mask values are 1.0); n = feature width (NUM_COLS). */
int spmm_sddmm_create(const int32_t *row_ptr, const int32_t *col_idx, const void *mask_vals, int64_t m, int64_t ncols,
                      int64_t nnz, int32_t n, int32_t dtype, int32_t flags, int32_t device, spmm_sddmm_t **out);
/* Host buffers (synchronous): Q [m][n], K [k_rows][n], y [nnz]. */
int spmm_sddmm_run(spmm_sddmm_t *s, const void *Q, const void *K, int64_t k_rows, void *y);
/* Device buffers, stream-ordered (graph-capturable). */
int spmm_sddmm_run_device(spmm_sddmm_t *s, const void *d_Q, const void *d_K, void *d_y, void *stream);
int spmm_sddmm_destroy(spmm_sddmm_t *s);
const char *spmm_sddmm_last_error_detail(void);

#ifdef __cplusplus
}
#endif

#endif /* SPMM_PIPELINE_H */
