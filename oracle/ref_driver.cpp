/*
 * oracle/ref_driver.cpp -- a thin extern "C" driver over the REFERENCE's own compiled sources.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/spmm_oracle.c header).  oracle/Makefile compiles this file together with
 * the reference's sources *where they lie* under /root/reference (nothing is copied into this repo) into
 * oracle/_ref/libspmm_ref_{d,f}.so.  It is used to (1) generate the golden fixtures in tests/golden/ and
 * (2) time the reference kernel as bench.py's cpu_baseline (kind "reference").
 *
 * Everything below calls reference code; the only logic here is the call sequence the reference harness uses:
 *   ref_spmm         csr_to_format(...)->spmm(x, y, k)  (spmv_bench.cpp:996, :372 -> spmm_kernel_csr.cpp:51-96)
 *   ref_mtx_to_csr   mtx_read + field conversion + coo_to_csr(..., sort_columns=1, transpose=0)
 *                    (spmv_bench.cpp:724-763 and :805-826)
 *   ref_smtx_read    DLMC smtx_read (lib/storage_formats/dlcm_matrices/dlcm_matrix.c:258-324), offsets and columns
 *   ref_partition    loop_partitioner_balance_prefix_sums (lib/parallel_util.h:141-165)
 *   ref_metrics      the 8 array_metrics calls of CheckAccuracy (spmv_bench.cpp:189-203)
 *   ref_features     csr_matrix_features_validation (lib/storage_formats/csr_util/csr_util_gen.c:889-990, built as
 *                    lib/aux/csr_util.c): the feature extractor that prints a matrix's 11-field generator "twin" line
 *                    (rows cols avg std normal random bw skew neighbours cross_row_similarity 14) on stderr
 */
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <math.h>
#include <complex.h>
#include <omp.h>

#include "macros/cpp_defines.h"
#include "spmv_bench_common.h"
#include "spmv_kernel.h"

extern "C" {
#include "macros/macrolib.h"
#include "parallel_util.h"
#include "array_metrics.h"
#include "storage_formats/matrix_market/matrix_market.h"
#include "aux/csr_converter_double.h"
#include "aux/csr_util.h"
#include "storage_formats/dlcm_matrices/dlcm_matrix.h"
}
#include <unistd.h>

extern "C" {

/* The reference extractor writes its result to stderr (and timings to stdout): capture both into a temporary file
 * and return the stderr text (at most out_n - 1 chars).  Returns the length, or -1. */
long ref_features(INT_T *row_ptr, INT_T *col_idx, long m, long n, long nnz, char *out, long out_n)
{
	fflush(stdout);
	fflush(stderr);
	FILE *tmp = tmpfile();
	FILE *devnull = fopen("/dev/null", "w");
	if (!tmp || !devnull) return -1;
	int saved_err = dup(2), saved_out = dup(1);
	dup2(fileno(tmp), 2);
	dup2(fileno(devnull), 1);
	csr_matrix_features_validation_csr_util((char *) "twin", row_ptr, col_idx, m, n, nnz);
	fflush(stdout);
	fflush(stderr);
	dup2(saved_err, 2);
	dup2(saved_out, 1);
	close(saved_err);
	close(saved_out);
	fclose(devnull);
	rewind(tmp);
	long len = (long) fread(out, 1, out_n - 1, tmp);
	out[len < 0 ? 0 : len] = 0;
	fclose(tmp);
	return len;
}

const char *ref_value_type(void) { return (sizeof(ValueType) == 8) ? "double" : "float"; }

/* Thread count of the OpenMP team the reference kernel opens (run.sh:353-355 sets OMP_NUM_THREADS). */
void ref_set_threads(int n) { omp_set_num_threads(n); }

/* One spmm call through the reference plugin.  The plugin object only borrows the arrays here; it is
 * released as a Matrix_Format* exactly like the harness (spmv_bench.cpp:1033), which never runs the plugin
 * destructor (no virtual destructor), so the caller's arrays survive. */
void *ref_create(INT_T *row_ptr, INT_T *col_idx, ValueType *values, long m, long n, long nnz, int k)
{
	return (void *) csr_to_format(row_ptr, col_idx, values, m, n, nnz, k);
}

void ref_run(void *mf, ValueType *x, ValueType *y, int k)
{
	((struct Matrix_Format *) mf)->spmm(x, y, k);
}

void ref_destroy(void *mf)
{
	struct Matrix_Format *MF = (struct Matrix_Format *) mf;
	delete MF;
}

void ref_spmm(INT_T *row_ptr, INT_T *col_idx, ValueType *values, long m, long n, long nnz, ValueType *x,
              ValueType *y, int k)
{
	struct Matrix_Format *MF = csr_to_format(row_ptr, col_idx, values, m, n, nnz, k);
	MF->spmm(x, y, k);
	delete MF;
}

/* Reads a DLMC .smtx file with the reference's smtx_read (dlcm_matrix.c:258-324): row offsets and column indices
 * as stored (the harness copies them without coo_to_csr, spmv_bench.cpp:667-696,769-801).  Its values are
 * time-seeded rand() and are not returned.  Arrays malloc'ed (ref_free). */
int ref_smtx_read(char *path, long *m_out, long *k_out, long *nnz_out, INT_T **row_ptr_out, INT_T **col_idx_out)
{
	struct DLCM_Matrix *MTX = smtx_read(path, 1, 1);
	*m_out = MTX->m;
	*k_out = MTX->k;
	*nnz_out = MTX->nnz;
	*row_ptr_out = (INT_T *) MTX->R;
	*col_idx_out = (INT_T *) MTX->C;
	free(MTX->V);
	return 0;
}

/* Reads a .mtx file the way the harness does.  Returns 0 on success; arrays are malloc'ed (free with
 * ref_free).  values_ref = csr_a_ref (double) as CheckAccuracy sees it. */
int ref_mtx_to_csr(char *path, long *m_out, long *n_out, long *nnz_out, INT_T **row_ptr_out, INT_T **col_idx_out,
                   double **values_out)
{
	struct Matrix_Market *MTX = mtx_read(path, 1, 1);
	long m = MTX->m, k = MTX->k, nnz = MTX->nnz;
	double *mtx_val = (double *) malloc((nnz > 0 ? nnz : 1) * sizeof(double));
	if (!strcmp(MTX->field, "integer")) {
		for (long i = 0; i < nnz; i++) mtx_val[i] = ((int *) MTX->V)[i];
	} else if (!strcmp(MTX->field, "complex")) {
		for (long i = 0; i < nnz; i++) {
#if DOUBLE == 0
			mtx_val[i] = cabsf(((_Complex ValueType *) MTX->V)[i]);
#else
			mtx_val[i] = cabs(((_Complex ValueType *) MTX->V)[i]);
#endif
		}
	} else {
		for (long i = 0; i < nnz; i++) mtx_val[i] = ((ValueType *) MTX->V)[i];
	}
	INT_T *ia = (INT_T *) calloc(m + 1 + VECTOR_ELEM_NUM, sizeof(INT_T));
	INT_T *ja = (INT_T *) calloc(nnz + VECTOR_ELEM_NUM, sizeof(INT_T));
	double *a = (double *) calloc(nnz + VECTOR_ELEM_NUM, sizeof(double));
	coo_to_csr(MTX->R, MTX->C, mtx_val, m, k, nnz, ia, ja, a, 1, 0);
	free(mtx_val);
	*m_out = m; *n_out = k; *nnz_out = nnz;
	*row_ptr_out = ia; *col_idx_out = ja; *values_out = a;
	return 0;
}

void ref_free(void *p) { free(p); }

void ref_partition(INT_T *row_ptr, long m, long nnz, long num_workers, long worker_pos, long *s, long *e)
{
	long ls, le;
	loop_partitioner_balance_prefix_sums(num_workers, worker_pos, row_ptr, m, nnz, &ls, &le);
	*s = ls; *e = le;
}

static double get_d(void *A, long i) { return ((double *) A)[i]; }

/* out: mae, max_ae, mse, mape, smape, lnQ_error, mlare, gmare  (A = gold, F = test, both double) */
void ref_metrics(double *gold, double *test, long N, double *out)
{
	#pragma omp parallel
	{
		double mae, max_ae, mse, mape, smape, lnQ_error, mlare, gmare;
		array_mae_concurrent(gold, test, N, &mae, get_d);
		array_max_ae_concurrent(gold, test, N, &max_ae, get_d);
		array_mse_concurrent(gold, test, N, &mse, get_d);
		array_mape_concurrent(gold, test, N, &mape, get_d);
		array_smape_concurrent(gold, test, N, &smape, get_d);
		array_lnQ_error_concurrent(gold, test, N, &lnQ_error, get_d);
		array_mlare_concurrent(gold, test, N, &mlare, get_d);
		array_gmare_concurrent(gold, test, N, &gmare, get_d);
		#pragma omp single
		{
			out[0] = mae; out[1] = max_ae; out[2] = mse; out[3] = mape;
			out[4] = smape; out[5] = lnQ_error; out[6] = mlare; out[7] = gmare;
		}
	}
}

} /* extern "C" */
