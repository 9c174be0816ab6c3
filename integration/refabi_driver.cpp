// integration/refabi_driver.cpp -- drives the reference-ABI plugin (integration/spmm_kernel_hip.cpp, compiled
// against the reference's spmv_kernel.h) the way the reference harness does (spmv_bench.cpp:996 factory,
// :318,372 spmm calls, :351,442,475 statistics): .mtx -> CSR (engine host reader, libspmm_host) -> csr_to_format ->
// MF->spmm(x, y, K) with x = drand48(seed 42) column-major -> y written raw to <out>.
//   usage: refabi_driver <file.mtx> <K> <out.bin>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "macros/cpp_defines.h"
#include "spmv_bench_common.h"
#include "spmv_kernel.h"
#include "spmm_host.h"

int main(int argc, char **argv)
{
	if (argc != 4) { fprintf(stderr, "usage: %s file.mtx K out.bin\n", argv[0]); return 2; }
	const int K = atoi(argv[2]);
	spmm_csr_t A; char field[32]; int32_t sym = 0;
	if (spmm_host_mtx_read(argv[1], &A, field, sizeof(field), &sym)) { fprintf(stderr, "cannot read %s\n", argv[1]); return 1; }
	// the harness hands over aligned copies it no longer frees (the plugin owns them: spmm_kernel_csr.cpp:34-39)
	INT_T *ia = (INT_T *) malloc((A.m + 1) * sizeof(INT_T));
	INT_T *ja = (INT_T *) malloc((A.nnz + 1) * sizeof(INT_T));
	ValueType *a = (ValueType *) malloc((A.nnz + 1) * sizeof(ValueType));
	memcpy(ia, A.row_ptr, (A.m + 1) * sizeof(INT_T));
	memcpy(ja, A.col_idx, A.nnz * sizeof(INT_T));
	for (long j = 0; j < A.nnz; j++) a[j] = (ValueType) A.values[j];
	double *xd = (double *) malloc((A.ncols * K + 1) * sizeof(double));
	spmm_host_drand48_fill(42, xd, A.ncols * K);
	ValueType *x = (ValueType *) malloc((A.ncols * K + 1) * sizeof(ValueType));
	for (long i = 0; i < A.ncols * K; i++) x[i] = (ValueType) xd[i];
	ValueType *y = (ValueType *) calloc(A.m * K + 1, sizeof(ValueType));

	struct Matrix_Format *MF = csr_to_format(ia, ja, a, A.m, A.ncols, A.nnz, K);
	MF->statistics_start();
	MF->spmm(x, y, K);
	char lab[4096], dat[4096];
	int wl = statistics_print_labels(lab, sizeof(lab)), wd = MF->statistics_print_data(dat, sizeof(dat));
	printf("format_name=%s m=%d n=%d nnz=%d csr_mem_footprint=%.0f mem_footprint=%.0f\n", MF->format_name, MF->m,
	       MF->n, MF->nnz, MF->csr_mem_footprint, MF->mem_footprint);
	printf("labels%.*s\nstats%.*s\n", wl, lab, wd, dat);
	FILE *f = fopen(argv[3], "wb");
	fwrite(y, sizeof(ValueType), A.m * K, f);
	fclose(f);
	spmm_host_csr_free(&A);
	return 0;
}
