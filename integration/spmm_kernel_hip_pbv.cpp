// integration/spmm_kernel_hip_pbv.cpp -- the reference-side plugin of the perfect-balance format (include/spmm_pbv.h),
// the GPU counterpart of the reference's CUSTOM_VECTOR_PERFECT_NNZ_BALANCE build of its CSR plugin
// (spmv_kernel_csr.cpp:183-184,196-201: format "Custom_CSR_PBV").  Compiled against the REFERENCE's own plugin header
// (spmv_kernel.h:9-30) like integration/spmm_kernel_hip.cpp, and bound to libspmm_pbv.so.
//
// Contract kept: the plugin owns the harness's CSR arrays; spmm(x, y, k) is synchronous with x column-major [k][n]
// and y row-major [m][k] (k SpMVs: the format is a K = 1 format); fatal errors exit(EXIT_FAILURE).  SPMM_HIP_DEVICE
// picks the GPU, SPMM_PBV_ITEMS the items per lane (4, 8 or 16; default 8).
#include <stdlib.h>
#include <stdio.h>
#include "macros/cpp_defines.h"
#include "spmv_bench_common.h"
#include "spmv_kernel.h"
#include "spmm_pbv.h"                       // <engine>/include

struct HipPBV : Matrix_Format
{
	INT_T * ia; INT_T * ja; ValueType * a;
	spmm_pbv_t * h;
	HipPBV(long m, long n, long nnz) : Matrix_Format(m, n, nnz), ia(NULL), ja(NULL), a(NULL), h(NULL) {}
	~HipPBV() { spmm_pbv_destroy(h); free(a); free(ia); free(ja); }
	void spmm(ValueType * x, ValueType * y, INT_T k)
	{
		int st = spmm_pbv_run(h, x, y, k);
		if (st) { fprintf(stderr, "spmm_pbv_run: status %d (%s)\n", st, spmm_pbv_last_error_detail()); exit(EXIT_FAILURE); }
	}
	void statistics_start() {}
	int statistics_print_data(char * buf, long buf_n) { int w = spmm_pbv_stats(h, buf, buf_n); return w < 0 ? 0 : w; }
};

struct Matrix_Format *
csr_to_format(INT_T * row_ptr, INT_T * col_ind, ValueType * values, long m, long n, long nnz, __attribute__((unused)) int k)
{
	struct HipPBV * csr = new HipPBV(m, n, nnz);
	csr->format_name = (char *) "HIP_CSR_PBV_MI355X";
	csr->ia = row_ptr; csr->ja = col_ind; csr->a = values;
	const char * dev = getenv("SPMM_HIP_DEVICE");
	const char * e = getenv("SPMM_PBV_ITEMS");
	const int dt = sizeof(ValueType) == 8 ? SPMM_HIP_F64 : SPMM_HIP_F32;
	int st = spmm_pbv_create(row_ptr, col_ind, values, m, n, nnz, dt, dev ? atoi(dev) : 0, e ? atoi(e) : 0, &csr->h);
	if (st) { fprintf(stderr, "spmm_pbv_create: status %d (%s)\n", st, spmm_pbv_last_error_detail()); exit(EXIT_FAILURE); }
	int64_t info[5]; spmm_pbv_info(csr->h, info, 5); csr->mem_footprint = (double) info[4];
	return csr;
}

int statistics_print_labels(char * buf, long buf_n) { int w = spmm_pbv_stats_labels(buf, buf_n); return w < 0 ? 0 : w; }
