// integration/spmm_kernel_hip.cpp -- the reference-side plugin of INTEGRATION.md §1, as a compilable file.
//
// A maintainer drops this next to benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp; it compiles against
// the REFERENCE's own plugin header (spmv_kernel.h:9-30, with spmv_bench_common.h and macros/cpp_defines.h from
// its lib/) and binds the engine's C ABI (include/spmm_hip.h).  integration/Makefile builds it exactly that way
// against /root/reference (tests/test_integration.py); nothing of the reference is copied here.
//
// Reference contract kept: csr_to_format takes the harness's CSR arrays and the plugin owns them afterwards
// (spmm_kernel_csr.cpp:34-39); spmm(x, y, k) is synchronous with x column-major [k][n] and y row-major [m][k]
// (spmm_kernel_csr.cpp:51-54,88,93); fatal errors exit(EXIT_FAILURE) like lib/debug.h:117,127.  SPMM_HIP_NGPUS /
// SPMM_HIP_DEVICES make the handle multi-GPU (SURVEY §8b ngpus; include/spmm_hip.h spmm_hip_create_multi).
#include <stdlib.h>
#include <stdio.h>
#include "macros/cpp_defines.h"
#include "spmv_bench_common.h"
#include "spmv_kernel.h"
#include "spmm_hip.h"                       // <engine>/include

struct HipCSR : Matrix_Format
{
	INT_T * ia; INT_T * ja; ValueType * a;
	spmm_hip_t * h;
	HipCSR(long m, long n, long nnz) : Matrix_Format(m, n, nnz), ia(NULL), ja(NULL), a(NULL), h(NULL) {}
	~HipCSR() { spmm_hip_destroy(h); free(a); free(ia); free(ja); }   // not run by `delete MF` (no virtual dtor)
	void spmm(ValueType * x, ValueType * y, INT_T k)
	{
		int st = spmm_hip_run(h, x, y, k);      // x: column-major [k][n], y: row-major [m][k], synchronous
		if (st) { fprintf(stderr, "spmm_hip_run: %s (%s)\n", spmm_hip_strerror(st), spmm_hip_last_error_detail()); exit(EXIT_FAILURE); }
	}
	void statistics_start() { spmm_hip_set_timing(h, 1); }
	int statistics_print_data(char * buf, long buf_n) { int w = spmm_hip_stats(h, buf, buf_n); return w < 0 ? 0 : w; }
};

struct Matrix_Format *
csr_to_format(INT_T * row_ptr, INT_T * col_ind, ValueType * values, long m, long n, long nnz, int k)
{
	struct HipCSR * csr = new HipCSR(m, n, nnz);
	csr->format_name = (char *) "HIP_CSR_MI355X";
	csr->ia = row_ptr; csr->ja = col_ind; csr->a = values;
	// SPMM_HIP_NGPUS=<g> (SURVEY §8b ngpus): one multi-GPU handle, rows split over g GPUs by the reference
	// partitioner; SPMM_HIP_DEVICES=<d0,d1,...> names them (default 0..g-1; repeats allowed, e.g. 0,0,0,0 runs
	// every shard on one GPU); otherwise one GPU, SPMM_HIP_DEVICE (default 0)
	const char * dev = getenv("SPMM_HIP_DEVICE");
	const char * ng = getenv("SPMM_HIP_NGPUS");
	const char * devs = getenv("SPMM_HIP_DEVICES");
	const int dt = sizeof(ValueType) == 8 ? SPMM_HIP_F64 : SPMM_HIP_F32;
	int st;
	if (ng && atoi(ng) > 1) {
		int32_t dl[64]; int nd = 0;
		for (const char * p = devs; p && *p && nd < 64; ) { dl[nd++] = (int32_t) strtol(p, (char **) &p, 10); if (*p == ',') p++; else break; }
		const int g = atoi(ng) < 64 ? atoi(ng) : 64;
		if (devs && nd != g) { fprintf(stderr, "SPMM_HIP_DEVICES lists %d devices, SPMM_HIP_NGPUS=%d\n", nd, g); exit(EXIT_FAILURE); }
		st = spmm_hip_create_multi(row_ptr, col_ind, values, m, n, nnz, k, dt, g, devs ? dl : NULL, &csr->h);
	} else {
		st = spmm_hip_create(row_ptr, col_ind, values, m, n, nnz, k, dt, dev ? atoi(dev) : 0, &csr->h);
	}
	if (st) { fprintf(stderr, "spmm_hip_create: %s (%s)\n", spmm_hip_strerror(st), spmm_hip_last_error_detail()); exit(EXIT_FAILURE); }
	int64_t info[SPMM_HIP_INFO_SLOTS]; spmm_hip_info(csr->h, info); csr->mem_footprint = (double) info[7];
	return csr;
}

int statistics_print_labels(char * buf, long buf_n) { int w = spmm_hip_stats_labels(buf, buf_n); return w < 0 ? 0 : w; }
