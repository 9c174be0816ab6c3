// integration/sddmm_kernel_hip.cpp -- reference-side plugin for the sparse-attention pipeline bench
// (INTEGRATION.md §4), compiled against the REFERENCE's pipeline plugin header
// (benchmark_code/CPU/AMD/pipeline_code_bench/sddmm_kernel.h:9-31, with sddmm_bench_common.h and
// macros/cpp_defines.h) and bound to the engine's C ABI (include/spmm_hip.h, include/spmm_pipeline.h).
//
// Contract kept (sddmm_bench.cpp:918-937, sddmm_taco_naive.cpp:211-277):
//   csr_to_format(mask row_ptr, col_ind, values, m, nnz, n)       the mask the SDDMM samples (m x m)
//   spmm(type, m, k, n, ia, ja, a, x, y, threads)                  y[m][n] = A x, x row-major [k][n], synchronous;
//                                                                  type 'K' / 'Q' results are what sddmm() reads
//   sddmm(y, threads)                                              y[mask nnz] = SDDMM(mask, Q, K)
//   spmm('final', m, m, n, mask ia, mask ja, y, V, y_final)        the values (y) change every call
// Fatal errors exit(EXIT_FAILURE) like the reference's error() (lib/debug.h:117,127).  SPMM_SDDMM_MODE=1 selects the
// Q K^T SDDMM instead of the reference's row-i-of-K product (spmm_pipeline.h); SPMM_HIP_DEVICE picks the GPU.
#include <stdlib.h>
#include <stdio.h>
#include "macros/cpp_defines.h"
#include "sddmm_bench_common.h"
#include "sddmm_kernel.h"
#include "spmm_hip.h"                       // <engine>/include
#include "spmm_pipeline.h"

static void die(const char * what, int st, const char * detail)
{
	fprintf(stderr, "%s: %s (%s)\n", what, spmm_hip_strerror(st), detail ? detail : "");
	exit(EXIT_FAILURE);
}

struct HipPipe : Matrix_Format
{
	spmm_sddmm_t * sd;
	spmm_hip_t * h[4];                      // 'K', 'Q', 'V', final
	struct Key { const INT_T * ia; const INT_T * ja; INT_T m, k, nnz; } key[4];   // what each handle was built from
	ValueType * K; ValueType * Q; INT_T krows;
	int dev;
	HipPipe(long m, long n, long nnz) : Matrix_Format(m, n, nnz), sd(NULL), K(NULL), Q(NULL), krows(0), dev(0)
	{
		for (int i = 0; i < 4; i++) { h[i] = NULL; key[i] = Key{NULL, NULL, 0, 0, 0}; }
	}
	~HipPipe() { for (int i = 0; i < 4; i++) spmm_hip_destroy(h[i]); spmm_sddmm_destroy(sd); }

	void spmm(char type, INT_T m, INT_T k, INT_T n, INT_T * ia, INT_T * ja, ValueType * a, ValueType * x, ValueType * y,
	          __attribute__((unused)) int num_threads)
	{
		const int s = type == 'K' ? 0 : type == 'Q' ? 1 : type == 'V' ? 2 : 3;
		const int dt = sizeof(ValueType) == 8 ? SPMM_HIP_F64 : SPMM_HIP_F32;
		int st;
		// a handle is reused only for the same pattern (arrays AND sizes: a new matrix allocated at a freed address
		// must not inherit a stale plan); its values are re-uploaded on every call, since the caller may pass new
		// values in the same arrays (the final SpMM always does: the SDDMM output, sddmm_bench.cpp:934-936)
		const Key want = {ia, ja, m, k, ia[m]};
		const Key & have = key[s];
		if (!h[s] || have.ia != want.ia || have.ja != want.ja || have.m != want.m || have.k != want.k ||
		    have.nnz != want.nnz) {
			spmm_hip_destroy(h[s]);
			h[s] = NULL;
			if ((st = spmm_hip_create(ia, ja, a, m, k, ia[m], n, dt, dev, &h[s])))
				die("spmm_hip_create", st, spmm_hip_last_error_detail());
			key[s] = want;
		} else if ((st = spmm_hip_update_values(h[s], a))) {
			die("spmm_hip_update_values", st, spmm_hip_last_error_detail());
		}
		if ((st = spmm_hip_run_rowmajor(h[s], x, y, n)))
			die("spmm_hip_run_rowmajor", st, spmm_hip_last_error_detail());
		if (s == 0) { K = y; krows = m; }
		if (s == 1) Q = y;
	}
	void sddmm(ValueType * y, __attribute__((unused)) int num_threads)
	{
		int st = spmm_sddmm_run(sd, Q, K, krows, y);
		if (st) die("spmm_sddmm_run", st, spmm_sddmm_last_error_detail());
	}
	void statistics_start() {}
	int statistics_print_data(__attribute__((unused)) char * buf, __attribute__((unused)) long buf_n) { return 0; }
};

struct Matrix_Format *
csr_to_format(INT_T * row_ptr, INT_T * col_ind, ValueType * values, long m, long nnz, long n)
{
	struct HipPipe * p = new HipPipe(m, n, nnz);
	p->format_name = (char *) "HIP_SDDMM_PIPELINE_MI355X";
	const char * dev = getenv("SPMM_HIP_DEVICE");
	const char * mode = getenv("SPMM_SDDMM_MODE");
	p->dev = dev ? atoi(dev) : 0;
	int st = spmm_sddmm_create(row_ptr, col_ind, values, m, m, nnz, n, sizeof(ValueType) == 8 ? SPMM_HIP_F64 : SPMM_HIP_F32,
	                           mode ? atoi(mode) : SPMM_SDDMM_REF_ROWDIAG, p->dev, &p->sd);
	if (st) die("spmm_sddmm_create", st, spmm_sddmm_last_error_detail());
	p->mem_footprint = p->csr_mem_footprint;
	return p;
}

int statistics_print_labels(__attribute__((unused)) char * buf, __attribute__((unused)) long buf_n) { return 0; }
