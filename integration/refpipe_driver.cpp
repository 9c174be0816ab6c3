// integration/refpipe_driver.cpp -- drives integration/sddmm_kernel_hip.cpp exactly like the reference pipeline
// bench's compute() step (sddmm_bench.cpp:918-937: spmm K, Q, V; sddmm; spmm 'final') through the reference's
// Matrix_Format (sddmm_kernel.h).  Test harness: reads the inputs from a raw file written by
// tests/test_gpu_pipeline.py and writes K, Q, V, y, y_final back (ValueType, row-major).
//   input : n (int64); for W_K, W_Q, W_V, mask: m, k, nnz (int64), row_ptr[m+1], col[nnz] (int32), val[nnz];
//           x [k][n] (ValueType)
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "macros/cpp_defines.h"
#include "sddmm_bench_common.h"
#include "sddmm_kernel.h"

struct Mat { int64_t m, k, nnz; INT_T * rp; INT_T * ci; ValueType * v; };

static void rd(FILE * f, void * p, size_t b) { if (fread(p, 1, b, f) != b) { fprintf(stderr, "short read\n"); exit(1); } }

static Mat read_mat(FILE * f)
{
	Mat a;
	rd(f, &a.m, 8); rd(f, &a.k, 8); rd(f, &a.nnz, 8);
	a.rp = (INT_T *) malloc((a.m + 1) * sizeof(INT_T)); a.ci = (INT_T *) malloc((a.nnz + 1) * sizeof(INT_T));
	a.v = (ValueType *) malloc((a.nnz + 1) * sizeof(ValueType));
	rd(f, a.rp, (a.m + 1) * sizeof(INT_T)); rd(f, a.ci, a.nnz * sizeof(INT_T)); rd(f, a.v, a.nnz * sizeof(ValueType));
	return a;
}

int main(int argc, char ** argv)
{
	if (argc != 3) { fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 2; }
	FILE * f = fopen(argv[1], "rb");
	if (!f) { perror("in"); return 2; }
	int64_t n;
	rd(f, &n, 8);
	Mat W[3], M;
	for (int i = 0; i < 3; i++) W[i] = read_mat(f);
	M = read_mat(f);
	ValueType * x = (ValueType *) malloc(W[0].k * n * sizeof(ValueType));
	rd(f, x, W[0].k * n * sizeof(ValueType));
	fclose(f);
	ValueType * out[3];
	for (int i = 0; i < 3; i++) out[i] = (ValueType *) calloc(W[i].m * n, sizeof(ValueType));
	ValueType * y = (ValueType *) calloc(M.nnz + 1, sizeof(ValueType));
	ValueType * yf = (ValueType *) calloc(M.m * n, sizeof(ValueType));
	struct Matrix_Format * MF = csr_to_format(M.rp, M.ci, M.v, M.m, M.nnz, n);
	const char types[3] = {'K', 'Q', 'V'};
	for (int it = 0; it < 2; it++) {                          // twice: the second call reuses the cached handles
		for (int i = 0; i < 3; i++)
			MF->spmm(types[i], W[i].m, W[i].k, n, W[i].rp, W[i].ci, W[i].v, x, out[i], 1);
		MF->sddmm(y, 1);
		MF->spmm((char) 'l', M.m, M.m, n, M.rp, M.ci, y, out[2], yf, 1);   // the reference passes 'final'
	}
	f = fopen(argv[2], "wb");
	for (int i = 0; i < 3; i++) fwrite(out[i], sizeof(ValueType), W[i].m * n, f);
	fwrite(y, sizeof(ValueType), M.nnz, f);
	fwrite(yf, sizeof(ValueType), M.m * n, f);
	fclose(f);
	printf("%s: ok\n", MF->format_name);
	return 0;
}
