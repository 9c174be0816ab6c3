// matrix_format.h -- the plugin interface the harness drives, mirroring the reference's
// benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel.h:9-30 (same member names and call signatures, so a kernel
// plugin written against the reference compiles against this and vice versa).
//
// Differences from the reference, both deliberate:
//   * the destructor is virtual (the reference's `delete MF` at spmv_bench.cpp:1033 never runs the plugin's
//     destructor because the base has none);
//   * INT_T / ValueType default to int32_t / double and are overridable with -D, as in spmv_bench_common.h:10-16.
#pragma once
#include <stdint.h>

#ifndef INT_T
#define INT_T int32_t
#endif
#ifndef ValueType
#define ValueType double
#endif

struct Matrix_Format {
    char *format_name;         // e.g. "HIP_CSR_MI355X"
    INT_T m;                   // rows of A
    INT_T n;                   // columns of A (= rows of B)
    INT_T nnz;                 // nonzeros of A
    double mem_footprint;      // bytes the format holds (device side for the HIP plugin)
    double csr_mem_footprint;  // bytes of the plain CSR: nnz*(sizeof(ValueType)+sizeof(INT_T)) + (m+1)*sizeof(INT_T)

    Matrix_Format(long m_, long n_, long nnz_) : format_name(nullptr), m((INT_T)m_), n((INT_T)n_), nnz((INT_T)nnz_) {
        mem_footprint = 0;
        csr_mem_footprint = (double)nnz_ * (sizeof(ValueType) + sizeof(INT_T)) + (double)(m_ + 1) * sizeof(INT_T);
    }
    virtual ~Matrix_Format() {}

    // C = A * B: x = B column-major [k][n] (x[c*n + col]), y = C row-major [m][k] (y[i*k + c]), overwritten.
    virtual void spmm(ValueType *x, ValueType *y, INT_T k) = 0;
    virtual void statistics_start() = 0;
    virtual int statistics_print_data(char *buf, long buf_n) = 0;
};

// Factory: the harness hands over its CSR arrays; the plugin owns them afterwards (spmm_kernel_csr.cpp:34-39).
struct Matrix_Format *csr_to_format(INT_T *row_ptr, INT_T *col_ind, ValueType *values, long m, long n, long nnz,
                                    int k = 0);
int statistics_print_labels(char *buf, long buf_n);
