// spmm_kernel_hip.cpp -- the HIP plugin: a Matrix_Format whose spmm() runs on an MI355X through libspmm_hip.so.
//
// Drop-in for the reference plugin benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp (struct CSRArrays,
// :21-66): same factory (csr_to_format), same spmm(x, y, k) semantics (x column-major host B, y row-major host C,
// synchronous, y overwritten), same statistics hooks.  Linked into the harness exactly like the reference links
// one plugin per executable (Makefile_in:52-53): spmm_csr_hip_{d,f}.exe.
//
// Environment:
//   SPMM_HIP_DEVICE              device index (default 0)
//   SPMM_HIP_NGPUS, SPMM_HIP_DEVICES  multi-GPU handle: rows split over NGPUS GPUs (listed, default 0..NGPUS-1)
//   SPMM_HIP_ASSUME_X_UNCHANGED  1 = skip re-uploading B when the same x pointer comes back (see spmm_hip.h)
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "../../include/spmm_hip.h"
#include "matrix_format.h"

namespace {

constexpr int kDtype = (sizeof(ValueType) == 8) ? SPMM_HIP_F64 : SPMM_HIP_F32;

[[noreturn]] void die(const char *what, int st) {
    // the reference's fatal path: error() -> exit(EXIT_FAILURE) (lib/debug.h:117,127)
    fprintf(stderr, "HIP_CSR_MI355X: %s failed: %s (%s)\n", what, spmm_hip_strerror(st), spmm_hip_last_error_detail());
    exit(EXIT_FAILURE);
}

struct HipCSR : Matrix_Format {
    INT_T *ia = nullptr;      // row_ptr  [m+1]
    INT_T *ja = nullptr;      // col_idx  [nnz]
    ValueType *a = nullptr;   // values   [nnz]
    spmm_hip_t *h = nullptr;

    HipCSR(long m_, long n_, long nnz_) : Matrix_Format(m_, n_, nnz_) {}
    ~HipCSR() override {
        spmm_hip_destroy(h);
        free(a);
        free(ia);
        free(ja);
    }

    void spmm(ValueType *x, ValueType *y, INT_T k) override {
        int st = spmm_hip_run(h, x, y, k);
        if (st != SPMM_HIP_OK) die("spmm", st);
    }
    void statistics_start() override { spmm_hip_set_timing(h, 1); }
    int statistics_print_data(char *buf, long buf_n) override {
        int w = spmm_hip_stats(h, buf, buf_n);
        return w < 0 ? 0 : w;
    }
};

}  // namespace

struct Matrix_Format *csr_to_format(INT_T *row_ptr, INT_T *col_ind, ValueType *values, long m, long n, long nnz,
                                    int k) {
    HipCSR *csr = new HipCSR(m, n, nnz);
    csr->format_name = (char *)"HIP_CSR_MI355X";
    csr->ia = row_ptr;
    csr->ja = col_ind;
    csr->a = values;
    const char *dev = getenv("SPMM_HIP_DEVICE");
    const char *ng = getenv("SPMM_HIP_NGPUS");
    const char *devs = getenv("SPMM_HIP_DEVICES");
    int st;
    if (ng && atoi(ng) > 1) {   // multi-GPU handle (SURVEY §8b ngpus); SPMM_HIP_DEVICES=d0,d1,... (repeats allowed)
        const int g = std::min(atoi(ng), 64);
        int32_t dl[64];
        int nd = 0;
        for (const char *p = devs; p && *p && nd < 64;) {
            char *e = nullptr;
            dl[nd++] = (int32_t)strtol(p, &e, 10);
            p = (*e == ',') ? e + 1 : e;
            if (e && *e != ',') break;
        }
        if (devs && nd != g) {
            fprintf(stderr, "HIP_CSR_MI355X: SPMM_HIP_DEVICES lists %d devices, SPMM_HIP_NGPUS=%d\n", nd, g);
            exit(EXIT_FAILURE);
        }
        st = spmm_hip_create_multi(row_ptr, col_ind, values, m, n, nnz, k, kDtype, g, devs ? dl : nullptr, &csr->h);
    } else {
        st = spmm_hip_create(row_ptr, col_ind, values, m, n, nnz, k, kDtype, dev ? atoi(dev) : 0, &csr->h);
    }
    if (st != SPMM_HIP_OK) die("csr_to_format", st);
    int64_t info[SPMM_HIP_INFO_SLOTS];
    spmm_hip_info(csr->h, info);
    csr->mem_footprint = (double)info[7];
    return csr;
}

int statistics_print_labels(char *buf, long buf_n) {
    int w = spmm_hip_stats_labels(buf, buf_n);
    return w < 0 ? 0 : w;
}
