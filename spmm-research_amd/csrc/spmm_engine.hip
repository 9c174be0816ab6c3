// spmm_engine.hip -- C ABI (include/spmm_hip.h) of the MI355X-native CSR SpMM engine.
//
// Replaces the reference plugin surface (benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel.h:9-30):
//   csr_to_format        -> spmm_hip_create   (inspector: validate, copy A to HBM, build the row-block table)
//   Matrix_Format::spmm  -> spmm_hip_run      (host x/y, synchronous) / spmm_hip_run_device (HBM-resident)
//   statistics_*         -> spmm_hip_stats_labels / spmm_hip_stats
// Device kernels: spmm_kernels.hpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/spmm_hip.h"
#include "spmm_kernels.hpp"

using namespace spmm;

namespace {

thread_local std::string g_detail;

int fail(int status, const std::string &what) {
    g_detail = what;
    return status;
}

#define HIPCHK(expr)                                                                                     \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess)                                                                            \
            return fail(SPMM_HIP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));            \
    } while (0)

// Production kernel variant (chosen by tools/tune_kernel.py on MI355X; see DESIGN.md "Kernel tuning").
#ifndef DEF_U
#define DEF_U 16
#endif
#ifndef DEF_CAP
#define DEF_CAP 2048
#endif
#ifndef DEF_NTC
#define DEF_NTC 1
#endif
#ifndef DEF_REMAP
#define DEF_REMAP 0
#endif
#ifndef DEF_IL
#define DEF_IL 1
#endif
#ifndef DEF_BUF
#define DEF_BUF 0
#endif

struct Plan {
    int k = -1;
    int vec = 1;   // values per lane per load (16 B where K allows)
    int g = 1;     // lanes per row group
};

}  // namespace

struct spmm_hip_handle {
    int device = 0;
    int dtype = SPMM_HIP_F64;
    size_t vsize = 8;
    int64_t m = 0, ncols = 0, nnz = 0;

    // A in HBM
    int32_t *d_row_ptr = nullptr;
    int32_t *d_col = nullptr;
    void *d_val = nullptr;

    // inspector output (block capacity = the kernel variant's CAP)
    int cap = 2048;
    int variant[6] = {DEF_U, DEF_CAP, DEF_NTC, DEF_REMAP, DEF_IL, DEF_BUF};
    std::vector<int32_t> h_row_ptr_copy;  // kept only by the tuning build (re-blocking for another CAP)
    int nblk = 0;
    int32_t *d_blk_rows = nullptr;
    int nchunks = 0, nlong = 0;
    int4 *d_chunks = nullptr;
    int4 *d_long_rows = nullptr;
    std::vector<int4> h_chunks;

    // per-k buffers
    Plan plan;
    void *d_b = nullptr;      // row-major B [ncols][k]
    void *d_xcol = nullptr;   // column-major staging for host uploads / device col-major input
    void *d_c = nullptr;      // row-major C [m][k]
    void *d_part = nullptr;   // long-row partials [nchunks][k]
    size_t b_bytes = 0, c_bytes = 0;

    const void *last_x = nullptr;
    hipStream_t stream = nullptr;  // own stream for spmm_hip_run
    hipEvent_t ev[8] = {};
    bool have_times = false, have_transpose = false, have_copies = false;
    int64_t device_bytes = 0;
};

namespace {

int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

Plan make_plan(int k, size_t vsize) {
    Plan p;
    p.k = k;
    const size_t row_bytes = (size_t)k * vsize;
    if (row_bytes % 16 == 0)
        p.vec = (int)(16 / vsize);
    else if (row_bytes % 8 == 0 && vsize <= 8)
        p.vec = (int)(8 / vsize);
    else
        p.vec = 1;
    if (p.vec < 1) p.vec = 1;
    const int need = (k + p.vec - 1) / p.vec;
    p.g = std::min(64, next_pow2(std::max(1, need)));
    return p;
}

template <typename T, int VEC, int G>
void launch_long_path(spmm_hip_t *h, const T *B, T *C, int K, hipStream_t s) {
    if (h->nchunks > 0) {
        spmm_long_chunks_kernel<T, VEC, G>
            <<<h->nchunks, WG, 0, s>>>(h->d_col, (const T *)h->d_val, h->d_chunks, B, (T *)h->d_part, K);
        const int64_t tot = (int64_t)h->nlong * K;
        spmm_long_combine_kernel<T>
            <<<(unsigned)((tot + WG - 1) / WG), WG, 0, s>>>(h->d_long_rows, h->nlong, (const T *)h->d_part, C, K);
    }
}

// 32-bit buffer offsets for the B gather are valid while B fits 4 GiB (else the flat 64-bit path is used).
inline bool buf_ok(const spmm_hip_t *h) { return (uint64_t)h->ncols * (uint64_t)h->plan.k * h->vsize < (1ULL << 32); }

template <typename T, int VEC, int G, int U, int CAP, bool NTC, bool REMAP, int IL, bool BUF>
void launch_rows_v(spmm_hip_t *h, const T *B, T *C, int K, hipStream_t s) {
    if (h->nblk > 0) {
        const uint32_t bb = (uint32_t)std::min<uint64_t>((uint64_t)h->ncols * K * sizeof(T), 0xFFFFFFFFull);
        if (BUF && !buf_ok(h))
            spmm_rows_kernel<T, VEC, G, U, CAP, NTC, REMAP, IL, false><<<h->nblk, WG, 0, s>>>(
                h->d_row_ptr, h->d_col, (const T *)h->d_val, h->d_blk_rows, h->nblk, B, C, K, bb);
        else
            spmm_rows_kernel<T, VEC, G, U, CAP, NTC, REMAP, IL, BUF><<<h->nblk, WG, 0, s>>>(
                h->d_row_ptr, h->d_col, (const T *)h->d_val, h->d_blk_rows, h->nblk, B, C, K, bb);
    }
    launch_long_path<T, VEC, G>(h, B, C, K, s);
}

#ifdef SPMM_TUNING
// Tuning build only: the K=32 fp64 shape (VEC=2, G=16) over a grid of variants, selected at run time.
template <int U, int CAP, bool NTC, bool REMAP, int IL, bool BUF>
bool try_variant(spmm_hip_t *h, const double *B, double *C, int K, hipStream_t s) {
    const int *v = h->variant;
    if (v[0] != U || v[1] != CAP || v[2] != (int)NTC || v[3] != (int)REMAP || v[4] != IL || v[5] != (int)BUF)
        return false;
    launch_rows_v<double, 2, 16, U, CAP, NTC, REMAP, IL, BUF>(h, B, C, K, s);
    return true;
}
#define TV(U, CAP, NTC, REMAP, IL, BUF) try_variant<U, CAP, NTC, REMAP, IL, BUF>(h, B, C, K, s) ||
bool launch_tuned(spmm_hip_t *h, const double *B, double *C, int K, hipStream_t s) {
    return TV(8, 2048, true, false, 1, false) TV(16, 2048, true, false, 1, false) TV(16, 2048, true, false, 1, true)
        TV(24, 2048, true, false, 1, true) TV(16, 1024, true, false, 1, true) TV(16, 2048, false, false, 1, true)
        TV(16, 2048, true, true, 1, true) TV(8, 2048, true, false, 2, true) false;
}
#endif

template <typename T, int VEC, int G>
void launch_rows_t(spmm_hip_t *h, const T *B, T *C, int K, hipStream_t s) {
#ifdef SPMM_TUNING
    if constexpr (std::is_same<T, double>::value && VEC == 2 && G == 16) {
        if (launch_tuned(h, B, C, K, s)) return;
    }
#endif
    launch_rows_v<T, VEC, G, DEF_U, DEF_CAP, (bool)DEF_NTC, (bool)DEF_REMAP, DEF_IL, (bool)DEF_BUF>(h, B, C, K, s);
}

template <typename T, int VEC>
void launch_rows_g(spmm_hip_t *h, const T *B, T *C, int K, hipStream_t s) {
    switch (h->plan.g) {
        case 1: launch_rows_t<T, VEC, 1>(h, B, C, K, s); break;
        case 2: launch_rows_t<T, VEC, 2>(h, B, C, K, s); break;
        case 4: launch_rows_t<T, VEC, 4>(h, B, C, K, s); break;
        case 8: launch_rows_t<T, VEC, 8>(h, B, C, K, s); break;
        case 16: launch_rows_t<T, VEC, 16>(h, B, C, K, s); break;
        case 32: launch_rows_t<T, VEC, 32>(h, B, C, K, s); break;
        default: launch_rows_t<T, VEC, 64>(h, B, C, K, s); break;
    }
}

int launch_spmm(spmm_hip_t *h, const void *B, void *C, int K, hipStream_t s) {
    if (h->dtype == SPMM_HIP_F64) {
        if (h->plan.vec == 2)
            launch_rows_g<double, 2>(h, (const double *)B, (double *)C, K, s);
        else
            launch_rows_g<double, 1>(h, (const double *)B, (double *)C, K, s);
    } else {
        if (h->plan.vec == 4)
            launch_rows_g<float, 4>(h, (const float *)B, (float *)C, K, s);
        else if (h->plan.vec == 2)
            launch_rows_g<float, 2>(h, (const float *)B, (float *)C, K, s);
        else
            launch_rows_g<float, 1>(h, (const float *)B, (float *)C, K, s);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SPMM_HIP_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return SPMM_HIP_OK;
}

int launch_transpose(spmm_hip_t *h, const void *X, void *Bt, int K, hipStream_t s) {
    dim3 grid((unsigned)((h->ncols + 63) / 64), (unsigned)((K + 31) / 32));
    if (h->ncols == 0 || K == 0) return SPMM_HIP_OK;
    if (h->dtype == SPMM_HIP_F64)
        transpose_colmajor_kernel<double><<<grid, WG, 0, s>>>((const double *)X, (double *)Bt, h->ncols, K);
    else
        transpose_colmajor_kernel<float><<<grid, WG, 0, s>>>((const float *)X, (float *)Bt, h->ncols, K);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SPMM_HIP_ERR_HIP, std::string("transpose launch: ") + hipGetErrorString(e));
    return SPMM_HIP_OK;
}

void free_k_buffers(spmm_hip_t *h) {
    if (h->d_b) (void)hipFree(h->d_b);
    if (h->d_xcol) (void)hipFree(h->d_xcol);
    if (h->d_c) (void)hipFree(h->d_c);
    if (h->d_part) (void)hipFree(h->d_part);
    h->d_b = h->d_xcol = h->d_c = h->d_part = nullptr;
    h->b_bytes = h->c_bytes = 0;
    h->plan = Plan();
    h->last_x = nullptr;
}

// Inspector: greedy nnz-balanced row blocks (<= cap nonzeros, <= CAP_ROWS rows; a longer row is a block of
// its own and is cut into CAP_LONG chunks for the long path).
void build_blocks(const int32_t *rp, int64_t m, int cap, std::vector<int32_t> &blk, std::vector<int4> &chunks,
                  std::vector<int4> &long_rows) {
    blk.clear();
    chunks.clear();
    long_rows.clear();
    blk.push_back(0);
    int64_t r = 0;
    while (r < m) {
        const int64_t len = (int64_t)rp[r + 1] - rp[r];
        if (len > cap) {
            if (blk.back() != r) blk.push_back((int32_t)r);
            const int nslot = (int)((len + CAP_LONG - 1) / CAP_LONG);
            long_rows.push_back(make_int4((int)r, (int)chunks.size(), nslot, 0));
            for (int q = 0; q < nslot; ++q) {
                const int a = rp[r] + q * CAP_LONG;
                const int e = (int)std::min<int64_t>((int64_t)a + CAP_LONG, rp[r + 1]);
                chunks.push_back(make_int4((int)r, a, e, (int)chunks.size()));
            }
            blk.push_back((int32_t)(r + 1));
            ++r;
            continue;
        }
        int64_t start = blk.back();
        int64_t nnz_blk = (int64_t)rp[r] - rp[start];
        if (r - start >= CAP_ROWS || nnz_blk + len > cap) {
            blk.push_back((int32_t)r);
            continue;
        }
        ++r;
    }
    if (blk.back() != m) blk.push_back((int32_t)m);
}

}  // namespace

extern "C" {

const char *spmm_hip_version(void) { return "spmm-mi355x 0.1 (gfx950 row-block kernel)"; }

const char *spmm_hip_strerror(int s) {
    switch (s) {
        case SPMM_HIP_OK: return "ok";
        case SPMM_HIP_ERR_ARG: return "invalid argument";
        case SPMM_HIP_ERR_NOMEM: return "out of memory";
        case SPMM_HIP_ERR_HIP: return "HIP runtime error";
        case SPMM_HIP_ERR_NODEVICE: return "no such HIP device";
        case SPMM_HIP_ERR_K: return "k mismatch";
        case SPMM_HIP_ERR_CSR: return "malformed CSR";
        case SPMM_HIP_ERR_OVERFLOW: return "size overflow";
        default: return "unknown status";
    }
}

const char *spmm_hip_last_error_detail(void) { return g_detail.c_str(); }

int spmm_hip_device_count(int *count) {
    if (!count) return fail(SPMM_HIP_ERR_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return SPMM_HIP_OK;
}

double spmm_hip_bytes_alg(int64_t m, int64_t ncols, int64_t nnz, int32_t k, int32_t dtype) {
    const double s = (dtype == SPMM_HIP_F32) ? 4.0 : 8.0;
    return 4.0 * (double)(m + 1) + (4.0 + s) * (double)nnz + s * (double)k * (double)ncols +
           s * (double)k * (double)m;
}

// loop_partitioner_balance_prefix_sums (lib/parallel_util.h:141-165) with binary_search
// (lib/macros/macrolib.h:471-524, default comparator / distance :440-448).
static int64_t bsearch_nearest(const int32_t *A, int64_t lo, int64_t hi, int64_t target) {
    int64_t s = lo, e = hi;
    if (target < A[s]) return s;
    if (target > A[e]) return e;
    for (;;) {
        const int64_t mid = (s + e) / 2;
        if (mid == s || mid == e) break;
        if (target > A[mid])
            s = mid;
        else
            e = mid;
    }
    if (target == A[s]) return s;
    if (target == A[e]) return e;
    const int64_t ds = target - A[s] < 0 ? A[s] - target : target - A[s];
    const int64_t de = target - A[e] < 0 ? A[e] - target : target - A[e];
    return ds < de ? s : e;
}

int spmm_hip_partition_rows(const int32_t *row_ptr, int64_t m, int64_t nnz, int64_t W, int64_t w, int64_t *start,
                            int64_t *end) {
    if (!row_ptr || !start || !end || m < 1 || W < 1 || w < 0 || w >= W)
        return fail(SPMM_HIP_ERR_ARG, "partition: bad arguments");
    const int64_t t0 = (nnz * w) / W, t1 = (nnz * (w + 1)) / W;
    *start = (w == 0) ? 0 : bsearch_nearest(row_ptr, 0, m - 1, t0);
    *end = (w == W - 1) ? m : bsearch_nearest(row_ptr, 0, m - 1, t1);
    return SPMM_HIP_OK;
}

int spmm_hip_create(const int32_t *row_ptr, const int32_t *col_idx, const void *values, int64_t m, int64_t ncols,
                    int64_t nnz, int32_t k, int32_t dtype, int32_t device, spmm_hip_t **out) {
    if (!out) return fail(SPMM_HIP_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (m < 0 || ncols < 0 || nnz < 0 || k < 0) return fail(SPMM_HIP_ERR_ARG, "negative size");
    if (dtype != SPMM_HIP_F64 && dtype != SPMM_HIP_F32) return fail(SPMM_HIP_ERR_ARG, "dtype");
    if (!row_ptr || (nnz > 0 && (!col_idx || !values))) return fail(SPMM_HIP_ERR_ARG, "null CSR array");
    if (m >= INT32_MAX || ncols >= INT32_MAX || nnz >= INT32_MAX)
        return fail(SPMM_HIP_ERR_OVERFLOW, "m, ncols and nnz must fit int32 (reference INT_T = int32_t)");
    // validate the CSR (the reference trusts its input; we refuse malformed input instead of faulting the GPU)
    if (row_ptr[0] != 0 || row_ptr[m] != nnz) return fail(SPMM_HIP_ERR_CSR, "row_ptr[0] != 0 or row_ptr[m] != nnz");
    for (int64_t i = 0; i < m; ++i)
        if (row_ptr[i + 1] < row_ptr[i]) return fail(SPMM_HIP_ERR_CSR, "row_ptr not monotone at row " + std::to_string(i));
    for (int64_t j = 0; j < nnz; ++j)
        if (col_idx[j] < 0 || col_idx[j] >= ncols)
            return fail(SPMM_HIP_ERR_CSR, "col_idx out of range at nonzero " + std::to_string(j));

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SPMM_HIP_ERR_NODEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(SPMM_HIP_ERR_NODEVICE, "device index out of range");
    HIPCHK(hipSetDevice(device));

    spmm_hip_t *h = new spmm_hip_t();
    h->device = device;
    h->dtype = dtype;
    h->vsize = (dtype == SPMM_HIP_F64) ? 8 : 4;
    h->m = m;
    h->ncols = ncols;
    h->nnz = nnz;

    std::vector<int32_t> blk;
    std::vector<int4> long_rows;
    h->cap = DEF_CAP;
    build_blocks(row_ptr, m, h->cap, blk, h->h_chunks, long_rows);
#ifdef SPMM_TUNING
    h->h_row_ptr_copy.assign(row_ptr, row_ptr + m + 1);
#endif
    h->nblk = (int)blk.size() - 1;
    h->nchunks = (int)h->h_chunks.size();
    h->nlong = (int)long_rows.size();

    auto cleanup = [&](int st) {
        spmm_hip_destroy(h);
        return st;
    };
#define HIPCHK_C(expr)                                                                                   \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess) {                                                                          \
            int _s = (_e == hipErrorOutOfMemory) ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP;                 \
            fail(_s, std::string(#expr) + ": " + hipGetErrorString(_e));                                 \
            return cleanup(_s);                                                                          \
        }                                                                                                \
    } while (0)

    // col / val are padded by 64 B: the kernel stages 16-byte vectors from a 16-byte boundary (spmm_rows_kernel)
    const size_t rp_b = (size_t)(m + 1) * 4, col_b = (size_t)std::max<int64_t>(nnz, 1) * 4 + 64,
                 val_b = (size_t)std::max<int64_t>(nnz, 1) * h->vsize + 64, blk_b = blk.size() * 4;
    HIPCHK_C(hipMalloc(&h->d_row_ptr, rp_b));
    HIPCHK_C(hipMalloc(&h->d_col, col_b));
    HIPCHK_C(hipMalloc(&h->d_val, val_b));
    HIPCHK_C(hipMalloc(&h->d_blk_rows, blk_b));
    HIPCHK_C(hipMemcpy(h->d_row_ptr, row_ptr, rp_b, hipMemcpyHostToDevice));
    HIPCHK_C(hipMemset(h->d_col, 0, col_b));
    HIPCHK_C(hipMemset(h->d_val, 0, val_b));
    if (nnz > 0) {
        HIPCHK_C(hipMemcpy(h->d_col, col_idx, (size_t)nnz * 4, hipMemcpyHostToDevice));
        HIPCHK_C(hipMemcpy(h->d_val, values, (size_t)nnz * h->vsize, hipMemcpyHostToDevice));
    }
    HIPCHK_C(hipMemcpy(h->d_blk_rows, blk.data(), blk_b, hipMemcpyHostToDevice));
    h->device_bytes = (int64_t)(rp_b + col_b + val_b + blk_b);
    if (h->nchunks > 0) {
        HIPCHK_C(hipMalloc(&h->d_chunks, h->nchunks * sizeof(int4)));
        HIPCHK_C(hipMalloc(&h->d_long_rows, h->nlong * sizeof(int4)));
        HIPCHK_C(hipMemcpy(h->d_chunks, h->h_chunks.data(), h->nchunks * sizeof(int4), hipMemcpyHostToDevice));
        HIPCHK_C(hipMemcpy(h->d_long_rows, long_rows.data(), h->nlong * sizeof(int4), hipMemcpyHostToDevice));
        h->device_bytes += (int64_t)((h->nchunks + h->nlong) * sizeof(int4));
    }
    HIPCHK_C(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    for (auto &e : h->ev) HIPCHK_C(hipEventCreate(&e));
#undef HIPCHK_C
    if (k > 0) {
        int st = spmm_hip_plan(h, k);
        if (st != SPMM_HIP_OK) return cleanup(st);
    }
    *out = h;
    return SPMM_HIP_OK;
}

int spmm_hip_plan(spmm_hip_t *h, int32_t k) {
    if (!h || k < 1) return fail(SPMM_HIP_ERR_ARG, "plan: bad handle or k < 1");
    if (h->plan.k == k) return SPMM_HIP_OK;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    free_k_buffers(h);
    h->plan = make_plan(k, h->vsize);
    h->b_bytes = (size_t)std::max<int64_t>(h->ncols, 1) * k * h->vsize;
    h->c_bytes = (size_t)std::max<int64_t>(h->m, 1) * k * h->vsize;
    hipError_t e;
    if ((e = hipMalloc(&h->d_b, h->b_bytes)) != hipSuccess ||
        (e = hipMalloc(&h->d_xcol, h->b_bytes)) != hipSuccess || (e = hipMalloc(&h->d_c, h->c_bytes)) != hipSuccess ||
        (h->nchunks > 0 && (e = hipMalloc(&h->d_part, (size_t)h->nchunks * k * h->vsize)) != hipSuccess)) {
        free_k_buffers(h);
        return fail(e == hipErrorOutOfMemory ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP,
                    std::string("plan alloc: ") + hipGetErrorString(e));
    }
    return SPMM_HIP_OK;
}

int spmm_hip_run_device(spmm_hip_t *h, const void *d_b, int32_t b_layout, void *d_c, int32_t k, void *stream) {
    if (!h || !d_b || !d_c || k < 1) return fail(SPMM_HIP_ERR_ARG, "run_device: bad arguments");
    if (b_layout != SPMM_HIP_B_COL_MAJOR && b_layout != SPMM_HIP_B_ROW_MAJOR)
        return fail(SPMM_HIP_ERR_ARG, "run_device: b_layout");
    if (h->plan.k != k) {
        int st = spmm_hip_plan(h, k);
        if (st != SPMM_HIP_OK) return st;
    }
    if (((uintptr_t)d_b | (uintptr_t)d_c) % 16 != 0)
        return fail(SPMM_HIP_ERR_ARG, "run_device: device buffers must be 16-byte aligned");
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const void *B = d_b;
    h->have_transpose = false;
    if (b_layout == SPMM_HIP_B_COL_MAJOR) {
        HIPCHK(hipEventRecord(h->ev[2], s));
        int st = launch_transpose(h, d_b, h->d_b, k, s);
        if (st != SPMM_HIP_OK) return st;
        HIPCHK(hipEventRecord(h->ev[3], s));
        B = h->d_b;
        h->have_transpose = true;
    }
    HIPCHK(hipEventRecord(h->ev[0], s));
    if (h->m > 0) {
        int st = launch_spmm(h, B, d_c, k, s);
        if (st != SPMM_HIP_OK) return st;
    }
    HIPCHK(hipEventRecord(h->ev[1], s));
    h->have_times = true;
    h->have_copies = false;
    return SPMM_HIP_OK;
}

int spmm_hip_run(spmm_hip_t *h, const void *x, void *y, int32_t k) {
    if (!h || k < 1 || (!x && h->ncols > 0) || (!y && h->m > 0)) return fail(SPMM_HIP_ERR_ARG, "run: bad arguments");
    if (h->plan.k != k) {
        int st = spmm_hip_plan(h, k);
        if (st != SPMM_HIP_OK) return st;
    }
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const char *env = getenv("SPMM_HIP_ASSUME_X_UNCHANGED");
    const bool reuse = env && env[0] == '1' && x == h->last_x;
    HIPCHK(hipEventRecord(h->ev[4], s));
    if (!reuse && h->ncols > 0) {
        HIPCHK(hipMemcpyAsync(h->d_xcol, x, (size_t)h->ncols * k * h->vsize, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipEventRecord(h->ev[5], s));
    HIPCHK(hipEventRecord(h->ev[2], s));
    if (!reuse) {
        int st = launch_transpose(h, h->d_xcol, h->d_b, k, s);
        if (st != SPMM_HIP_OK) return st;
    }
    HIPCHK(hipEventRecord(h->ev[3], s));
    HIPCHK(hipEventRecord(h->ev[0], s));
    if (h->m > 0) {
        int st = launch_spmm(h, h->d_b, h->d_c, k, s);
        if (st != SPMM_HIP_OK) return st;
    }
    HIPCHK(hipEventRecord(h->ev[1], s));
    if (h->m > 0) HIPCHK(hipMemcpyAsync(y, h->d_c, (size_t)h->m * k * h->vsize, hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(h->ev[6], s));
    HIPCHK(hipStreamSynchronize(s));
    h->last_x = x;
    h->have_times = h->have_transpose = h->have_copies = true;
    return SPMM_HIP_OK;
}

int spmm_hip_last_times(spmm_hip_t *h, double *out_ms) {
    if (!h || !out_ms) return fail(SPMM_HIP_ERR_ARG, "last_times: bad arguments");
    for (int i = 0; i < 4; ++i) out_ms[i] = 0.0;
    if (!h->have_times) return SPMM_HIP_OK;
    float ms = 0.f;
    HIPCHK(hipEventSynchronize(h->ev[1]));
    HIPCHK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    out_ms[0] = ms;
    if (h->have_transpose) {
        HIPCHK(hipEventElapsedTime(&ms, h->ev[2], h->ev[3]));
        out_ms[1] = ms;
    }
    if (h->have_copies) {
        HIPCHK(hipEventSynchronize(h->ev[6]));
        HIPCHK(hipEventElapsedTime(&ms, h->ev[4], h->ev[5]));
        out_ms[2] = ms;
        HIPCHK(hipEventElapsedTime(&ms, h->ev[1], h->ev[6]));
        out_ms[3] = ms;
    }
    return SPMM_HIP_OK;
}

int spmm_hip_stats_labels(char *buf, long buf_n) {
    if (!buf || buf_n <= 0) return fail(SPMM_HIP_ERR_ARG, "stats_labels: buffer");
    int n = snprintf(buf, (size_t)buf_n,
                     ",kernel_ms,transpose_ms,h2d_ms,d2h_ms,bytes_alg,hbm_gbs_alg,roofline_frac,blocks,long_rows,device");
    return std::min<long>(n, buf_n - 1);
}

int spmm_hip_stats(spmm_hip_t *h, char *buf, long buf_n) {
    if (!h || !buf || buf_n <= 0) return fail(SPMM_HIP_ERR_ARG, "stats: bad arguments");
    double t[4];
    int st = spmm_hip_last_times(h, t);
    if (st != SPMM_HIP_OK) return st;
    const int k = h->plan.k > 0 ? h->plan.k : 0;
    const double bytes = spmm_hip_bytes_alg(h->m, h->ncols, h->nnz, k, h->dtype);
    const double gbs = t[0] > 0 ? bytes / (t[0] * 1e-3) / 1e9 : 0.0;
    int n = snprintf(buf, (size_t)buf_n, ",%.6f,%.6f,%.6f,%.6f,%.0f,%.2f,%.4f,%d,%d,%d", t[0], t[1], t[2], t[3], bytes,
                     gbs, gbs / 8000.0, h->nblk, h->nlong, h->device);
    return std::min<long>(n, buf_n - 1);
}

int spmm_hip_info(const spmm_hip_t *h, int64_t *out) {
    if (!h || !out) return fail(SPMM_HIP_ERR_ARG, "info: bad arguments");
    out[0] = h->m;
    out[1] = h->ncols;
    out[2] = h->nnz;
    out[3] = h->plan.k;
    out[4] = h->dtype;
    out[5] = h->nblk;
    out[6] = h->nchunks;
    out[7] = h->device_bytes + (int64_t)(2 * h->b_bytes + h->c_bytes);
    return SPMM_HIP_OK;
}

int spmm_hip_device_ptrs(spmm_hip_t *h, void **d_b_rowmajor, void **d_c) {
    if (!h || h->plan.k < 1) return fail(SPMM_HIP_ERR_ARG, "device_ptrs: handle not planned");
    if (d_b_rowmajor) *d_b_rowmajor = h->d_b;
    if (d_c) *d_c = h->d_c;
    return SPMM_HIP_OK;
}

int spmm_hip_destroy(spmm_hip_t *h) {
    if (!h) return SPMM_HIP_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    free_k_buffers(h);
    if (h->d_row_ptr) (void)hipFree(h->d_row_ptr);
    if (h->d_col) (void)hipFree(h->d_col);
    if (h->d_val) (void)hipFree(h->d_val);
    if (h->d_blk_rows) (void)hipFree(h->d_blk_rows);
    if (h->d_chunks) (void)hipFree(h->d_chunks);
    if (h->d_long_rows) (void)hipFree(h->d_long_rows);
    for (auto &e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SPMM_HIP_OK;
}

#ifdef SPMM_TUNING
// Tuning build only (lib/libspmm_hip_tune.so, tools/tune_kernel.py): pick the K=32 fp64 row-kernel variant and
// rebuild the row-block table for its capacity.
int spmm_hip_tune_select(spmm_hip_t *h, int u, int cap, int ntc, int remap, int il, int buf) {
    if (!h || h->h_row_ptr_copy.empty()) return fail(SPMM_HIP_ERR_ARG, "tune_select: bad handle");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    std::vector<int32_t> blk;
    std::vector<int4> long_rows;
    build_blocks(h->h_row_ptr_copy.data(), h->m, cap, blk, h->h_chunks, long_rows);
    if (h->d_blk_rows) (void)hipFree(h->d_blk_rows);
    if (h->d_chunks) (void)hipFree(h->d_chunks);
    if (h->d_long_rows) (void)hipFree(h->d_long_rows);
    h->d_blk_rows = nullptr;
    h->d_chunks = nullptr;
    h->d_long_rows = nullptr;
    h->nblk = (int)blk.size() - 1;
    h->nchunks = (int)h->h_chunks.size();
    h->nlong = (int)long_rows.size();
    HIPCHK(hipMalloc(&h->d_blk_rows, blk.size() * 4));
    HIPCHK(hipMemcpy(h->d_blk_rows, blk.data(), blk.size() * 4, hipMemcpyHostToDevice));
    if (h->nchunks > 0) {
        HIPCHK(hipMalloc(&h->d_chunks, h->nchunks * sizeof(int4)));
        HIPCHK(hipMalloc(&h->d_long_rows, h->nlong * sizeof(int4)));
        HIPCHK(hipMemcpy(h->d_chunks, h->h_chunks.data(), h->nchunks * sizeof(int4), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(h->d_long_rows, long_rows.data(), h->nlong * sizeof(int4), hipMemcpyHostToDevice));
        if (h->plan.k > 0) {
            if (h->d_part) (void)hipFree(h->d_part);
            HIPCHK(hipMalloc(&h->d_part, (size_t)h->nchunks * h->plan.k * h->vsize));
        }
    }
    h->cap = cap;
    h->variant[0] = u;
    h->variant[1] = cap;
    h->variant[2] = ntc;
    h->variant[3] = remap;
    h->variant[4] = il;
    h->variant[5] = buf;
    return SPMM_HIP_OK;
}
#endif

}  // extern "C"
