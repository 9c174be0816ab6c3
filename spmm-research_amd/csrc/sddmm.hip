// sddmm.hip -- gfx950 SDDMM (+ optional softmax) of the sparse-attention pipeline consumer.
//
// Reference: benchmark_code/CPU/AMD/pipeline_code_bench/, the plugin surface Matrix_Format::sddmm(y, threads)
// (sddmm_kernel.h:19-20) as implemented by CSRTensors::sddmm -> compute_csr -> compute2 (sddmm_taco_naive.cpp:98-140,
// 211-217, 280-290), driven by compute() (sddmm_bench.cpp:918-937):
//     K = W_K x, Q = W_Q x, V = W_V x        (SpMM, the engine)
//     y = SDDMM(mask, Q, K)                   (this file)
//     y_final = mask(y) V                     (SpMM with the SDDMM output as values, the engine)
// The reference's compute2 sums, for a mask nonzero p in row i, Q[i][n] * K[i][n] over n -- row i of K, not row
// j = col(p) (it computes pD2 = kA*D2_size + nD and never uses it); its own CheckAccuracy gold does the same
// (sddmm_bench.cpp:260-276).  SPMM_SDDMM_REF_ROWDIAG restates exactly that (the drop-in default, bit-identical:
// one fused multiply-add chain over n in order from 0, then one multiply by the mask value, like the reference built
// with its -O3 -march flags); SPMM_SDDMM_QKT is the attention SDDMM the pipeline is meant to compute,
// y[p] = a[p] * sum_n Q[i][n] K[j][n], same chain order.  SPMM_SDDMM_SOFTMAX applies the reference's softmax()
// (sddmm_taco_naive.cpp:191-209: one global max, exp, sum, divide over all nonzeros; commented out at :215 and in
// the gold, sddmm_bench.cpp:279) with fixed-tree reductions (deterministic, not the reference's serial sum order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/spmm_hip.h"
#include "../../include/spmm_pipeline.h"
#include "spmm_kernels.hpp"

using namespace spmm;

struct spmm_sddmm {
    int device = 0, dtype = SPMM_HIP_F64, flags = 0;
    size_t vsize = 8;
    int64_t m = 0, ncols = 0, nnz = 0;
    int32_t n = 0;
    int32_t *d_rp = nullptr, *d_ci = nullptr, *d_prow = nullptr;
    void *d_a = nullptr;           // mask values
    void *d_s = nullptr;           // ROWDIAG: per-row chain results [m]
    void *d_kt = nullptr;          // QKT: K transposed [n][ncols]
    void *d_red = nullptr;         // softmax: block partials + the two scalars
    int nred = 0;
    // host path staging
    void *d_q = nullptr, *d_k = nullptr, *d_y = nullptr;
    int64_t krows_alloc = 0;
    hipStream_t stream = nullptr;
};

namespace {

thread_local std::string g_sd_detail;

int sfail(int st, const std::string &w) {
    g_sd_detail = w;
    return st;
}

#define SDCHK(expr)                                                                                       \
    do {                                                                                                  \
        hipError_t _e = (expr);                                                                           \
        if (_e != hipSuccess)                                                                             \
            return sfail(_e == hipErrorOutOfMemory ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP,                \
                         std::string(#expr) + ": " + hipGetErrorString(_e));                              \
    } while (0)

__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// ROWDIAG: s[i] = fma chain over t of Q[i][t] * K[i][t] from 0 (compute2's inner loop for any nonzero of row i).
// One lane per row keeps the chain serial (bit-identical).  A one-wave workgroup owns RD_ROWS consecutive rows: the
// wave first stages their Q and K rows (up to RD_T elements at a time) in LDS by LDS-DMA -- every instruction moves
// 256 consecutive bytes of one row, all in flight before one wait -- then lanes 0..RD_ROWS-1 run their chains from LDS
// (row pitch RD_T+1: conflict-free).  Few rows per workgroup spread the m chains over many CUs.  The direct form,
// lane i reading Q[i][t] from HBM, touched 64 lines per load instruction (124 us at m = n = 512; this form, DESIGN
// §6.10).
constexpr int RD_ROWS = 16, RD_T = 512, RD_WG = 64;
template <typename T>
__global__ __launch_bounds__(RD_WG) void rowdiag_chain_kernel(const T *__restrict__ Q, const T *__restrict__ K,
                                                              T *__restrict__ s, int64_t m, int n) {
    __shared__ T sq[RD_ROWS][RD_T + 1], sk[RD_ROWS][RD_T + 1];
    const int l = threadIdx.x;
    const int64_t i0 = (int64_t)blockIdx.x * RD_ROWS;
    const int rows = (int)std::min<int64_t>(RD_ROWS, m - i0);
    T acc = T(0);
    typedef __attribute__((address_space(3))) void lds_void;
    for (int t0 = 0; t0 < n; t0 += RD_T) {
        const int tn = std::min(RD_T, n - t0);
        const int dw = tn * (int)sizeof(T) / 4;               // dwords of one row piece
        // LDS-DMA, 64 dwords (one 256-B row segment) per instruction, all issued before the one wait
        for (int r = 0; r < rows; ++r) {
            const char *q = reinterpret_cast<const char *>(Q + (i0 + r) * n + t0);
            const char *k = reinterpret_cast<const char *>(K + (i0 + r) * n + t0);
            for (int c = 0; c < dw; c += RD_WG)
                if (c + l < dw) {
                    __builtin_amdgcn_global_load_lds((const void *)(q + (c + l) * 4),
                                                     (lds_void *)(reinterpret_cast<char *>(&sq[r][0]) + c * 4), 4, 0, 0);
                    __builtin_amdgcn_global_load_lds((const void *)(k + (c + l) * 4),
                                                     (lds_void *)(reinterpret_cast<char *>(&sk[r][0]) + c * 4), 4, 0, 0);
                }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (l < rows) {
#pragma unroll 8
            for (int t = 0; t < tn; ++t) acc = fma_t(sq[l][t], sk[l][t], acc);
        }
        __syncthreads();
    }
    if (l < rows) s[i0 + l] = acc;
}

// y[p] = s[row(p)] * a[p]  (compute2's `B[pA2] *= A_vals[pA2]` after the chain)
template <typename T>
__global__ __launch_bounds__(WG) void rowdiag_scale_kernel(const T *__restrict__ s, const int32_t *__restrict__ prow,
                                                           const T *__restrict__ a, T *__restrict__ y, int64_t nnz) {
    const int64_t p = (int64_t)blockIdx.x * WG + threadIdx.x;
    if (p < nnz) y[p] = s[prow[p]] * a[p];
}

// QKT: y[p] = (fma chain over t of Q[i][t] * K[j][t]) * a[p], K read transposed (KT[t][j]: the lanes of a row's
// consecutive nonzeros gather from one row of KT; Q[i][t] is one broadcast address per row).
template <typename T>
__global__ __launch_bounds__(WG) void qkt_kernel(const T *__restrict__ Q, const T *__restrict__ KT,
                                                 const int32_t *__restrict__ prow, const int32_t *__restrict__ ci,
                                                 const T *__restrict__ a, T *__restrict__ y, int64_t nnz, int64_t ncols,
                                                 int n) {
    const int64_t p = (int64_t)blockIdx.x * WG + threadIdx.x;
    if (p >= nnz) return;
    const T *q = Q + (int64_t)prow[p] * n;
    const T *kt = KT + ci[p];
    T acc = T(0);
    for (int t = 0; t < n; ++t) acc = fma_t(q[t], kt[(int64_t)t * ncols], acc);
    y[p] = acc * a[p];
}

// ---- softmax over all nonzeros (reference softmax(), sddmm_taco_naive.cpp:191-209), fixed reduction trees
template <typename T, bool MAX>
__device__ __forceinline__ T block_reduce(T v, T *red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int w = WG / 2; w >= 1; w /= 2) {
        if ((int)threadIdx.x < w) {
            const T o = red[threadIdx.x + w];
            red[threadIdx.x] = MAX ? (o > red[threadIdx.x] ? o : red[threadIdx.x]) : red[threadIdx.x] + o;
        }
        __syncthreads();
    }
    return red[0];
}

// pass 1 (MAX): part[b] = max of block b's stride; pass 2 (!MAX): y = exp(y - max), part[b] = block sum
template <typename T, bool MAX>
__global__ __launch_bounds__(WG) void softmax_pass_kernel(T *__restrict__ y, int64_t nnz, T *__restrict__ part,
                                                          const T *__restrict__ mx) {
    __shared__ T red[WG];
    const int64_t stride = (int64_t)gridDim.x * WG;
    T v = MAX ? -INFINITY : T(0);
    const T m = MAX ? T(0) : *mx;
    for (int64_t p = (int64_t)blockIdx.x * WG + threadIdx.x; p < nnz; p += stride) {
        if (MAX) {
            v = y[p] > v ? y[p] : v;
        } else {
            const T e = (T)exp((double)(y[p] - m));
            y[p] = e;
            v += e;
        }
    }
    v = block_reduce<T, MAX>(v, red);
    if (threadIdx.x == 0) part[blockIdx.x] = v;
}

// one block folds the partials into out[0] (fixed tree)
template <typename T, bool MAX>
__global__ __launch_bounds__(WG) void softmax_fold_kernel(const T *__restrict__ part, int np, T *__restrict__ out) {
    __shared__ T red[WG];
    T v = MAX ? -INFINITY : T(0);
    for (int b = threadIdx.x; b < np; b += WG) v = MAX ? (part[b] > v ? part[b] : v) : v + part[b];
    v = block_reduce<T, MAX>(v, red);
    if (threadIdx.x == 0) out[0] = v;
}

template <typename T>
__global__ __launch_bounds__(WG) void softmax_div_kernel(T *__restrict__ y, int64_t nnz, const T *__restrict__ sum) {
    const int64_t p = (int64_t)blockIdx.x * WG + threadIdx.x;
    if (p < nnz) y[p] = y[p] / sum[0];
}

template <typename T>
int run_t(spmm_sddmm_t *s, const T *Q, const T *K, T *y, hipStream_t st) {
    const int64_t m = s->m, nnz = s->nnz;
    if (nnz == 0) return SPMM_HIP_OK;
    const unsigned gp = (unsigned)((nnz + WG - 1) / WG);
    if ((s->flags & 1) == SPMM_SDDMM_REF_ROWDIAG) {
        rowdiag_chain_kernel<T><<<(unsigned)((m + RD_ROWS - 1) / RD_ROWS), RD_WG, 0, st>>>(Q, K, (T *)s->d_s, m, s->n);
        rowdiag_scale_kernel<T><<<gp, WG, 0, st>>>((const T *)s->d_s, s->d_prow, (const T *)s->d_a, y, nnz);
    } else {
        // K [ncols][n] -> KT [n][ncols]: the engine's tile transpose (it maps X[r*ncols + c] -> Bt[c*R + r])
        dim3 grid((unsigned)((s->n + 63) / 64), (unsigned)((s->ncols + 31) / 32));
        transpose_colmajor_kernel<T><<<grid, WG, 0, st>>>(K, (T *)s->d_kt, s->n, (int)s->ncols);
        qkt_kernel<T><<<gp, WG, 0, st>>>(Q, (const T *)s->d_kt, s->d_prow, s->d_ci, (const T *)s->d_a, y, nnz,
                                         s->ncols, s->n);
    }
    if (s->flags & SPMM_SDDMM_SOFTMAX) {
        T *part = (T *)s->d_red, *mx = part + s->nred, *sum = mx + 1;
        softmax_pass_kernel<T, true><<<s->nred, WG, 0, st>>>(y, nnz, part, nullptr);
        softmax_fold_kernel<T, true><<<1, WG, 0, st>>>(part, s->nred, mx);
        softmax_pass_kernel<T, false><<<s->nred, WG, 0, st>>>(y, nnz, part, mx);
        softmax_fold_kernel<T, false><<<1, WG, 0, st>>>(part, s->nred, sum);
        softmax_div_kernel<T><<<gp, WG, 0, st>>>(y, nnz, sum);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SPMM_HIP_OK : sfail(SPMM_HIP_ERR_HIP, std::string("sddmm launch: ") + hipGetErrorString(e));
}

}  // namespace

extern "C" {

const char *spmm_sddmm_last_error_detail(void) { return g_sd_detail.c_str(); }

int spmm_sddmm_create(const int32_t *row_ptr, const int32_t *col_idx, const void *mask_vals, int64_t m, int64_t ncols,
                      int64_t nnz, int32_t n, int32_t dtype, int32_t flags, int32_t device, spmm_sddmm_t **out) {
    if (!out) return sfail(SPMM_HIP_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (m < 0 || ncols < 0 || nnz < 0 || n < 1 || (dtype != SPMM_HIP_F64 && dtype != SPMM_HIP_F32) || flags < 0 ||
        flags > 3 || !row_ptr || (nnz > 0 && (!col_idx || !mask_vals)))
        return sfail(SPMM_HIP_ERR_ARG, "sddmm_create: bad arguments");
    if (m >= INT32_MAX || ncols >= INT32_MAX || nnz >= INT32_MAX) return sfail(SPMM_HIP_ERR_OVERFLOW, "sizes");
    if (row_ptr[0] != 0 || row_ptr[m] != nnz) return sfail(SPMM_HIP_ERR_CSR, "row_ptr[0] != 0 or row_ptr[m] != nnz");
    std::vector<int32_t> prow((size_t)nnz);
    for (int64_t i = 0; i < m; ++i) {
        if (row_ptr[i + 1] < row_ptr[i]) return sfail(SPMM_HIP_ERR_CSR, "row_ptr not monotone");
        for (int32_t j = row_ptr[i]; j < row_ptr[i + 1]; ++j) prow[(size_t)j] = (int32_t)i;
    }
    for (int64_t j = 0; j < nnz; ++j)
        if (col_idx[j] < 0 || col_idx[j] >= ncols) return sfail(SPMM_HIP_ERR_CSR, "col_idx out of range");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return sfail(SPMM_HIP_ERR_NODEVICE, "no such HIP device");
    SDCHK(hipSetDevice(device));
    spmm_sddmm_t *s = new spmm_sddmm_t();
    s->device = device;
    s->dtype = dtype;
    s->flags = flags;
    s->vsize = dtype == SPMM_HIP_F64 ? 8 : 4;
    s->m = m;
    s->ncols = ncols;
    s->nnz = nnz;
    s->n = n;
    s->nred = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (nnz + WG * 8 - 1) / (WG * 8)));
    auto bail = [&](hipError_t e, const char *what) {
        spmm_sddmm_destroy(s);
        return sfail(e == hipErrorOutOfMemory ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP,
                     std::string(what) + ": " + hipGetErrorString(e));
    };
    auto up = [&](void **d, const void *h, size_t b) {
        hipError_t e = hipMalloc(d, std::max<size_t>(b, 16));
        if (e == hipSuccess && b) e = hipMemcpy(*d, h, b, hipMemcpyHostToDevice);
        return e;
    };
    hipError_t e = up((void **)&s->d_rp, row_ptr, (size_t)(m + 1) * 4);
    if (e == hipSuccess) e = up((void **)&s->d_ci, col_idx, (size_t)nnz * 4);
    if (e == hipSuccess) e = up((void **)&s->d_prow, prow.data(), (size_t)nnz * 4);
    if (e == hipSuccess) e = up(&s->d_a, mask_vals, (size_t)nnz * s->vsize);
    if (e == hipSuccess) e = hipMalloc(&s->d_s, std::max<size_t>((size_t)m * s->vsize, 16));
    if (e == hipSuccess && (flags & 1)) e = hipMalloc(&s->d_kt, std::max<size_t>((size_t)n * ncols * s->vsize, 16));
    if (e == hipSuccess) e = hipMalloc(&s->d_red, (size_t)(s->nred + 2) * s->vsize);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    if (e != hipSuccess) return bail(e, "sddmm_create");
    *out = s;
    return SPMM_HIP_OK;
}

int spmm_sddmm_run_device(spmm_sddmm_t *s, const void *d_Q, const void *d_K, void *d_y, void *stream) {
    if (!s || (s->nnz > 0 && (!d_Q || !d_K || !d_y))) return sfail(SPMM_HIP_ERR_ARG, "sddmm_run_device: bad arguments");
    SDCHK(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    return s->dtype == SPMM_HIP_F64 ? run_t<double>(s, (const double *)d_Q, (const double *)d_K, (double *)d_y, st)
                                    : run_t<float>(s, (const float *)d_Q, (const float *)d_K, (float *)d_y, st);
}

int spmm_sddmm_run(spmm_sddmm_t *s, const void *Q, const void *K, int64_t k_rows, void *y) {
    if (!s || (s->nnz > 0 && (!Q || !K || !y))) return sfail(SPMM_HIP_ERR_ARG, "sddmm_run: bad arguments");
    const int64_t need = (s->flags & 1) ? s->ncols : s->m;
    if (k_rows < need) return sfail(SPMM_HIP_ERR_ARG, "sddmm_run: K has fewer rows than the mask needs");
    SDCHK(hipSetDevice(s->device));
    const size_t qb = (size_t)s->m * s->n * s->vsize, kb = (size_t)k_rows * s->n * s->vsize;
    if (!s->d_q) SDCHK(hipMalloc(&s->d_q, std::max<size_t>(qb, 16)));
    if (!s->d_y) SDCHK(hipMalloc(&s->d_y, std::max<size_t>((size_t)s->nnz * s->vsize, 16)));
    if (k_rows > s->krows_alloc) {
        if (s->d_k) SDCHK(hipFree(s->d_k));
        s->d_k = nullptr;
        SDCHK(hipMalloc(&s->d_k, std::max<size_t>(kb, 16)));
        s->krows_alloc = k_rows;
    }
    SDCHK(hipMemcpyAsync(s->d_q, Q, qb, hipMemcpyHostToDevice, s->stream));
    SDCHK(hipMemcpyAsync(s->d_k, K, kb, hipMemcpyHostToDevice, s->stream));
    int st = spmm_sddmm_run_device(s, s->d_q, s->d_k, s->d_y, s->stream);
    if (st != SPMM_HIP_OK) return st;
    SDCHK(hipMemcpyAsync(y, s->d_y, (size_t)s->nnz * s->vsize, hipMemcpyDeviceToHost, s->stream));
    SDCHK(hipStreamSynchronize(s->stream));
    return SPMM_HIP_OK;
}

int spmm_sddmm_destroy(spmm_sddmm_t *s) {
    if (!s) return SPMM_HIP_OK;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    void *ps[] = {s->d_rp, s->d_ci, s->d_prow, s->d_a, s->d_s, s->d_kt, s->d_red, s->d_q, s->d_k, s->d_y};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return SPMM_HIP_OK;
}

}  // extern "C"
