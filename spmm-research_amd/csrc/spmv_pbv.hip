// spmv_pbv.hip -- the perfect-balance CSR format (include/spmm_pbv.h): K = 1 SpMV over a merge path, gfx950.
//
// Reference: the CUSTOM_VECTOR_PERFECT_NNZ_BALANCE build of the CSR plugin
// (benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel_csr.cpp:68-80 evenly split nonzeros + binary search of the
// first row, :626-680 partial first/last rows and the serial fix-up of thread partials).  On the GPU the balance
// unit is the LANE and the split covers row ends as well as nonzeros (merge path), so rows of any length and empty
// rows cost every lane the same E items:
//   * items = the m row ends and the nnz nonzeros, merged in CSR order (row end i comes after the nonzeros of row
//     i); block b = items [b*256E, (b+1)*256E), lane l of a block = E consecutive items of it.
//   * The host plans the block starts {row, nonzero} (a binary search per block, as the reference searches each
//     thread's first row).  A workgroup stages its block's row ends, column indices and values in LDS, each lane
//     finds its own start by a binary search over the staged row ends (the merge-path diagonal search), issues the
//     gathers x[col] of all its nonzeros at once (E in flight), then walks its items: a nonzero is one FMA into the
//     running row, a row end stores the row and restarts from +0.
//   * A row whose items lie in one lane is one FMA chain from 0 in CSR order: the reference's serial bits.  A row
//     cut by lane boundaries: each lane's piece is a chain; the lane holding the row end adds the pieces of the
//     lanes before it in lane order (LDS), then its own.  A row cut by block boundaries: the block's pieces go to
//     carry slots, and a second launch (one thread per run of slots) adds them in block order in front of the value
//     the closing block stored.  Deterministic, no atomics; split rows are reported inexact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/spmm_pbv.h"

namespace {

constexpr int WG = 256;
thread_local std::string g_detail;

int fail(int st, const std::string &what) {
    g_detail = what;
    return st;
}

__device__ __forceinline__ double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// One block of 256 x E merge items.  blk[b] = {first row, first nonzero} of block b (blk[nblk] = {m, nnz}).
// carry_row[b] / carry_val[b]: the block's piece of the row still open at its end (-1: none).
template <typename T, int E>
__global__ __launch_bounds__(WG) void pbv_block_kernel(const int32_t *__restrict__ row_ptr,
                                                        const int32_t *__restrict__ col_idx,
                                                        const T *__restrict__ vals, const int2 *__restrict__ blk, int m,
                                                        const T *__restrict__ x, T *__restrict__ y, long ldy,
                                                        int32_t *__restrict__ carry_row, T *__restrict__ carry_val) {
    constexpr int ITEMS = WG * E;
    __shared__ int32_t s_end[ITEMS + 1];   // row ends of the block's rows, relative to its first nonzero
    __shared__ int32_t s_col[ITEMS];
    __shared__ T s_val[ITEMS];
    __shared__ int32_t s_crow[WG];         // lane carry: row (block-relative) still open at the lane's end
    __shared__ T s_cval[WG];               //             and the lane's piece of it
    __shared__ int2 s_start[WG + 1];

    const int b = blockIdx.x, tid = threadIdx.x;
    const int2 c0 = blk[b], c1 = blk[b + 1];
    const int i0 = c0.x, j0 = c0.y;
    const int nr = c1.x - i0;              // row ends in the block
    const int nn = c1.y - j0;              // nonzeros in the block
#pragma unroll 4
    for (int t = tid; t < nr; t += WG) s_end[t] = row_ptr[i0 + t + 1] - j0;
#pragma unroll 4
    for (int t = tid; t < nn; t += WG) {
        s_col[t] = col_idx[j0 + t];
        s_val[t] = vals[j0 + t];
    }
    if (tid == 0) s_end[nr] = 0x7fffffff;  // the row open at the block end never closes here
    __syncthreads();

    // merge-path search of this lane's first item: the split (i, d - i) of diagonal d with row ends [0, i) and
    // nonzeros [0, d - i) consumed
    {
        const int d = min(tid * E, nr + nn);
        int lo = max(d - nn, 0), hi = min(d, nr);
        while (lo < hi) {
            const int p = (lo + hi) >> 1;
            if (s_end[p] <= d - p - 1) lo = p + 1;
            else hi = p;
        }
        s_start[tid] = make_int2(lo, d - lo);
        if (tid == 0) s_start[WG] = make_int2(nr, nn);
    }
    __syncthreads();
    const int il = s_start[tid].x, jl = s_start[tid].y;
    const int ie = s_start[tid + 1].x, je = s_start[tid + 1].y;
    const int nz = je - jl;

    T xv[E];
#pragma unroll
    for (int t = 0; t < E; ++t)
        if (t < nz) xv[t] = x[s_col[jl + t]];

    // does the lane's first row start before the lane (a piece of a row begun by earlier lanes / blocks)?
    const int rstart = il > 0 ? s_end[il - 1] : row_ptr[i0] - j0;
    bool head = rstart < jl;
    int hrow = -1;
    T hval = T(0);
    T acc = T(0);
    int i = il;
    auto close_row = [&](int r) {
        if (head) {           // combined with the earlier pieces below
            hrow = r;
            hval = acc;
            head = false;
        } else {
            y[(long)(i0 + r) * ldy] = acc;
        }
        acc = T(0);
    };
#pragma unroll
    for (int t = 0; t < E; ++t) {
        if (t < nz) {
            const int j = jl + t;
            while (s_end[i] <= j) close_row(i++);
            acc = fma_(s_val[j], xv[t], acc);
        }
    }
    while (i < ie) close_row(i++);
    s_crow[tid] = ie;
    s_cval[tid] = acc;
    __syncthreads();

    if (hrow >= 0) {   // pieces of row hrow in the lanes just before this one, added in lane order, then this one's
        int l = tid - 1;
        while (l >= 0 && s_crow[l] == hrow) --l;
        T s = hval;
        if (l + 1 < tid) {
            s = s_cval[l + 1];
            for (int q = l + 2; q < tid; ++q) s += s_cval[q];
            s += hval;
        }
        y[(long)(i0 + hrow) * ldy] = s;
    }
    if (tid == WG - 1) {   // the block's piece of its open row (lanes of the run ending here, in lane order)
        if (i0 + nr < m) {
            int l = WG - 1;
            while (l >= 0 && s_crow[l] == nr) --l;
            T s = s_cval[l + 1];
            for (int q = l + 2; q < WG; ++q) s += s_cval[q];
            carry_row[b] = i0 + nr;
            carry_val[b] = s;
        } else {
            carry_row[b] = -1;
        }
    }
}

// Rows cut by block boundaries: the first slot of each run of equal rows adds the run in block order, then the value
// the closing block stored.
template <typename T>
__global__ __launch_bounds__(WG) void pbv_fixup_kernel(const int32_t *__restrict__ carry_row,
                                                        const T *__restrict__ carry_val, int nblk, T *__restrict__ y,
                                                        long ldy) {
    const int b = blockIdx.x * WG + threadIdx.x;
    if (b >= nblk) return;
    const int r = carry_row[b];
    if (r < 0 || (b > 0 && carry_row[b - 1] == r)) return;
    T s = carry_val[b];
    for (int q = b + 1; q < nblk && carry_row[q] == r; ++q) s += carry_val[q];
    y[(long)r * ldy] = s + y[(long)r * ldy];
}

#define HIP_TRY(call)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (call);                                                                        \
        if (e_ != hipSuccess) return fail(SPMM_HIP_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

struct spmm_pbv_handle {
    int64_t m = 0, ncols = 0, nnz = 0;
    int32_t dtype = SPMM_HIP_F64, device = 0, e = 8;
    int64_t nblk = 0, exact = 0, block_cut = 0, bytes = 0;
    std::vector<uint8_t> exact_mask;
    int32_t *d_rp = nullptr, *d_col = nullptr, *d_crow = nullptr;
    void *d_val = nullptr, *d_cval = nullptr;
    int2 *d_blk = nullptr;
    void *d_x = nullptr, *d_y = nullptr;   // host-run staging
    size_t x_cap = 0, y_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipStream_t stream = nullptr;
    double last_ms = 0.0;
};

namespace {
template <typename T, int E>
void launch(spmm_pbv_t *h, const T *x, T *y, long ldy, hipStream_t s) {
    const int nb = (int)h->nblk;
    pbv_block_kernel<T, E><<<nb, WG, 0, s>>>(h->d_rp, h->d_col, (const T *)h->d_val, h->d_blk, (int)h->m, x, y, ldy,
                                              h->d_crow, (T *)h->d_cval);
    pbv_fixup_kernel<T><<<(nb + WG - 1) / WG, WG, 0, s>>>(h->d_crow, (const T *)h->d_cval, nb, y, ldy);
}

template <typename T>
void launch_e(spmm_pbv_t *h, const void *x, void *y, long ldy, hipStream_t s) {
    if (h->e == 4) launch<T, 4>(h, (const T *)x, (T *)y, ldy, s);
    else if (h->e == 8) launch<T, 8>(h, (const T *)x, (T *)y, ldy, s);
    else launch<T, 16>(h, (const T *)x, (T *)y, ldy, s);
}
}  // namespace

extern "C" {

int64_t spmm_pbv_nblk(int64_t m, int64_t nnz, int32_t e) {
    if (m <= 0 || e <= 0) return 0;
    const int64_t items = (int64_t)WG * e;
    return (m + nnz + items - 1) / items;
}

int spmm_pbv_plan_host(const int32_t *row_ptr, int64_t m, int64_t nnz, int32_t e, int32_t *blk_out,
                       uint8_t *exact_out) {
    if (!row_ptr || m < 0 || nnz < 0 || e < SPMM_PBV_E_MIN || e > SPMM_PBV_E_MAX || (!blk_out && m > 0))
        return fail(SPMM_HIP_ERR_ARG, "pbv plan: bad arguments");
    if (m + nnz + (int64_t)WG * e >= INT32_MAX) return fail(SPMM_HIP_ERR_OVERFLOW, "pbv plan: m + nnz exceeds int32");
    const int64_t items = (int64_t)WG * e;
    const int64_t nblk = spmm_pbv_nblk(m, nnz, e);
    for (int64_t b = 0; b <= nblk; ++b) {
        const int64_t d = std::min(b * items, m + nnz);
        int64_t lo = std::max<int64_t>(d - nnz, 0), hi = std::min<int64_t>(d, m);
        while (lo < hi) {   // the merge-path split of diagonal d, as the kernel's per-lane search
            const int64_t p = (lo + hi) >> 1;
            if (row_ptr[p + 1] <= d - p - 1) lo = p + 1;
            else hi = p;
        }
        blk_out[2 * b] = (int32_t)lo;
        blk_out[2 * b + 1] = (int32_t)(d - lo);
    }
    if (exact_out)
        for (int64_t r = 0; r < m; ++r)   // first nonzero item and row-end item in the same lane
            exact_out[r] = (r + row_ptr[r]) / e == (r + row_ptr[r + 1]) / e;
    return SPMM_HIP_OK;
}

int spmm_pbv_create(const int32_t *row_ptr, const int32_t *col_idx, const void *values, int64_t m, int64_t ncols,
                    int64_t nnz, int32_t dtype, int32_t device, int32_t e, spmm_pbv_t **out) {
    if (!out || !row_ptr || m < 0 || ncols < 0 || nnz < 0 || (nnz > 0 && (!col_idx || !values)))
        return fail(SPMM_HIP_ERR_ARG, "pbv create: bad arguments");
    if (dtype != SPMM_HIP_F64 && dtype != SPMM_HIP_F32) return fail(SPMM_HIP_ERR_ARG, "pbv create: dtype");
    if (e == 0) e = 8;
    if (e != 4 && e != 8 && e != 16) return fail(SPMM_HIP_ERR_ARG, "pbv create: items_per_lane must be 4, 8 or 16");
    *out = nullptr;
    if (row_ptr[0] != 0 || row_ptr[m] != nnz) return fail(SPMM_HIP_ERR_CSR, "pbv create: row_ptr[0] / row_ptr[m]");
    for (int64_t r = 0; r < m; ++r)
        if (row_ptr[r + 1] < row_ptr[r]) return fail(SPMM_HIP_ERR_CSR, "pbv create: row_ptr not monotone");
    for (int64_t j = 0; j < nnz; ++j)
        if (col_idx[j] < 0 || col_idx[j] >= ncols) return fail(SPMM_HIP_ERR_CSR, "pbv create: column out of range");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(SPMM_HIP_ERR_NODEVICE, "pbv create: no such device");
    auto *h = new spmm_pbv_handle;
    h->m = m, h->ncols = ncols, h->nnz = nnz, h->dtype = dtype, h->device = device, h->e = e;
    h->nblk = spmm_pbv_nblk(m, nnz, e);
    std::vector<int32_t> blk(2 * (h->nblk + 1));
    h->exact_mask.resize(m);
    int st = spmm_pbv_plan_host(row_ptr, m, nnz, e, blk.data(), h->exact_mask.data());
    if (st != SPMM_HIP_OK) {
        delete h;
        return st;
    }
    const int64_t items = (int64_t)WG * e;
    for (int64_t r = 0; r < m; ++r) {
        h->exact += h->exact_mask[r];
        h->block_cut += (r + row_ptr[r]) / items != (r + row_ptr[r + 1]) / items;
    }
    const size_t s = dtype == SPMM_HIP_F64 ? 8 : 4;
    auto up = [&](void **d, const void *src, size_t bytes) -> int {
        if (hipMalloc(d, std::max<size_t>(bytes, 16)) != hipSuccess) return fail(SPMM_HIP_ERR_NOMEM, "pbv create: hipMalloc");
        h->bytes += (int64_t)std::max<size_t>(bytes, 16);
        if (bytes && src && hipMemcpy(*d, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
            return fail(SPMM_HIP_ERR_HIP, "pbv create: hipMemcpy");
        return SPMM_HIP_OK;
    };
    if (hipSetDevice(device) != hipSuccess ||
        (st = up((void **)&h->d_rp, row_ptr, (m + 1) * 4)) != SPMM_HIP_OK ||
        (st = up((void **)&h->d_col, col_idx, nnz * 4)) != SPMM_HIP_OK || (st = up(&h->d_val, values, nnz * s)) != SPMM_HIP_OK ||
        (st = up((void **)&h->d_blk, blk.data(), blk.size() * 4)) != SPMM_HIP_OK ||
        (st = up((void **)&h->d_crow, nullptr, h->nblk * 4)) != SPMM_HIP_OK ||
        (st = up(&h->d_cval, nullptr, h->nblk * s)) != SPMM_HIP_OK ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
        spmm_pbv_destroy(h);
        return st != SPMM_HIP_OK ? st : fail(SPMM_HIP_ERR_HIP, "pbv create: device setup");
    }
    *out = h;
    return SPMM_HIP_OK;
}

int spmm_pbv_run_device(spmm_pbv_t *h, const void *d_x, void *d_y, int64_t ldy, void *stream) {
    if (!h || (h->m > 0 && !d_y) || (h->nnz > 0 && !d_x) || ldy < 1) return fail(SPMM_HIP_ERR_ARG, "pbv run_device: bad arguments");
    if (h->m == 0) return SPMM_HIP_OK;
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipEventRecord(h->ev0, s));
    if (h->dtype == SPMM_HIP_F64) launch_e<double>(h, d_x, d_y, (long)ldy, s);
    else launch_e<float>(h, d_x, d_y, (long)ldy, s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev1, s));
    h->stream = s;
    return SPMM_HIP_OK;
}

int spmm_pbv_run(spmm_pbv_t *h, const void *x, void *y, int32_t k) {
    if (!h || k < 1 || (h->m > 0 && !y) || (h->ncols > 0 && !x)) return fail(SPMM_HIP_ERR_ARG, "pbv run: bad arguments");
    if (h->m == 0) return SPMM_HIP_OK;
    HIP_TRY(hipSetDevice(h->device));
    const size_t s = h->dtype == SPMM_HIP_F64 ? 8 : 4;
    const size_t xb = (size_t)h->ncols * k * s, yb = (size_t)h->m * k * s;
    if (xb > h->x_cap) {
        if (h->d_x) (void)hipFree(h->d_x);
        h->d_x = nullptr;
        if (hipMalloc(&h->d_x, std::max<size_t>(xb, 16)) != hipSuccess) return fail(SPMM_HIP_ERR_NOMEM, "pbv run: x");
        h->x_cap = xb;
    }
    if (yb > h->y_cap) {
        if (h->d_y) (void)hipFree(h->d_y);
        h->d_y = nullptr;
        if (hipMalloc(&h->d_y, yb) != hipSuccess) return fail(SPMM_HIP_ERR_NOMEM, "pbv run: y");
        h->y_cap = yb;
    }
    if (xb) HIP_TRY(hipMemcpy(h->d_x, x, xb, hipMemcpyHostToDevice));
    for (int c = 0; c < k; ++c) {   // one SpMV per column of x (column-major), into column c of row-major y
        const int st = spmm_pbv_run_device(h, (const char *)h->d_x + (size_t)c * h->ncols * s, (char *)h->d_y + c * s,
                                           k, nullptr);
        if (st != SPMM_HIP_OK) return st;
    }
    HIP_TRY(hipMemcpy(y, h->d_y, yb, hipMemcpyDeviceToHost));
    return SPMM_HIP_OK;
}

int spmm_pbv_last_ms(spmm_pbv_t *h, double *ms) {
    if (!h || !ms) return fail(SPMM_HIP_ERR_ARG, "pbv last_ms: bad arguments");
    *ms = 0.0;
    if (h->m == 0) return SPMM_HIP_OK;
    HIP_TRY(hipEventSynchronize(h->ev1));
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, h->ev0, h->ev1));
    *ms = h->last_ms = t;
    return SPMM_HIP_OK;
}

int spmm_pbv_exact_rows(spmm_pbv_t *h, uint8_t *out) {
    if (!h || (!out && h->m > 0)) return fail(SPMM_HIP_ERR_ARG, "pbv exact_rows: bad arguments");
    if (h->m) std::memcpy(out, h->exact_mask.data(), h->m);
    return SPMM_HIP_OK;
}

int spmm_pbv_info(spmm_pbv_t *h, int64_t *out, int32_t n) {
    if (!h || !out || n < 0) return fail(SPMM_HIP_ERR_ARG, "pbv info: bad arguments");
    const int64_t v[5] = {h->nblk, h->e, h->exact, h->block_cut, h->bytes};
    for (int i = 0; i < n && i < 5; ++i) out[i] = v[i];
    return SPMM_HIP_OK;
}

int spmm_pbv_stats_labels(char *buf, long buf_n) {
    if (!buf || buf_n <= 0) return fail(SPMM_HIP_ERR_ARG, "pbv stats_labels: buffer");
    const int n = snprintf(buf, (size_t)buf_n,
                           ",kernel_ms,bytes_alg,hbm_gbs_alg,roofline_frac,blocks,items_per_lane,exact_rows,device");
    return (int)std::min<long>(n, buf_n - 1);
}

int spmm_pbv_stats(spmm_pbv_t *h, char *buf, long buf_n) {
    if (!h || !buf || buf_n <= 0) return fail(SPMM_HIP_ERR_ARG, "pbv stats: bad arguments");
    double ms = 0.0;
    const int st = spmm_pbv_last_ms(h, &ms);
    if (st != SPMM_HIP_OK) return st;
    const double s = h->dtype == SPMM_HIP_F64 ? 8 : 4;   // K = 1: row_ptr, A, x once, y once
    const double bytes = 4.0 * (h->m + 1) + (4 + s) * h->nnz + s * h->ncols + s * h->m;
    const double gbs = ms > 0 ? bytes / (ms * 1e-3) / 1e9 : 0.0;
    const int n = snprintf(buf, (size_t)buf_n, ",%.6f,%.0f,%.2f,%.4f,%lld,%d,%lld,%d", ms, bytes, gbs, gbs / 8000.0,
                           (long long)h->nblk, h->e, (long long)h->exact, h->device);
    return (int)std::min<long>(n, buf_n - 1);
}

int spmm_pbv_destroy(spmm_pbv_t *h) {
    if (!h) return SPMM_HIP_OK;
    (void)hipSetDevice(h->device);
    for (void *p : {(void *)h->d_rp, (void *)h->d_col, h->d_val, (void *)h->d_blk, (void *)h->d_crow, h->d_cval, h->d_x,
                    h->d_y})
        if (p) (void)hipFree(p);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    delete h;
    return SPMM_HIP_OK;
}

const char *spmm_pbv_last_error_detail(void) { return g_detail.c_str(); }

}  // extern "C"
