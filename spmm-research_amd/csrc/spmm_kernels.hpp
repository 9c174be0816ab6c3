// spmm_kernels.hpp -- gfx950 (CDNA4) device kernels of the CSR SpMM engine.
//
// Hot path restated from the reference naive plugin compute_csr
// (benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp:70-96):
//     C[i][n] = sum_{j in row i} a[j] * B[ja[j]][n]      (left-to-right, from 0)
// re-designed for MI355X:
//   * one workgroup (256 lanes = 4 wave64) per nnz-balanced ROW BLOCK (<= CAP_NNZ nonzeros, <= CAP_ROWS rows),
//     consecutive row blocks dealt to the same XCD (L2 reuse of B rows shared by neighbouring rows);
//   * the block's col_idx / values are streamed from HBM once, coalesced, into LDS;
//   * a "row group" of G lanes owns one row: each lane owns VEC consecutive columns of K (16-byte loads of the
//     row-major B row), walks the row's nonzeros in CSR order and accumulates with one FMA per nonzero --
//     the same left-to-right fused chain as the reference built with its own flags, so results are bit-equal;
//   * 256/G row groups per workgroup, 64/G per wavefront.
// Rows longer than CAP_NNZ are split into chunks (spmm_long_chunks_kernel) whose partial sums are combined in
// a fixed order (spmm_long_combine_kernel): deterministic, no atomics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spmm {

constexpr int WG = 256;          // lanes per workgroup (4 wavefronts)
constexpr int CAP_NNZ = 2048;    // nonzeros staged per row block (also the longest row kept sequential)
constexpr int CAP_ROWS = 512;    // rows per row block
constexpr int NXCD = 8;          // MI355X: 8 accelerator dies, one L2 each

template <typename T, int N>
struct alignas(sizeof(T) * N) vec {
    T v[N];
};

template <typename T, int N>
__device__ __forceinline__ vec<T, N> vzero() {
    vec<T, N> r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = T(0);
    return r;
}

__device__ __forceinline__ double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

template <typename T, int N>
__device__ __forceinline__ void vfma(vec<T, N> &acc, T a, const vec<T, N> &b) {
#pragma unroll
    for (int i = 0; i < N; ++i) acc.v[i] = fma_(a, b.v[i], acc.v[i]);
}

// Bijective XCD-aware remap: hardware deals workgroups round-robin over the 8 XCDs (bid % 8 share one), so
// give each XCD a contiguous run of row blocks.  Speed only; any placement gives the same result.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int q = nblk / NXCD, r = nblk % NXCD;
    const int x = bid % NXCD, i = bid / NXCD;
    return x * q + (x < r ? x : r) + i;
}

// ------------------------------------------------------------------------------------------------ row blocks
// blk_rows[b] .. blk_rows[b+1]: the rows of block b (every row of the block has <= CAP_NNZ nonzeros and the block
// holds <= CAP_NNZ nonzeros; rows longer than CAP_NNZ form blocks of their own that this kernel skips: the long
// path writes them).
template <typename T, int VEC, int G, int UNROLL>
__global__ __launch_bounds__(WG) void spmm_rows_kernel(const int32_t *__restrict__ row_ptr,
                                                       const int32_t *__restrict__ col_idx,
                                                       const T *__restrict__ vals,
                                                       const int32_t *__restrict__ blk_rows, int nblk,
                                                       const T *__restrict__ B, T *__restrict__ C, int K) {
    __shared__ int32_t s_rp[CAP_ROWS + 1];
    __shared__ int32_t s_col[CAP_NNZ];
    __shared__ T s_val[CAP_NNZ];
    using V = vec<T, VEC>;
    constexpr int NG = WG / G;

    const int b = xcd_remap(blockIdx.x, nblk);
    const int tid = threadIdx.x;
    const int r0 = blk_rows[b], r1 = blk_rows[b + 1];
    const int nrows = r1 - r0;
    const int j0 = row_ptr[r0];
    const int nnz = row_ptr[r1] - j0;
    if (nnz > CAP_NNZ) return;  // a long row: written by the long path

    for (int i = tid; i <= nrows; i += WG) s_rp[i] = row_ptr[r0 + i] - j0;
    for (int i = tid; i < nnz; i += WG) {
        s_col[i] = __builtin_nontemporal_load(col_idx + j0 + i);
        s_val[i] = __builtin_nontemporal_load(vals + j0 + i);
    }
    __syncthreads();

    const int lane = tid % G;
    const int grp = tid / G;
    for (int kc = 0; kc < K; kc += G * VEC) {
        const int kk = kc + lane * VEC;
        const bool active = kk < K;
        const T *__restrict__ Bk = B + kk;
        for (int r = grp; r < nrows; r += NG) {
            const int a = s_rp[r], e = s_rp[r + 1];
            V acc = vzero<T, VEC>();
            if (active) {
                int j = a;
                for (; j + UNROLL <= e; j += UNROLL) {
                    V bv[UNROLL];
                    T av[UNROLL];
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) {
                        const int c = s_col[j + u];
                        av[u] = s_val[j + u];
                        bv[u] = *reinterpret_cast<const V *>(Bk + (size_t)c * K);
                    }
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) vfma(acc, av[u], bv[u]);
                }
                for (; j < e; ++j) {
                    const int c = s_col[j];
                    const V bv = *reinterpret_cast<const V *>(Bk + (size_t)c * K);
                    vfma(acc, s_val[j], bv);
                }
                *reinterpret_cast<V *>(C + (size_t)(r0 + r) * K + kk) = acc;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------- long rows
// chunk = {row, j_begin, j_end, slot}: one workgroup per chunk; its 256/G row groups each take a contiguous
// sub-range of the chunk, sum it left to right, and group partials are added in group order into P[slot][:].
template <typename T, int VEC, int G>
__global__ __launch_bounds__(WG) void spmm_long_chunks_kernel(const int32_t *__restrict__ col_idx,
                                                              const T *__restrict__ vals,
                                                              const int4 *__restrict__ chunks,
                                                              const T *__restrict__ B, T *__restrict__ P,
                                                              int K) {
    __shared__ T s_part[WG * VEC];
    using V = vec<T, VEC>;
    constexpr int NG = WG / G;
    const int4 ch = chunks[blockIdx.x];
    const int tid = threadIdx.x, lane = tid % G, grp = tid / G;
    const int len = ch.z - ch.y;
    const int sub = (len + NG - 1) / NG;
    const int ga = ch.y + grp * sub;
    const int ge = min(ga + sub, ch.z);
    for (int kc = 0; kc < K; kc += G * VEC) {
        const int kk = kc + lane * VEC;
        const bool active = kk < K;
        V acc = vzero<T, VEC>();
        if (active) {
            for (int j = ga; j < ge; ++j) {
                const int c = col_idx[j];
                const V bv = *reinterpret_cast<const V *>(B + (size_t)c * K + kk);
                vfma(acc, vals[j], bv);
            }
        }
#pragma unroll
        for (int i = 0; i < VEC; ++i) s_part[tid * VEC + i] = acc.v[i];
        __syncthreads();
        if (grp == 0 && active) {
            V tot = vzero<T, VEC>();
            for (int g = 0; g < NG; ++g) {
#pragma unroll
                for (int i = 0; i < VEC; ++i) tot.v[i] += s_part[(g * G + lane) * VEC + i];
            }
            *reinterpret_cast<V *>(P + (size_t)ch.w * K + kk) = tot;
        }
        __syncthreads();
    }
}

// long_rows[r] = {row, first_slot, nslots, 0}: C[row][n] = sum over the row's chunks, in chunk order.
template <typename T>
__global__ __launch_bounds__(WG) void spmm_long_combine_kernel(const int4 *__restrict__ long_rows, int nlong,
                                                               const T *__restrict__ P, T *__restrict__ C, int K) {
    const int64_t t = (int64_t)blockIdx.x * WG + threadIdx.x;
    if (t >= (int64_t)nlong * K) return;
    const int li = (int)(t / K), n = (int)(t % K);
    const int4 lr = long_rows[li];
    T s = T(0);
    for (int q = 0; q < lr.z; ++q) s += P[(size_t)(lr.y + q) * K + n];
    C[(size_t)lr.x * K + n] = s;
}

// ------------------------------------------------------------------------------------------------ transpose
// Reference B layout (column-major, x[n*ncols + c]) -> engine layout (row-major, B[c*K + n]).
// 64 (c) x 32 (n) tiles through LDS; reads coalesced along c, writes coalesced along n.
template <typename T>
__global__ __launch_bounds__(WG) void transpose_colmajor_kernel(const T *__restrict__ X, T *__restrict__ Bt,
                                                                int64_t ncols, int K) {
    __shared__ T tile[32][64 + 1];
    const int64_t c0 = (int64_t)blockIdx.x * 64;
    const int n0 = blockIdx.y * 32;
    const int tx = threadIdx.x % 64, ty = threadIdx.x / 64;  // 64 x 4
    for (int n = ty; n < 32; n += 4) {
        const int64_t c = c0 + tx;
        if (n0 + n < K && c < ncols) tile[n][tx] = X[(int64_t)(n0 + n) * ncols + c];
    }
    __syncthreads();
    const int tn = threadIdx.x % 32, tc = threadIdx.x / 32;  // 32 x 8
    for (int c = tc; c < 64; c += 8) {
        const int64_t cc = c0 + c;
        if (n0 + tn < K && cc < ncols) Bt[cc * K + n0 + tn] = tile[tn][c];
    }
}

}  // namespace spmm
