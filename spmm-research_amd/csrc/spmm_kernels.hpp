// spmm_kernels.hpp -- gfx950 (CDNA4) device kernels of the CSR SpMM engine.
//
// Hot path restated from the reference naive plugin compute_csr
// (benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp:70-96):
//     C[i][n] = sum_{j in row i} a[j] * B[ja[j]][n]      (left-to-right, from 0)
// re-designed for MI355X:
//   * one workgroup (256 lanes = 4 wave64) per nnz-balanced ROW BLOCK (<= CAP nonzeros, <= CAP_ROWS rows),
//     consecutive row blocks dealt to the same XCD (L2 reuse of B rows shared by neighbouring rows);
//   * the block's col_idx / values are streamed from HBM once, coalesced and non-temporal, into LDS;
//   * a "row group" of G lanes owns one row: each lane owns VEC consecutive columns of K (16-byte loads of the
//     row-major B row), walks the row's nonzeros in CSR order and accumulates with one FMA per nonzero --
//     the same left-to-right fused chain as the reference built with its own flags, so results are bit-equal;
//     U gathers are issued before their FMAs (memory-level parallelism), optionally for IL rows at once;
//   * 256/G row groups per workgroup, 64/G per wavefront; C rows written with (optionally non-temporal)
//     16-byte stores so the streamed output does not evict B from L2 / the Infinity Cache.
// Rows longer than CAP are split into chunks (spmm_long_chunks_kernel) whose partial sums are combined in a
// fixed order (spmm_long_combine_kernel): deterministic, no atomics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spmm {

constexpr int WG = 256;          // lanes per workgroup (4 wavefronts)
constexpr int CAP_ROWS = 512;    // rows per row block
constexpr int CAP_LONG = 2048;   // nonzeros per long-row chunk
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

template <typename T, int N, bool NT>
__device__ __forceinline__ void vstore(T *p, const vec<T, N> &v) {
    if constexpr (NT) {
#pragma unroll
        for (int i = 0; i < N; ++i) __builtin_nontemporal_store(v.v[i], p + i);
    } else {
        *reinterpret_cast<vec<T, N> *>(p) = v;
    }
}

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <typename T> struct stage_vec;
template <> struct stage_vec<double> { using type = f64x2; static constexpr int n = 2; };
template <> struct stage_vec<float> { using type = f32x4; static constexpr int n = 4; };

// B row gather: 64-bit flat address, or a buffer load with a 32-bit byte offset from a wave-uniform resource
// descriptor (fewer VGPRs per gather in flight; valid while ncols*K*sizeof(T) < 4 GiB, checked on the host).
template <typename T, int VEC, bool BUF>
struct BGather {
    const T *__restrict__ base;  // B + kk
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t lane_off;           // kk * sizeof(T)
    uint32_t row_bytes;          // K * sizeof(T)
    int K;
    __device__ __forceinline__ BGather(const T *B, int kk, int K_, uint32_t total_bytes) : K(K_) {
        base = B + kk;
        lane_off = (uint32_t)kk * sizeof(T);
        row_bytes = (uint32_t)K_ * sizeof(T);
        if constexpr (BUF) rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)B, (short)0, (int)total_bytes, 0x00020000);
    }
    __device__ __forceinline__ vec<T, VEC> operator()(int c) const {
        if constexpr (BUF && VEC * sizeof(T) == 16) {
            const i32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (uint32_t)c * row_bytes + lane_off, 0, 0);
            vec<T, VEC> v;
            __builtin_memcpy(&v, &r, 16);
            return v;
        } else {
            return *reinterpret_cast<const vec<T, VEC> *>(base + (size_t)c * K);
        }
    }
};

// Bijective XCD-aware remap: hardware deals workgroups round-robin over the 8 XCDs (bid % 8 share one), so
// give each XCD a contiguous run of row blocks.  Speed only; any placement gives the same result.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int q = nblk / NXCD, r = nblk % NXCD;
    const int x = bid % NXCD, i = bid / NXCD;
    return x * q + (x < r ? x : r) + i;
}

// One row, nonzeros [a, e) of the LDS-staged block: U gathers in flight, then U FMAs in CSR order.
template <typename T, int VEC, int U, typename Gather>
__device__ __forceinline__ vec<T, VEC> row_dot(const int32_t *s_col, const T *s_val, int a, int e,
                                               const Gather &gather) {
    using V = vec<T, VEC>;
    V acc = vzero<T, VEC>();
    int j = a;
    for (; j + U <= e; j += U) {
        V bv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) bv[u] = gather(s_col[j + u]);
#pragma unroll
        for (int u = 0; u < U; ++u) vfma(acc, s_val[j + u], bv[u]);
    }
    if (j < e) {  // tail: predicated gathers, FMAs only for real nonzeros (keeps -0.0 sums bit-exact)
        V bv[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j + u < e) bv[u] = gather(s_col[j + u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j + u < e) vfma(acc, s_val[j + u], bv[u]);
    }
    return acc;
}

// Two rows at once: their gathers interleave (2U in flight), each row still summed in its own CSR order.
template <typename T, int VEC, int U, typename Gather>
__device__ __forceinline__ void row_dot2(const int32_t *s_col, const T *s_val, int a0, int e0, int a1, int e1,
                                         const Gather &gather, vec<T, VEC> &acc0, vec<T, VEC> &acc1) {
    using V = vec<T, VEC>;
    acc0 = vzero<T, VEC>();
    acc1 = vzero<T, VEC>();
    const int n = max(e0 - a0, e1 - a1);
    for (int t = 0; t < n; t += U) {
        V b0[U], b1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (a0 + t + u < e0) b0[u] = gather(s_col[a0 + t + u]);
            if (a1 + t + u < e1) b1[u] = gather(s_col[a1 + t + u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (a0 + t + u < e0) vfma(acc0, s_val[a0 + t + u], b0[u]);
            if (a1 + t + u < e1) vfma(acc1, s_val[a1 + t + u], b1[u]);
        }
    }
}

// ------------------------------------------------------------------------------------------------ row blocks
// blk_rows[b] .. blk_rows[b+1]: the rows of block b (every row has <= CAP nonzeros, the block <= CAP in all);
// a row longer than CAP is a block of its own that this kernel skips (the long path writes it).
template <typename T, int VEC, int G, int U, int CAP, bool NTC, bool REMAP, int IL, bool BUF>
__global__ __launch_bounds__(WG) void spmm_rows_kernel(const int32_t *__restrict__ row_ptr,
                                                       const int32_t *__restrict__ col_idx,
                                                       const T *__restrict__ vals,
                                                       const int32_t *__restrict__ blk_rows, int nblk,
                                                       const T *__restrict__ B, T *__restrict__ C, int K,
                                                       uint32_t b_bytes) {
    using SV = typename stage_vec<T>::type;
    constexpr int SVN = stage_vec<T>::n;
    constexpr int CAPP = CAP + 4;                         // staged window starts at a 16-byte boundary
    __shared__ int32_t s_rp[CAP_ROWS + 1];
    __shared__ __attribute__((aligned(16))) int32_t s_col[CAPP];
    __shared__ __attribute__((aligned(16))) T s_val[CAPP];
    using V = vec<T, VEC>;
    constexpr int NG = WG / G;

    const int b = REMAP ? xcd_remap(blockIdx.x, nblk) : (int)blockIdx.x;
    const int tid = threadIdx.x;
    const int r0 = blk_rows[b], r1 = blk_rows[b + 1];
    const int nrows = r1 - r0;
    const int j0 = row_ptr[r0];
    const int j1 = row_ptr[r1];
    if (j1 - j0 > CAP) return;  // a long row: written by the long path

    // Stage the block's col_idx / values: 16-byte non-temporal loads, ALL issued before the first wait (one
    // memory round trip per block), from the 16-byte boundary jb <= j0 (arrays are padded on the device).
    const int jb = j0 & ~3;
    const int cnt = j1 - jb;
    {
        constexpr int NC = (CAPP / 4 + WG - 1) / WG;
        constexpr int NV = (CAPP / SVN + WG - 1) / WG;
        const int nc = (cnt + 3) / 4, nv = (cnt + SVN - 1) / SVN;
        i32x4 cb[NC];
        SV vb[NV];
        int rp[(CAP_ROWS + 1 + WG - 1) / WG];
#pragma unroll
        for (int u = 0; u < NC; ++u)
            if (tid + u * WG < nc)
                cb[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4 *>(col_idx + jb) + tid + u * WG);
#pragma unroll
        for (int u = 0; u < NV; ++u)
            if (tid + u * WG < nv)
                vb[u] = __builtin_nontemporal_load(reinterpret_cast<const SV *>(vals + jb) + tid + u * WG);
#pragma unroll
        for (int u = 0; u < (CAP_ROWS + 1 + WG - 1) / WG; ++u)
            if (tid + u * WG <= nrows) rp[u] = row_ptr[r0 + tid + u * WG];
#pragma unroll
        for (int u = 0; u < NC; ++u)
            if (tid + u * WG < nc) reinterpret_cast<i32x4 *>(s_col)[tid + u * WG] = cb[u];
#pragma unroll
        for (int u = 0; u < NV; ++u)
            if (tid + u * WG < nv) reinterpret_cast<SV *>(s_val)[tid + u * WG] = vb[u];
#pragma unroll
        for (int u = 0; u < (CAP_ROWS + 1 + WG - 1) / WG; ++u)
            if (tid + u * WG <= nrows) s_rp[tid + u * WG] = rp[u] - jb;
    }
    __syncthreads();

    const int lane = tid % G;
    const int grp = tid / G;
    for (int kc = 0; kc < K; kc += G * VEC) {
        const int kk = kc + lane * VEC;
        if (kk >= K) continue;
        const BGather<T, VEC, BUF> gather(B, kk, K, b_bytes);
        if constexpr (IL == 1) {
            for (int r = grp; r < nrows; r += NG) {
                const V acc = row_dot<T, VEC, U>(s_col, s_val, s_rp[r], s_rp[r + 1], gather);
                vstore<T, VEC, NTC>(C + (size_t)(r0 + r) * K + kk, acc);
            }
        } else {
            for (int r = grp; r < nrows; r += 2 * NG) {
                const int r2 = r + NG;
                const bool has2 = r2 < nrows;
                V acc0, acc1;
                row_dot2<T, VEC, U>(s_col, s_val, s_rp[r], s_rp[r + 1], has2 ? s_rp[r2] : 0, has2 ? s_rp[r2 + 1] : 0,
                                    gather, acc0, acc1);
                vstore<T, VEC, NTC>(C + (size_t)(r0 + r) * K + kk, acc0);
                if (has2) vstore<T, VEC, NTC>(C + (size_t)(r0 + r2) * K + kk, acc1);
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
