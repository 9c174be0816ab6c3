// spmm_kernels.hpp -- gfx950 (CDNA4) device kernels of the CSR SpMM engine.
//
// Hot path restated from the reference naive plugin compute_csr
// (benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp:70-96):
//     C[i][n] = sum_{j in row i} a[j] * B[ja[j]][n]      (left-to-right, from 0)
// re-designed for MI355X:
//   * The inspector (spmm_engine.hip) turns A's rows into VIRTUAL ROWS of at most T nonzeros (a row longer than T
//     becomes ceil(len/T) consecutive pieces) and packs consecutive virtual rows into nnz-balanced BLOCKS.
//   * One workgroup (256 lanes = 4 wave64) per block: the block's col_idx / values / row offsets are staged into
//     LDS (16-byte lanes); a ROW GROUP of G lanes owns one virtual row; each lane owns VEC consecutive
//     columns of the K-panel (16-byte gathers of the row-major B row), issues U gathers, then accumulates them in
//     CSR order with one FMA each -- the same left-to-right fused chain as the reference built with its own flags,
//     so every row that is not split is bit-identical to the reference.
//   * A virtual row's result goes to its C row, or (split rows) to a partial row P[slot]; the combine kernel adds a
//     split row's partials in slot order (deterministic, no atomics).
//   * C and P rows are written with non-temporal 16-byte stores so the output stream does not evict B from the
//     Infinity Cache; K wider than the cache-sized panel is processed panel by panel (one launch each).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spmm {

constexpr int WG = 256;          // lanes per workgroup (4 wavefronts)
constexpr int CAP_ROWS = 512;    // virtual rows per block

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

// B row gather: 64-bit flat address, or a buffer load with a 32-bit byte offset from a wave-uniform resource
// descriptor (valid while ncols*K*sizeof(T) < 4 GiB; the host falls back to the flat form otherwise).
template <typename T, int VEC, bool BUF>
struct BGather {
    const T *__restrict__ base;  // B + panel offset + lane columns
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t lane_off;           // (panel offset + lane columns) * sizeof(T)
    uint32_t row_bytes;          // ld * sizeof(T)
    int ld;
    __device__ __forceinline__ BGather(const T *B, int kk, int ld_, uint32_t total_bytes) : ld(ld_) {
        base = B + kk;
        lane_off = (uint32_t)kk * sizeof(T);
        row_bytes = (uint32_t)ld_ * sizeof(T);
        if constexpr (BUF) rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)B, (short)0, (int)total_bytes, 0x00020000);
    }
    __device__ __forceinline__ vec<T, VEC> operator()(int c) const {
        if constexpr (BUF && VEC * sizeof(T) == 16) {
            const i32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (uint32_t)c * row_bytes + lane_off, 0, 0);
            vec<T, VEC> v;
            __builtin_memcpy(&v, &r, 16);
            return v;
        } else {
            return *reinterpret_cast<const vec<T, VEC> *>(base + (size_t)c * ld);
        }
    }
};

// Software-pipelined row (tuning build: U < 0 selects it with |U| per batch): batch j+1's gathers are issued before
// batch j's FMAs, so between |U| and 2|U| gathers stay in flight instead of U then none; same FMA order.
template <typename T, int VEC, int U, typename Gather>
__device__ __forceinline__ vec<T, VEC> row_dot_pipe(vec<T, VEC> acc, const int32_t *s_col, const T *s_val, int a,
                                                    int e, const Gather &gather) {
    using V = vec<T, VEC>;
    V b0[U], b1[U];
    auto issue = [&](V *b, int j) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j + u < e) b[u] = gather(s_col[j + u]);
    };
    auto fold = [&](const V *b, int j) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j + u < e) vfma(acc, s_val[j + u], b[u]);
    };
    int j = a;
    if (j < e) issue(b0, j);
    while (j < e) {
        issue(b1, j + U);
        fold(b0, j);
        j += U;
        if (j >= e) break;
        issue(b0, j + U);
        fold(b1, j);
        j += U;
    }
    return acc;
}

// One virtual row, nonzeros [a, e) of the LDS-staged block: U gathers in flight, then U FMAs in CSR order.
template <typename T, int VEC, int U, typename Gather>
__device__ __forceinline__ vec<T, VEC> row_dot_batch(vec<T, VEC> acc, const int32_t *s_col, const T *s_val, int a,
                                                     int e, const Gather &gather) {
    using V = vec<T, VEC>;
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

template <typename T, int VEC, int U, typename Gather>
__device__ __forceinline__ vec<T, VEC> row_dot(vec<T, VEC> acc, const int32_t *s_col, const T *s_val, int a, int e,
                                               const Gather &gather) {
    if constexpr (U < 0) return row_dot_pipe<T, VEC, -U>(acc, s_col, s_val, a, e, gather);
    else return row_dot_batch<T, VEC, U>(acc, s_col, s_val, a, e, gather);
}

// Strided piece of a virtual row for vector lanes: nonzeros a, a+L, a+2L, ... < e (L = 1: the whole row, in order).
template <typename T, int VEC, int U, typename Gather>
__device__ __forceinline__ vec<T, VEC> row_dot_strided(vec<T, VEC> acc, const int32_t *s_col, const T *s_val, int a,
                                                       int e, int L, const Gather &gather) {
    using V = vec<T, VEC>;
    for (int j = a; j < e; j += U * L) {
        V bv[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j + u * L < e) bv[u] = gather(s_col[j + u * L]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j + u * L < e) vfma(acc, s_val[j + u * L], bv[u]);
    }
    return acc;
}

template <typename T, int N>
__device__ __forceinline__ void vshfl_add(vec<T, N> &acc, int off) {
#pragma unroll
    for (int i = 0; i < N; ++i) acc.v[i] += __shfl_xor(acc.v[i], off);
}

// ------------------------------------------------------------------------------------------------ row blocks
// blk[b] = {first, end | flags, j0, j1}: the virtual rows of block b and their nonzero range (<= CAP nonzeros in
// all, <= CAP_ROWS rows); blocks holding long serial rows come first in the table (they start at time 0), the rest
// in row order.  vrow_ptr indexes
// col_idx / values (the original arrays, or the window-major copy in chained mode).  B and C point at the panel's
// first column; ld is their row stride (K); kw the panel width.  Destination of virtual row v by MODE:
//   DEST_ROW   v IS C row v;
//   DEST_SPLIT vdest[v] >= 0 is v's C row, < 0 is partial slot -vdest[v]-1;
//   DEST_CHAIN vdest[v] = (d << 1) | cont with d as DEST_SPLIT; cont = 1: v continues the FMA chain of an earlier
//              column window (one launch per window), so the accumulator starts from the value stored in the
//              destination instead of 0 -- stored fp64/fp32 values are exact, so the chained result has the bits
//              of one unbroken left-to-right chain.
// XCD: workgroups are dealt round-robin over the 8 XCDs (blocks b and b+8 share one); the bijective remap gives each
// XCD one contiguous eighth of the block table, i.e. of the rows, so an XCD's L2 only ever holds the B rows of its
// own row range (speed only: any placement computes the same result).
enum { DEST_ROW = 0, DEST_SPLIT = 1, DEST_CHAIN = 2 };
constexpr int BLK_VL_FLAG = 1 << 30;          // blk[b].y: vector lanes allowed in this block
constexpr int BLK_SPLIT_FLAG = 1 << 29;       // blk[b].y: the block writes partial slots (fused combine, below)
constexpr int BLK_ROWS_MASK = BLK_SPLIT_FLAG - 1;
constexpr int CPOL_SC1 = 16;                  // buffer intrinsics' aux operand: sc1 (agent-coherent) on gfx950

typedef int32_t i32x2 __attribute__((ext_vector_type(2)));

// 4/8/16-byte sc1 store (written through to the agent-coherent level: visible to sc1 loads of other XCDs once the
// storing wave has waited vmcnt(0) -- MI355X_MICROARCH.md, inter-workgroup visibility, hand-off table row 1)
template <typename T, int N>
__device__ __forceinline__ void vstore_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off, const vec<T, N> &v) {
    constexpr int BYTES = (int)sizeof(T) * N;
    static_assert(BYTES == 4 || BYTES == 8 || BYTES == 16, "sc1 store width");
    if constexpr (BYTES == 16) {
        i32x4 r;
        __builtin_memcpy(&r, &v, 16);
        __builtin_amdgcn_raw_buffer_store_b128(r, rs, off, 0, CPOL_SC1);
    } else if constexpr (BYTES == 8) {
        i32x2 r;
        __builtin_memcpy(&r, &v, 8);
        __builtin_amdgcn_raw_buffer_store_b64(r, rs, off, 0, CPOL_SC1);
    } else {
        int32_t r;
        __builtin_memcpy(&r, &v, 4);
        __builtin_amdgcn_raw_buffer_store_b32(r, rs, off, 0, CPOL_SC1);
    }
}

template <typename T>
__device__ __forceinline__ T load_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    T v;
    if constexpr (sizeof(T) == 8) {
        const i32x2 r = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, CPOL_SC1);
        __builtin_memcpy(&v, &r, 8);
    } else {
        const int32_t r = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, CPOL_SC1);
        __builtin_memcpy(&v, &r, 4);
    }
    return v;
}

// Sum of a split row's partial slots: C[row][0..kw) = sum_q P[first_slot + q][0..kw) (row stride ld), by the whole
// workgroup: KW = min(pow2ceil(kw), 64) columns per pass x SL = 256/KW slot lanes; slot lane l sums slots l, l+SL, ...
// in order (CA independent accumulators, slot j of the lane into acc[j % CA], then added in order) so a row of
// thousands of pieces keeps CA loads in flight; then a fixed binary tree over the slot lanes in LDS.  Deterministic:
// the shape depends only on nslots and kw.  ldp(i) loads P element i.
template <typename T, typename LoadP>
__device__ __forceinline__ void combine_row(const int4 lr, T *__restrict__ C, int ld, int kw, T *red,
                                            const LoadP &ldp) {
    int KW = 1;
    while (KW < kw && KW < 64) KW <<= 1;
    const int sl_n = WG / KW;
    const int n = threadIdx.x % KW, sl = threadIdx.x / KW;
    for (int c0 = 0; c0 < kw; c0 += KW) {
        const int col = c0 + n;
        constexpr int CA = 8;
        T a[CA];
#pragma unroll
        for (int c = 0; c < CA; ++c) a[c] = T(0);
        if (col < kw) {
            int q = sl, j = 0;
            for (; q + (CA - 1) * sl_n < lr.z; q += CA * sl_n)
#pragma unroll
                for (int c = 0; c < CA; ++c) a[c] += ldp((size_t)(lr.y + q + c * sl_n) * ld + col);
            for (; q < lr.z; q += sl_n, ++j) a[j] += ldp((size_t)(lr.y + q) * ld + col);
        }
        T s = a[0];
#pragma unroll
        for (int c = 1; c < CA; ++c) s += a[c];
        red[threadIdx.x] = s;
        __syncthreads();
        for (int w = sl_n / 2; w >= 1; w /= 2) {
            if (sl < w) red[threadIdx.x] += red[threadIdx.x + w * KW];
            __syncthreads();
        }
        if (sl == 0 && col < kw) C[(size_t)lr.x * ld + col] = red[n];
        __syncthreads();
    }
}
#ifdef SPMM_STAMPS
// Diagnostic build only (lib/libspmm_hip_stamps.so, tools/small_breakdown.py): per block of the row kernel, lane 0
// stores {block start, block staged (after the staging barrier), block done (after the last row), workgroup id} in
// s_memrealtime ticks (100 MHz, one clock for the whole chip).  The shipped engine never compiles this.
static __device__ long long *g_row_stamps;
#endif
__device__ __forceinline__ int xcd_block(int w, int nb) {
    const int x = w & 7, i = w >> 3, q = nb >> 3, r = nb & 7;
    return x * q + (x < r ? x : r) + i;
}
// VL (vector lanes, SURVEY §8f "K=1 SpMV specialisation"): when a block holds fewer rows than row groups (long
// rows at small K: K=1 has 256 one-lane groups but a 2048-nonzero block holds 4 rows of 500), each row is given
// L = min(lmax, pow2floor(NG / rows)) groups; sub-lane l sums nonzeros l, l+L, ... and the L partials are added by a
// fixed xor-shuffle tree.  Deterministic, within the 1e-10 normwise contract, but not the reference's single chain:
// rows of blocks with L > 1 are reported as inexact (spmm_hip_exact_rows).  L is block-uniform; L = 1 blocks are
// exactly the plain kernel.  Only blocks flagged by the inspector (bit 30 of blk.y: all blocks when the matrix-wide
// policy chose vector lanes, else blocks made only of split-row pieces, which are inexact anyway) may use L > 1.
// PAIR (round 6, short rows): a row group takes its rows two at a time -- row r in gather slots 0..U/2-1,
// row r + NG in slots U/2..U-1 -- so two short rows share one gather round trip.  The four groups of a wave keep
// walking ADJACENT rows at the SAME slots (r, r+1, r+2, r+3 in the first half, the rows NG further in the second), so
// the texture unit still merges the B lines that similar neighbouring rows share (the in-step merge of DESIGN §6.31,
// which the packed stream of §6.32 lost).  A pair step is taken only when every group of the wave has both its rows
// within U/2 nonzeros (a wave vote, so the branch is uniform); otherwise the two rows run the plain per-row loop.
// Every row is still one FMA chain from 0 in CSR order (bit-identical).  DEST_ROW / DEST_SPLIT; blocks that take
// vector lanes (split-row pieces) run their own loop.
template <typename T, int VEC, int U, typename Gather, typename Init, typename Store>
__device__ __forceinline__ bool rows_pair_step(const int32_t *s_rp, const int32_t *s_col, const T *s_val, int jb,
                                               int r, int r2, int nrows, const Gather &gather, const Init &init,
                                               const Store &store) {
    using V = vec<T, VEC>;
    constexpr int H = U / 2;
    const int a0 = s_rp[r] - jb, e0 = s_rp[r + 1] - jb;
    const bool two = r2 < nrows;
    const int a1 = two ? s_rp[r2] - jb : 0, e1 = two ? s_rp[r2 + 1] - jb : 0;
    if (!__all(e0 - a0 <= H && e1 - a1 <= H)) return false;
    V bv[U];
#pragma unroll
    for (int u = 0; u < H; ++u)
        if (a0 + u < e0) bv[u] = gather(s_col[a0 + u]);
#pragma unroll
    for (int u = 0; u < H; ++u)
        if (a1 + u < e1) bv[H + u] = gather(s_col[a1 + u]);
    V acc0 = init(r);
#pragma unroll
    for (int u = 0; u < H; ++u)
        if (a0 + u < e0) vfma(acc0, s_val[a0 + u], bv[u]);
    store(r, acc0);
    if (two) {
        V acc1 = init(r2);
#pragma unroll
        for (int u = 0; u < H; ++u)
            if (a1 + u < e1) vfma(acc1, s_val[a1 + u], bv[H + u]);
        store(r2, acc1);
    }
    return true;
}

template <typename T, int VEC, int G, int U, int CAP, bool NTC, bool DMA, bool BUF, int MODE, bool XCD = false,
          bool VL = false, bool PAIR = false>
__global__ __launch_bounds__(WG, 4) void spmm_rows_kernel(const int32_t *__restrict__ vrow_ptr,
                                                       const int32_t *__restrict__ col_idx,
                                                       const T *__restrict__ vals,
                                                       const int4 *__restrict__ blk, int nblk,
                                                       const int32_t *__restrict__ vdest,
                                                       const T *__restrict__ B, T *__restrict__ C, T *__restrict__ P,
                                                       int ld, int kw, uint32_t b_bytes, int lmax,
                                                       int32_t *__restrict__ lr_cnt,
                                                       const int32_t *__restrict__ slot_lr,
                                                       const int4 *__restrict__ long_rows, uint32_t p_bytes) {
    constexpr int SVN = 16 / (int)sizeof(T);
    constexpr int CAPP = CAP + 4;                         // staged window starts at a 16-byte boundary
    __shared__ __attribute__((aligned(16))) int32_t s_rp[CAP_ROWS + 64];
    __shared__ __attribute__((aligned(16))) int32_t s_col[CAPP];
    __shared__ __attribute__((aligned(16))) T s_val[CAPP];
    using V = vec<T, VEC>;
    constexpr int NG = WG / G;

    const int b = XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const int tid = threadIdx.x;
#ifdef SPMM_STAMPS
    const long long st_start = __builtin_amdgcn_s_memrealtime();
#endif
    if (blockIdx.y > 0) {       // K panels of one launch (small matrices, plan.ygrid): panel blockIdx.y of width kw
        const uint32_t off = blockIdx.y * (uint32_t)kw;
        B += off, C += off;
        b_bytes -= off * (uint32_t)sizeof(T);
        if (P) P += off, p_bytes -= off * (uint32_t)sizeof(T);   // partial slots [nslots][ld]; combined afterwards
    }
    __shared__ int s_ndone;
    if (tid == 0) s_ndone = 0;
    const int4 rr = blk[b];                                 // {first, end | flags, vrow_ptr[first], vrow_ptr[end]}
    const int r0 = rr.x, r1 = rr.y & BLK_ROWS_MASK;
    const int nrows = r1 - r0;
    const int j0 = rr.z;
    const int j1 = rr.w;

    // Stage the block (col_idx / values from the 16-byte boundary jb <= j0 -- the device arrays are padded -- and the
    // virtual-row offsets).  DMA: LDS-DMA (global_load_lds, no VGPR destinations) in 1-KiB wave pieces of 16-byte
    // lanes; otherwise 16-byte non-temporal vector loads through VGPRs and ds_write.
    const int jb = j0 & ~3;
    const int cnt = j1 - jb;
    if constexpr (DMA) {
        typedef __attribute__((address_space(3))) void lds_void;
        const int wave = tid / 64, wl = tid % 64;
        const int ncp = (cnt + 255) / 256;                        // 256 int32 per KiB piece
        for (int q = wave; q < ncp; q += WG / 64) {
            const int e = q * 256 + wl * 4;
            if (e < cnt) __builtin_amdgcn_global_load_lds((const void *)(col_idx + jb + e), (lds_void *)(s_col + q * 256), 16, 0, 0);
        }
        constexpr int EPK = 1024 / (int)sizeof(T);               // values per KiB piece
        const int nvp = (cnt + EPK - 1) / EPK;
        for (int q = wave; q < nvp; q += WG / 64) {
            const int e = q * EPK + wl * SVN;
            if (e < cnt) __builtin_amdgcn_global_load_lds((const void *)(vals + jb + e), (lds_void *)(s_val + q * EPK), 16, 0, 0);
        }
        const int nrp = (nrows + 1 + 63) / 64;
        for (int q = wave; q < nrp; q += WG / 64) {
            const int i = q * 64 + wl;
            if (i <= nrows) __builtin_amdgcn_global_load_lds((const void *)(vrow_ptr + r0 + i), (lds_void *)(s_rp + q * 64), 4, 0, 0);
        }
    } else {
        // every load of the block issued into VGPRs before the first LDS write: one memory round trip per block
        typedef T tv __attribute__((ext_vector_type(SVN)));
        constexpr int NC = (CAPP / 4 + WG - 1) / WG;
        constexpr int NV = (CAPP / SVN + WG - 1) / WG;
        constexpr int NR = (CAP_ROWS + 1 + WG - 1) / WG;
        const int nc = (cnt + 3) / 4, nv = (cnt + SVN - 1) / SVN;
        i32x4 cb[NC];
        tv vb[NV];
        int rp[NR];
#pragma unroll
        for (int u = 0; u < NC; ++u)
            if (tid + u * WG < nc)
                cb[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4 *>(col_idx + jb) + tid + u * WG);
#pragma unroll
        for (int u = 0; u < NV; ++u)
            if (tid + u * WG < nv)
                vb[u] = __builtin_nontemporal_load(reinterpret_cast<const tv *>(vals + jb) + tid + u * WG);
#pragma unroll
        for (int u = 0; u < NR; ++u)
            if (tid + u * WG <= nrows) rp[u] = vrow_ptr[r0 + tid + u * WG];
#pragma unroll
        for (int u = 0; u < NC; ++u)
            if (tid + u * WG < nc) reinterpret_cast<i32x4 *>(s_col)[tid + u * WG] = cb[u];
#pragma unroll
        for (int u = 0; u < NV; ++u)
            if (tid + u * WG < nv) reinterpret_cast<tv *>(s_val)[tid + u * WG] = vb[u];
#pragma unroll
        for (int u = 0; u < NR; ++u)
            if (tid + u * WG <= nrows) s_rp[tid + u * WG] = rp[u];
    }
    __syncthreads();
#ifdef SPMM_STAMPS
    const long long st_staged = __builtin_amdgcn_s_memrealtime();
#endif

    const int lane = tid % G;
    int L = 1;
    if constexpr (VL) {
        if ((rr.y & BLK_VL_FLAG) && nrows < NG) {
            L = 1 << (31 - __builtin_clz(NG / nrows));
            L = L < lmax ? L : lmax;
        }
    }
    const int sub = (tid / G) % L;               // 0 when L = 1
    const int grp = tid / (G * L);
    const int rstep = NG / L;
    // fused combine (DEST_SPLIT with lr_cnt): partial slots are stored sc1 and the block that completes a split row
    // sums it (below), so no second launch
    const bool fuse = MODE == DEST_SPLIT && lr_cnt != nullptr;
    __amdgpu_buffer_rsrc_t prs;
    if (MODE == DEST_SPLIT) prs = __builtin_amdgcn_make_buffer_rsrc((void *)P, (short)0, (int)p_bytes, 0x00020000);
    for (int kc = 0; kc < kw; kc += G * VEC) {
        const int kk = kc + lane * VEC;
        if (kk >= kw) continue;
        const BGather<T, VEC, BUF> gather(B, kk, ld, b_bytes);
        if constexpr (PAIR && MODE != DEST_CHAIN && U > 1) if (L == 1) {   // L: block-uniform (vector-lane blocks below)
            auto init = [&](int) { return vzero<T, VEC>(); };
            auto store_row = [&](int r, const vec<T, VEC> &acc) {
                if constexpr (MODE == DEST_SPLIT) {
                    const int d = vdest[r0 + r];
                    if (fuse && d < 0)
                        vstore_sc1<T, VEC>(prs, (uint32_t)(((size_t)(-d - 1) * ld + kk) * sizeof(T)), acc);
                    else
                        vstore<T, VEC, NTC>(((d >= 0) ? C + (size_t)d * ld : P + (size_t)(-d - 1) * ld) + kk, acc);
                } else {
                    vstore<T, VEC, NTC>(C + (size_t)(r0 + r) * ld + kk, acc);
                }
            };
            for (int r = grp; r < nrows; r += 2 * rstep) {
                const int r2 = r + rstep;
                if (rows_pair_step<T, VEC, U>(s_rp, s_col, s_val, jb, r, r2, nrows, gather, init, store_row)) continue;
                store_row(r, row_dot<T, VEC, U>(vzero<T, VEC>(), s_col, s_val, s_rp[r] - jb, s_rp[r + 1] - jb, gather));
                if (r2 < nrows)
                    store_row(r2, row_dot<T, VEC, U>(vzero<T, VEC>(), s_col, s_val, s_rp[r2] - jb, s_rp[r2 + 1] - jb,
                                                     gather));
            }
            continue;
        }
        for (int r = grp; r < nrows; r += rstep) {
            T *dst;
            V acc = vzero<T, VEC>();
            bool sc1 = false;      // partial slot of a fused launch: sc1 store at byte offset poff of P
            uint32_t poff = 0;
            if constexpr (MODE == DEST_SPLIT) {
                const int d = vdest[r0 + r];
                dst = (d >= 0) ? C + (size_t)d * ld : P + (size_t)(-d - 1) * ld;
                sc1 = fuse && d < 0;
                poff = (uint32_t)(((size_t)(-d - 1) * ld + kk) * sizeof(T));
            } else if constexpr (MODE == DEST_CHAIN) {
                const int code = vdest[r0 + r];
                const int d = code >> 1;
                dst = (d >= 0) ? C + (size_t)d * ld : P + (size_t)(-d - 1) * ld;
                if ((code & 1) && sub == 0) acc = *reinterpret_cast<const V *>(dst + kk);
            } else {
                dst = C + (size_t)(r0 + r) * ld;
            }
            if (VL && L > 1) {   // block-uniform branch: L = 1 blocks run the plain unit-stride chain below
                acc = row_dot_strided<T, VEC, (U < 0 ? -U : U) / 2>(acc, s_col, s_val, s_rp[r] - jb + sub, s_rp[r + 1] - jb,
                                                                    L, gather);
                for (int off = (G * L) >> 1; off >= G; off >>= 1) vshfl_add(acc, off);   // fixed tree over sub-lanes
                if (sub == 0) {
                    if (MODE == DEST_SPLIT && sc1) vstore_sc1<T, VEC>(prs, poff, acc);
                    else vstore<T, VEC, NTC>(dst + kk, acc);
                }
            } else {
                acc = row_dot<T, VEC, U>(acc, s_col, s_val, s_rp[r] - jb, s_rp[r + 1] - jb, gather);
                if (MODE == DEST_SPLIT && sc1) vstore_sc1<T, VEC>(prs, poff, acc);
                else vstore<T, VEC, NTC>(dst + kk, acc);
            }
        }
    }

#ifdef SPMM_STAMPS
    __syncthreads();
    if (tid == 0 && g_row_stamps != nullptr && blockIdx.y == 0) {
        long long *st = g_row_stamps + (size_t)b * 4;
        st[0] = st_start;
        st[1] = st_staged;
        st[2] = __builtin_amdgcn_s_memrealtime();
        st[3] = (long long)blockIdx.x;
    }
#endif
    if constexpr (MODE == DEST_SPLIT) {
        // Fused combine.  Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility), ordering spelled out:
        //   producer  every partial is an sc1 (write-through) store -> every wave waits vmcnt(0) -> workgroup barrier
        //             -> per split row touched, ONE lane adds this block's piece count to the row's agent-scope
        //             counter.  No release fence: the payload never sits dirty in an L2 (sc1), so buffer_wbl2 would
        //             only write back unrelated lines (the guide's "(2) without an agent release").
        //   consumer  the block whose add completes the count (told by the value its add returned) -> barrier ->
        //             agent-scope ACQUIRE fence (buffer_inv sc1: this CU's L1 holds no stale partial line) ->
        //             vmcnt(0) -> barrier -> sc1 loads of the partials; then it re-arms the counter.
        // The acquire makes the consumer side independent of the sc1-load-only argument, which the guide has
        // measured for one workgroup per CU only (this kernel runs up to four).  It costs ~2 us per completing block
        // and runs only in blocks that complete a split row.
        // The pieces of a split row are consecutive virtual rows with consecutive slots (checked by the host).
        if (!fuse || !(rr.y & BLK_SPLIT_FLAG)) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int *s_done = s_rp;                    // s_rp / s_val are free after the barrier
        for (int t = tid; t < nrows; t += WG) {
            const int d = vdest[r0 + t];
            if (d >= 0) continue;
            const int sl = -d - 1;
            const int li = slot_lr[sl];
            const int4 lr = long_rows[li];
            if (t > 0 && sl > lr.y && vdest[r0 + t - 1] == d + 1) continue;   // not the first piece of its run here
            const int np = min(lr.y + lr.z - sl, nrows - t);
            const int old = __hip_atomic_fetch_add(lr_cnt + li, np, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old + np == lr.z) s_done[atomicAdd(&s_ndone, 1)] = li;
        }
        __syncthreads();
        const int nd = s_ndone;
        if (nd == 0) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        T *red = s_val;
        for (int i = 0; i < nd; ++i) {
            const int li = s_done[i];
            combine_row<T>(long_rows[li], C, ld, kw, red,
                           [&](size_t e) { return load_sc1<T>(prs, (uint32_t)(e * sizeof(T))); });
            if (tid == 0) __hip_atomic_store(lr_cnt + li, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ------------------------------------------------------------------------------------------------ LDS B tiles
// TILE mode: for rows that share their columns -- similar consecutive rows (cross-row similarity) or
// dense column bands -- the row kernel re-gathers the same B row once per nonzero through L1/L2 (~15 TB/s chip-wide,
// the TA/L2 request path), while the LDS reads at ~150 TB/s.  A TILE is up to RMAX consecutive C rows; the
// inspector lists the union U of their columns (sorted) and cuts it into CHUNKS of <= UCB bytes of B rows and <=
// CAPA entries.  Per chunk the workgroup stages (through VGPRs) the chunk's B rows and the chunk's entries from a
// chunk-major copy of A: values and 16-bit byte offsets of their B rows in the staged image, row by row, each
// row's segment padded to a multiple of 4 entries with (value -0, the all-zero B row) -- fma(-0, +0, acc) == acc
// exactly for every acc, -0 included (a chain can reach -0 through an underflowing product) -- so the inner loop
// reads 4 offsets and 4 values
// per step with no predication.  Row group g (G lanes, VEC columns each) owns rows g, g+NG, ... of the tile and
// carries their accumulators in registers across chunks; chunks go in column order and each row's columns are
// sorted, so every row is still ONE fused multiply-add chain from 0 in CSR order -- bit-identical to the
// reference, like an unsplit row of the row kernel.  Descriptors:
//   tiles[t]  = {first C row, rows, first chunk, chunks}
//   tchunk[c] = {first union column (tcol), columns, first entry (tval/toff, 8-aligned), first segment offset
//               (tseg, 8-aligned)}; chunk c's staged sizes are the gaps to chunk c+1 (a sentinel ends the table)
//   tseg[...] = per chunk, rows+1 entry offsets (relative to the chunk's first entry; multiples of 4)
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

// LDS budget of one tile workgroup (3 per CU: 3 x 53,248 B with the 512-B allocation granule).
#ifndef SPMM_TILE_WGS
#define SPMM_TILE_WGS 3                        // A/B builds only: tile workgroups per CU (LDS budget and launch bounds)
#endif
constexpr int TILE_WGS = SPMM_TILE_WGS;
constexpr int TILE_LDS_BYTES = TILE_WGS == 3 ? 53248 : TILE_WGS == 4 ? 40448 : 79872;
constexpr int TILE_DMAX = 64;                  // chunk descriptors per tile (incl. the end marker)

template <typename T, int VEC, int G, int UCB, int CAPA, int RMAX>
struct TileBuf {
    vec<T, VEC> b[UCB / 16 + G];                  // staged B rows, then the zero row (byte offset UCB)
    vec<T, 4> v[CAPA / 4];                        // the chunk's values, 4 per step
    u16x4 o[CAPA / 4];                            // byte offset (in b) of each value's B row, 4 per step
    uint16_t s[RMAX + 8];                         // row segment offsets (entries)
};
// Union columns one tile may hold in LDS (the rest of the budget after two chunk buffers and the descriptors).
template <typename T, int VEC, int G, int UCB, int CAPA, int RMAX>
constexpr int tile_colmax() {
    return (int)((TILE_LDS_BYTES - 2 * (int)sizeof(TileBuf<T, VEC, G, UCB, CAPA, RMAX>) - TILE_DMAX * 16) / 4) & ~63;
}

// One row segment [a4, e4) (in steps of 4 entries), two steps per iteration: the offsets and values of both steps
// are read together, then the 8 B rows, so each pair of steps waits on two LDS round trips (offsets, B rows).
// `bl` = the lane's byte address in the B image.
template <typename T, int VEC, typename Buf>
__device__ __forceinline__ void tile_step(vec<T, VEC> &acc, const char *bb, int bl, const u16x4 o,
                                          const vec<T, 4> &av) {
    using V = vec<T, VEC>;             // VEC = the lane's values of one B row (16 or 32 bytes)
    const V b0 = *reinterpret_cast<const V *>(bb + (bl + (int)o.x));
    const V b1 = *reinterpret_cast<const V *>(bb + (bl + (int)o.y));
    const V b2 = *reinterpret_cast<const V *>(bb + (bl + (int)o.z));
    const V b3 = *reinterpret_cast<const V *>(bb + (bl + (int)o.w));
    vfma(acc, av.v[0], b0);
    vfma(acc, av.v[1], b1);
    vfma(acc, av.v[2], b2);
    vfma(acc, av.v[3], b3);
}

template <typename T, int VEC, typename Buf>
__device__ __forceinline__ vec<T, VEC> tile_dot(vec<T, VEC> acc, const Buf &cur, int bl, int a4, int e4) {
    using V = vec<T, VEC>;
    const char *bb = reinterpret_cast<const char *>(cur.b);
    int t = a4;
    for (; t + 2 <= e4; t += 2) {
        const u16x4 o0 = cur.o[t], o1 = cur.o[t + 1];
        const vec<T, 4> v0 = cur.v[t], v1 = cur.v[t + 1];
        const V b0 = *reinterpret_cast<const V *>(bb + (bl + (int)o0.x));
        const V b1 = *reinterpret_cast<const V *>(bb + (bl + (int)o0.y));
        const V b2 = *reinterpret_cast<const V *>(bb + (bl + (int)o0.z));
        const V b3 = *reinterpret_cast<const V *>(bb + (bl + (int)o0.w));
        const V b4 = *reinterpret_cast<const V *>(bb + (bl + (int)o1.x));
        const V b5 = *reinterpret_cast<const V *>(bb + (bl + (int)o1.y));
        const V b6 = *reinterpret_cast<const V *>(bb + (bl + (int)o1.z));
        const V b7 = *reinterpret_cast<const V *>(bb + (bl + (int)o1.w));
        vfma(acc, v0.v[0], b0);
        vfma(acc, v0.v[1], b1);
        vfma(acc, v0.v[2], b2);
        vfma(acc, v0.v[3], b3);
        vfma(acc, v1.v[0], b4);
        vfma(acc, v1.v[1], b5);
        vfma(acc, v1.v[2], b6);
        vfma(acc, v1.v[3], b7);
    }
    if (t < e4) tile_step<T, VEC, Buf>(acc, bb, bl, cur.o[t], cur.v[t]);
    return acc;
}

// LDS-DMA of `bytes` (multiple of 16) from src to the LDS at dst by the whole workgroup, 1-KiB wave pieces.
__device__ __forceinline__ void dma_to_lds(const char *src, char *dst, int bytes, int wave, int wl) {
    typedef __attribute__((address_space(3))) void lds_void;
    for (int q = wave; q * 1024 < bytes; q += WG / 64) {
        const int off = q * 1024 + wl * 16;
        if (off < bytes) __builtin_amdgcn_global_load_lds((const void *)(src + off), (lds_void *)(dst + q * 1024), 16, 0, 0);
    }
}

// Prologue: the tile's chunk descriptors and its whole union of columns land in LDS by one DMA round trip, so the
// chunk loop never waits on a global or scalar load.  Chunk pipeline (double-buffered LDS, register staged): at the
// top of step c a barrier makes chunk c visible to every wave and frees chunk c-1's buffer; the workgroup then
// issues chunk c+1's global loads into VGPRs (B rows through the LDS column list; values, offsets and segment
// offsets non-temporal), computes chunk c from LDS while they land, and writes them to the free buffer.  Register
// staging, not LDS-DMA: a DMA in flight makes the compiler wait for lgkmcnt(0) at every LDS read of the compute
// (measured: 0.243 vs 0.253 ms on the 39120 x 500 dense band).
//
// S = 16-byte pieces of a B row per compute lane (1, or 2 / 4 = "wide" lanes): G/S lanes per row group and RPG rows
// per group (the host passes RPG / S, so the tile geometry NG x RPG -- and with it the inspector's layout -- is the
// same); wide lanes divide the broadcast reads of values and offsets per FMA by S.  Staging moves 16-byte pieces.
template <typename T, int VEC, int G, int RPG, int UCB, int CAPA, bool NTC, bool XCD, int S = 1>
__global__ __launch_bounds__(WG, TILE_WGS) void spmm_tile_kernel(const int4 *__restrict__ tiles,
                                                          const int4 *__restrict__ tchunk,
                                                          const int32_t *__restrict__ tcol,
                                                          const uint16_t *__restrict__ tseg,
                                                          const T *__restrict__ tval,
                                                          const uint16_t *__restrict__ toff,
                                                          const T *__restrict__ B, T *__restrict__ C, int ld,
                                                          long long *__restrict__ stamps) {
    constexpr int GC = G / S;                      // compute lanes per row group
    constexpr int NG = WG / GC;
    constexpr int RMAX = NG * RPG;
    static_assert(S == 1 || S == 2 || S == 4, "16-, 32- or 64-byte compute lanes");
    static_assert(GC >= 1 && G % S == 0, "lanes");
    constexpr int NPL = UCB / 16 / WG;             // B pieces per lane per chunk
    constexpr int NPV = (CAPA * (int)sizeof(T) / 16 + WG - 1) / WG;   // value pieces per lane
    constexpr int NPO = (CAPA * 2 / 16 + WG - 1) / WG;                // offset pieces per lane
    constexpr int NPS = ((RMAX + 8) * 2 / 16 + WG - 1) / WG;          // segment-offset pieces per lane
    constexpr int LPPR = __builtin_ctz(G);         // 16-byte pieces per staged B row == G (power of two, host)
    static_assert(UCB % (16 * WG) == 0, "UCB must be a multiple of 4 KiB");
    static_assert(VEC * sizeof(T) == 16, "16-byte lanes");
    using VW = vec<T, VEC * S>;                    // a compute lane's slice of a B / C row
    using Buf = TileBuf<T, VEC, G, UCB, CAPA, RMAX>;
    constexpr int COLMAX = tile_colmax<T, VEC, G, UCB, CAPA, RMAX>();
    __shared__ __attribute__((aligned(16))) Buf sbuf0;
    __shared__ __attribute__((aligned(16))) Buf sbuf1;
    __shared__ __attribute__((aligned(16))) int4 sdesc[TILE_DMAX];
    __shared__ __attribute__((aligned(16))) int32_t scol[COLMAX];

    const int b = XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const int4 tl = tiles[b];
    const int tid = threadIdx.x, wave = tid / 64, wl = tid % 64;
    const int grp = tid / GC, lane = tid % GC;
    if (tid < G) {
        sbuf0.b[UCB / 16 + tid] = vzero<T, VEC>();
        sbuf1.b[UCB / 16 + tid] = vzero<T, VEC>();
    }
    VW acc[RPG];
#pragma unroll
    for (int q = 0; q < RPG; ++q) acc[q] = vzero<T, VEC * S>();
    // measurement stamps (stamps != nullptr): s_memtime returns through the lgkm counter out of order, so each
    // read is waited for at once -- a pending one would make every LDS wait of the chunk loop a full drain
    auto stamp = [&]() -> long long {
        const long long t = (long long)__builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_waitcnt(0xc07f);        // lgkmcnt(0)
        return t;
    };
    const long long t_start = stamps ? stamp() : 0;

    // prologue: descriptors [tl.z, tl.z + tl.w] (the last one is the next chunk: sizes) and the union columns
    const int col0 = tchunk[tl.z].x, col1 = tchunk[tl.z + tl.w].x;
    dma_to_lds((const char *)(tchunk + tl.z), (char *)sdesc, (tl.w + 1) * 16, wave, wl);
    {   // tcol is 64-B padded on the device; copy from the 16-B boundary below col0
        const int c0a = col0 & ~3;
        dma_to_lds((const char *)(tcol + c0a), (char *)scol, ((col1 - c0a + 3) & ~3) * 4, wave, wl);
    }
    const int cbase = col0 & ~3;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const char *Bb = reinterpret_cast<const char *>(B);
    const size_t ldb = (size_t)ld * sizeof(T);
    // Every lane loads unconditionally (piece indices clamped into the chunk) and only the LDS writes are
    // predicated: predicated loads leave partly defined registers that make the compiler wait for vmcnt(0) in
    // front of every later load.
    i32x4 rb[NPL], rv[NPV], ro[NPO], rs[NPS];
    int nb = 0, nv = 0, no = 0, ns = 0;            // 16-byte pieces of the chunk in flight
    auto load = [&](int c) {
        const int4 ch = sdesc[c], cn = sdesc[c + 1];
        nb = ch.y << LPPR;
        nv = (cn.z - ch.z) * (int)sizeof(T) / 16;
        no = (cn.z - ch.z) * 2 / 16;
        ns = (cn.w - ch.w) * 2 / 16;
        const i32x4 *gv = reinterpret_cast<const i32x4 *>(tval + ch.z);
        const i32x4 *go = reinterpret_cast<const i32x4 *>(toff + ch.z);
        const i32x4 *gs = reinterpret_cast<const i32x4 *>(tseg + ch.w);
#pragma unroll
        for (int it = 0; it < NPL; ++it) {
            const int p = min(it * WG + tid, nb - 1);
            const int row = scol[ch.x - cbase + (p >> LPPR)];
            rb[it] = *reinterpret_cast<const i32x4 *>(Bb + (size_t)row * ldb + (p & (G - 1)) * 16);
        }
#pragma unroll
        for (int it = 0; it < NPV; ++it) rv[it] = __builtin_nontemporal_load(gv + min(it * WG + tid, nv - 1));
#pragma unroll
        for (int it = 0; it < NPO; ++it) ro[it] = __builtin_nontemporal_load(go + min(it * WG + tid, no - 1));
#pragma unroll
        for (int it = 0; it < NPS; ++it) rs[it] = __builtin_nontemporal_load(gs + min(it * WG + tid, ns - 1));
    };
    auto store = [&](Buf &bf) {
#pragma unroll
        for (int it = 0; it < NPL; ++it)
            if (it * WG + tid < nb) reinterpret_cast<i32x4 *>(bf.b)[it * WG + tid] = rb[it];
#pragma unroll
        for (int it = 0; it < NPV; ++it)
            if (it * WG + tid < nv) reinterpret_cast<i32x4 *>(bf.v)[it * WG + tid] = rv[it];
#pragma unroll
        for (int it = 0; it < NPO; ++it)
            if (it * WG + tid < no) reinterpret_cast<i32x4 *>(bf.o)[it * WG + tid] = ro[it];
#pragma unroll
        for (int it = 0; it < NPS; ++it)
            if (it * WG + tid < ns) reinterpret_cast<i32x4 *>(bf.s)[it * WG + tid] = rs[it];
    };
    long long t_wait = 0, t_comp = 0, t_mark = 0;        // measurement only (stamps != nullptr)
    auto step = [&](const Buf &cur, Buf &nxt, int c) {
        if (stamps) t_mark = stamp();
        __syncthreads();                                     // chunk c visible to every wave; c-1's buffer is free
        if (stamps) {
            const long long t = stamp();
            t_wait += t - t_mark;
            t_mark = t;
        }
        // the last chunk reloads itself into the free buffer (unconditional, so no load is ever left in flight
        // on a path the compiler cannot rule out)
        load(min(c + 1, tl.w - 1));
#pragma unroll
        for (int q = 0; q < RPG; ++q) {
            const int r = grp + q * NG;
            if (r < tl.y) acc[q] = tile_dot<T, VEC * S>(acc[q], cur, lane * 16 * S, cur.s[r] >> 2, cur.s[r + 1] >> 2);
        }
        store(nxt);
        if (stamps) t_comp += stamp() - t_mark;
    };
    load(0);
    store(sbuf0);
    for (int c = 0; c < tl.w; c += 2) {
        step(sbuf0, sbuf1, c);
        if (c + 1 < tl.w) step(sbuf1, sbuf0, c + 1);
    }
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
        const int r = grp + q * NG;
        if (r < tl.y) vstore<T, VEC * S, NTC>(C + (size_t)(tl.x + r) * ld + lane * VEC * S, acc[q]);
    }
    if (stamps && tid == 0) {
        long long *st = stamps + (size_t)b * 4;
        st[0] = t_start;
        st[1] = stamp();
        st[2] = t_wait;
        st[3] = t_comp;
    }
}

// long_rows[b] = {row, first_slot, nslots, 0}: C[row][n] = sum of the row's partial slots P[first_slot + q][n].
// Separate combine launch (column-window plans, or partials beyond 4 GiB): one workgroup per split row.
template <typename T>
__global__ __launch_bounds__(WG) void spmm_combine_kernel(const int4 *__restrict__ long_rows,
                                                          const T *__restrict__ P, T *__restrict__ C, int K) {
    __shared__ T red[WG];
    combine_row<T>(long_rows[blockIdx.x], C, K, K, red, [&](size_t e) { return P[e]; });
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
