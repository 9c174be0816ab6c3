// tools/shape_probe.hip -- measurement-only probe (round 6, verdict r05 item 1): the row kernel's exact B access shape
// (spmm_rows_kernel, csrc/spmm_kernels.hpp: 16-lane row groups x 16-byte lanes = one 256-B B row per group load,
// 4 row groups per wave instruction, the block's columns read from LDS, U = 16 gathers in flight per group) on a
// real matrix's column stream, with the parts of the kernel switched on one at a time:
//   flat        every 16-lane group walks 128 consecutive nonzeros of the stream (no rows, all 16 groups busy);
//   rows        the kernel's blocks: at most CAPN nonzeros (and their row offsets) staged into LDS per 256-lane
//               workgroup, row group g sums rows g, g+16, ... (a row = one chain of U-gather batches), one 256-B C row
//               stored per row -- gather-only (sum of B rows) or with the A values (FMA chain, as the kernel);
//   CAPN 8192   the same with 4x the LDS window (16 rows of 500 per block: all four waves busy, 1 workgroup per CU).
// Built into spmm-research_amd/lib/libshape_probe.so, driven by tools/shape_probe.py.  Not part of the engine.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int U>
__global__ __launch_bounds__(256) void flat_probe(const int32_t *__restrict__ idx, int64_t n,
                                                  const f64x2 *__restrict__ B, f64x2 *__restrict__ out) {
    __shared__ int32_t s_idx[2048];
    const int lane = threadIdx.x % 16, grp = threadIdx.x / 16;
    const int64_t b0 = (int64_t)blockIdx.x * 2048;
    for (int i = threadIdx.x; i < 2048; i += 256) s_idx[i] = (b0 + i < n) ? idx[b0 + i] : idx[n - 1];
    __syncthreads();
    f64x2 acc = {0, 0};
    const int a = grp * 128;
    for (int j = a; j < a + 128; j += U) {
        f64x2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = B[(int64_t)s_idx[j + u] * 16 + lane];
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

// blk[b] = first piece of block b (pieces = rows cut at CAPN nonzeros); pp = piece offsets into col/val
template <int U, int CAPN, bool FMA>
__global__ __launch_bounds__(256) void rows_probe(const int32_t *__restrict__ blk, const int32_t *__restrict__ pp,
                                                  const int32_t *__restrict__ col, const double *__restrict__ val,
                                                  const f64x2 *__restrict__ B, f64x2 *__restrict__ C) {
    __shared__ int32_t s_col[CAPN];
    __shared__ double s_val[FMA ? CAPN : 2];
    __shared__ int32_t s_rp[CAPN / 4 + 1];
    const int p0 = blk[blockIdx.x], p1 = blk[blockIdx.x + 1];
    const int np = p1 - p0;
    const int j0 = pp[p0], j1 = pp[p1];
    for (int i = threadIdx.x; i < j1 - j0; i += 256) {
        s_col[i] = __builtin_nontemporal_load(col + j0 + i);
        if constexpr (FMA) s_val[i] = __builtin_nontemporal_load(val + j0 + i);
    }
    for (int i = threadIdx.x; i <= np; i += 256) s_rp[i] = pp[p0 + i] - j0;
    __syncthreads();
    const int lane = threadIdx.x % 16, grp = threadIdx.x / 16;
    for (int r = grp; r < np; r += 16) {
        f64x2 acc = {0, 0};
        const int a = s_rp[r], e = s_rp[r + 1];
        for (int j = a; j < e; j += U) {
            f64x2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (j + u < e) v[u] = B[(int64_t)s_col[j + u] * 16 + lane];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (j + u < e) {
                    if constexpr (FMA) {
                        acc.x = __builtin_fma(s_val[j + u], v[u].x, acc.x);
                        acc.y = __builtin_fma(s_val[j + u], v[u].y, acc.y);
                    } else {
                        acc += v[u];
                    }
                }
        }
        __builtin_nontemporal_store(acc, C + (int64_t)(p0 + r) * 16 + lane);
    }
}

extern "C" {
int probe_flat(const int32_t *idx, int64_t n, const void *B, void *out, void *stream) {
    flat_probe<16><<<(unsigned)((n + 2047) / 2048), 256, 0, (hipStream_t)stream>>>(idx, n, (const f64x2 *)B,
                                                                                   (f64x2 *)out);
    return (int)hipGetLastError();
}
// variant: 0 rows gather-only CAPN 2048, 1 rows FMA CAPN 2048, 2 rows FMA CAPN 8192
int probe_rows(int variant, const int32_t *blk, int nblk, const int32_t *pp, const int32_t *col, const double *val,
               const void *B, void *C, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (variant) {
        case 0: rows_probe<16, 2048, false><<<nblk, 256, 0, s>>>(blk, pp, col, val, (const f64x2 *)B, (f64x2 *)C); break;
        case 1: rows_probe<16, 2048, true><<<nblk, 256, 0, s>>>(blk, pp, col, val, (const f64x2 *)B, (f64x2 *)C); break;
        default: rows_probe<16, 8192, true><<<nblk, 256, 0, s>>>(blk, pp, col, val, (const f64x2 *)B, (f64x2 *)C); break;
    }
    return (int)hipGetLastError();
}
}
