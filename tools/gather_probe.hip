// tools/gather_probe.hip -- measurement-only probe: how fast does MI355X gather 256-byte rows (fp64 K=32 B rows)?
// Each 16-lane group walks a contiguous slice of an index stream, issues U 16-byte loads per lane (one 256-B row
// per group load) and sums them; no A values, no rows, no C.  Tables sized for L2 / Infinity Cache / HBM, with
// uniformly random indices or a given index stream (e.g. a matrix's col_idx).  Built into
// spmm-research_amd/lib/libgather_probe.so, driven by tools/gather_probe.py.  Not part of the engine.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

// A workgroup stages 2048 consecutive indices into LDS (as the SpMM kernel stages col_idx), then each of its 16
// row groups walks 128 of them: U gathers in flight, summed.
template <int U>
__global__ __launch_bounds__(256) void gather_sum(const int32_t *__restrict__ idx, int64_t n,
                                                  const f64x2 *__restrict__ table, f64x2 *__restrict__ out,
                                                  int64_t per_group) {
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
        for (int u = 0; u < U; ++u) v[u] = table[(int64_t)s_idx[j + u] * 16 + lane];
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    out[((int64_t)blockIdx.x * 256 + threadIdx.x)] = acc;
}

__global__ void fill_random_idx(int32_t *idx, int64_t n, int64_t rows, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ULL ^ seed;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ULL; x ^= x >> 29; x *= 0x94D049BB133111EBULL; x ^= x >> 32;
    idx[i] = (int32_t)(x % (uint64_t)rows);
}

__global__ void stream_read(const f64x2 *__restrict__ a, int64_t n, f64x2 *__restrict__ out) {
    f64x2 acc = {0, 0};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += a[i];
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" {
int probe_gather(const int32_t *idx, int64_t n, const void *table, void *out, int64_t per_group, int u,
                 void *stream) {
    (void)per_group;
    const unsigned blocks = (unsigned)((n + 2047) / 2048);
    hipStream_t s = (hipStream_t)stream;
    switch (u) {
        case 4: gather_sum<4><<<blocks, 256, 0, s>>>(idx, n, (const f64x2 *)table, (f64x2 *)out, per_group); break;
        case 8: gather_sum<8><<<blocks, 256, 0, s>>>(idx, n, (const f64x2 *)table, (f64x2 *)out, per_group); break;
        default: gather_sum<16><<<blocks, 256, 0, s>>>(idx, n, (const f64x2 *)table, (f64x2 *)out, per_group); break;
    }
    return (int)hipGetLastError();
}
int probe_fill_idx(int32_t *idx, int64_t n, int64_t rows, uint64_t seed, void *stream) {
    fill_random_idx<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(idx, n, rows, seed);
    return (int)hipGetLastError();
}
int probe_stream(const void *a, int64_t n16, void *out, int blocks, void *stream) {
    stream_read<<<blocks, 256, 0, (hipStream_t)stream>>>((const f64x2 *)a, n16, (f64x2 *)out);
    return (int)hipGetLastError();
}
}
