// tools/mfma_chain_probe.hip -- measurement only: is a matrix-core instruction a chain of fused multiply-adds in k
// order?  (the engine's matrix-core tiles are bit-exact only if it is.)  One wave per
// problem: D = MFMA(A, B, C) for a 16x16x4 tile, written out with each lane's operands so the host can match every
// output against candidate orders (tools/mfma_chain_probe.py).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/mfma_chain_probe.hip -o spmm-research_amd/lib/libmfma_chain_probe.so
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// per problem p: a[p][64] (lane l's A operand), b[p][64] (lane l's B operand), c[p][64][4] (lane l's accumulator),
// d[p][64][4] the result
__global__ void probe_f32(const float *a, const float *b, const float *c, float *d, int n) {
    const int p = blockIdx.x, l = threadIdx.x;
    if (p >= n) return;
    f32x4 acc = {c[(p * 64 + l) * 4], c[(p * 64 + l) * 4 + 1], c[(p * 64 + l) * 4 + 2], c[(p * 64 + l) * 4 + 3]};
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[p * 64 + l], b[p * 64 + l], acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) d[(p * 64 + l) * 4 + i] = acc[i];
}

__global__ void probe_f64(const double *a, const double *b, const double *c, double *d, int n) {
    const int p = blockIdx.x, l = threadIdx.x;
    if (p >= n) return;
    f64x4 acc = {c[(p * 64 + l) * 4], c[(p * 64 + l) * 4 + 1], c[(p * 64 + l) * 4 + 2], c[(p * 64 + l) * 4 + 3]};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[p * 64 + l], b[p * 64 + l], acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) d[(p * 64 + l) * 4 + i] = acc[i];
}

extern "C" int chain_probe(int f64, const void *a, const void *b, const void *c, void *d, int n, void *stream) {
    if (f64)
        probe_f64<<<n, 64, 0, (hipStream_t)stream>>>((const double *)a, (const double *)b, (const double *)c,
                                                     (double *)d, n);
    else
        probe_f32<<<n, 64, 0, (hipStream_t)stream>>>((const float *)a, (const float *)b, (const float *)c,
                                                     (float *)d, n);
    return (int)hipGetLastError();
}
