// LDS gather probe: cycles per ds_read_b128 wave instruction for a given
// per-lane 16-B slot pattern (a table of 64-lane patterns, cycled), every CU
// busy, 512-thread blocks, 32 KB of LDS per block.  Test tooling only
// (tools/lds_probe.py): sizes the bank-conflict cost of serving bilinear
// taps from LDS.
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void lds_probe(const unsigned *__restrict__ pat, int npat, int iters,
                                                 float *__restrict__ out) {
    __shared__ f32x4 buf[2048];  // 32 KB
    for (int i = threadIdx.x; i < 2048; i += 512) buf[i] = f32x4{(float)i, 1.f, 2.f, 3.f};
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int p = (wave * 7 + blockIdx.x) % npat;
    unsigned o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) o[u] = pat[((p + u) % npat) * 64 + lane];
    for (int it = 0; it < iters; ++it) {  // a uniform shift keeps each pattern's bank conflicts
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += buf[(o[u] + (unsigned)it) & 2047];
    }
    if (acc[0] == -1.0f) out[blockIdx.x * 512 + threadIdx.x] = acc[1];
}

extern "C" int lds_probe_run(const unsigned *pat, int npat, int iters, float *out, int blocks, void *stream) {
    hipLaunchKernelGGL(lds_probe, dim3(blocks), dim3(512), 0, (hipStream_t)stream, pat, npat, iters, out);
    return (int)hipGetLastError();
}
