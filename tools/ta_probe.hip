// Vector-memory gather probe: cycles per wave load instruction on gfx950 as a
// function of access width and of how many distinct cache lines the 64 lanes
// touch.  Results guide the voxelize kernel's layout (tools/ta_probe.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int WIDTH>
struct VecT;
template <> struct VecT<4> { using T = float; };
template <> struct VecT<8> { using T = float2; };
template <> struct VecT<16> { using T = float4; };

__device__ __forceinline__ float sum(float v) { return v; }
__device__ __forceinline__ float sum(float2 v) { return v.x + v.y; }
__device__ __forceinline__ float sum(float4 v) { return v.x + v.y + v.z + v.w; }

// lane_off: byte offset of each lane inside a 'window' (precomputed table, 64
// entries per pattern); each iteration the window base moves by `step` bytes
// modulo `span` (to choose L1- vs L2-resident footprints).
template <int WIDTH, int UNROLL>
__global__ __launch_bounds__(256) void probe(const unsigned char *__restrict__ buf, const unsigned *__restrict__ lane_off,
                                             int iters, unsigned step, unsigned span, float *__restrict__ out) {
    using T = typename VecT<WIDTH>::T;
    const int lane = threadIdx.x & 63;
    const unsigned off = lane_off[lane];
    const unsigned wave_salt = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 4096u;
    float acc = 0.f;
    unsigned base = wave_salt % span;
    for (int i = 0; i < iters; ++i) {
        T v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const unsigned a = (base + (unsigned)u * step) % span;
            v[u] = *reinterpret_cast<const T *>(buf + a + off);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc += sum(v[u]);
        base = (base + UNROLL * step) % span;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

extern "C" int ta_probe(int width, const void *buf, const unsigned *lane_off, int iters, unsigned step, unsigned span,
                        float *out, int blocks, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (width == 4)
        hipLaunchKernelGGL((probe<4, 16>), dim3(blocks), dim3(256), 0, s, (const unsigned char *)buf, lane_off, iters,
                           step, span, out);
    else if (width == 8)
        hipLaunchKernelGGL((probe<8, 16>), dim3(blocks), dim3(256), 0, s, (const unsigned char *)buf, lane_off, iters,
                           step, span, out);
    else
        hipLaunchKernelGGL((probe<16, 16>), dim3(blocks), dim3(256), 0, s, (const unsigned char *)buf, lane_off,
                           iters, step, span, out);
    return (int)hipGetLastError();
}
