// Probe: float4 device-copy variants (the measured-roofline calibration kernel).
//   hipcc --offload-arch=gfx950 -O3 tools/copy_probe.hip -o copy_probe && ./copy_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int U>
__global__ __launch_bounds__(256) void grid_stride(const float4 *__restrict__ s, float4 *__restrict__ d, long long n4) {
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long b = (long long)blockIdx.x * 256 * U + threadIdx.x; b < n4; b += stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (b + u * 256 < n4) v[u] = s[b + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) if (b + u * 256 < n4) d[b + u * 256] = v[u];
    }
}

__global__ __launch_bounds__(256) void one_per_thread(const float4 *__restrict__ s, float4 *__restrict__ d, long long n4) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) d[i] = s[i];
}

template <int U>
__global__ __launch_bounds__(256) void chunked(const float4 *__restrict__ s, float4 *__restrict__ d, long long n4) {
    const long long b = ((long long)blockIdx.x * U) * 256 + threadIdx.x;
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (b + u * 256 < n4) v[u] = s[b + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) if (b + u * 256 < n4) d[b + u * 256] = v[u];
}

int main() {
    const size_t bytes = 1ull << 30;
    const long long n4 = bytes / 16;
    float4 *s, *d;
    hipMalloc(&s, bytes);
    hipMalloc(&d, bytes);
    hipMemset(s, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, auto launch) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %7.1f GB/s\n", name, 2.0 * bytes * 20 / (ms * 1e-3) / 1e9);
    };
    run("one_per_thread", [&] { one_per_thread<<<(unsigned)((n4 + 255) / 256), 256>>>(s, d, n4); });
    run("chunked U=2", [&] { chunked<2><<<(unsigned)((n4 + 511) / 512), 256>>>(s, d, n4); });
    run("chunked U=4", [&] { chunked<4><<<(unsigned)((n4 + 1023) / 1024), 256>>>(s, d, n4); });
    run("chunked U=8", [&] { chunked<8><<<(unsigned)((n4 + 2047) / 2048), 256>>>(s, d, n4); });
    for (int bpc : {4, 8, 16, 32}) {
        char nm[64];
        snprintf(nm, 64, "grid_stride U=4 %d/CU", bpc);
        run(nm, [&] { grid_stride<4><<<256 * bpc, 256>>>(s, d, n4); });
        snprintf(nm, 64, "grid_stride U=8 %d/CU", bpc);
        run(nm, [&] { grid_stride<8><<<256 * bpc, 256>>>(s, d, n4); });
    }
    return 0;
}
