// Streaming copy used as the measured HBM roofline (bench.py "measured_copy_gbs").
//
// The roofline of the voxelize op is HBM bandwidth; the
// nominal 8 TB/s is not reachable by any access pattern, so the bench also
// reports its fraction of what a plain float4 copy achieves on the same box
// (MI355X_MICROARCH.md: 6.29 TB/s measured).  One 16-B element per thread:
// measured on the box (tools/copy_probe.hip, 1 GiB) 6.31 TB/s, against 5.2-5.7
// with 2-8 elements per thread or grid-stride loops.  Not on the product path.
#include "fvp_device.h"

namespace fvp {

__global__ __launch_bounds__(256) void copy_f4_kernel(const float4 *__restrict__ src, float4 *__restrict__ dst,
                                                      long long n4) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) dst[i] = src[i];
}

}  // namespace fvp

extern "C" int fvp_copy_f4(const void *src, void *dst, size_t bytes, void *stream) {
    if (!src || !dst) return FVP_ERR_NULL;
    if (bytes % 16) return FVP_ERR_SHAPE;
    const long long n4 = (long long)(bytes / 16);
    if (n4 == 0) return FVP_OK;
    const long long blocks = (n4 + 255) / 256;
    if (blocks > 0x7fffffffLL) return FVP_ERR_SHAPE;
    hipLaunchKernelGGL(fvp::copy_f4_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4 *>(src), reinterpret_cast<float4 *>(dst), n4);
    return (int)hipGetLastError();
}
