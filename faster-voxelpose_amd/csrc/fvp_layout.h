// Channels-last heatmap layout shared by the whole-space and per-person
// gathers (see fvp_voxelize.hip for why): [b][V][H*W][JP] fp32, JP = 4*LPV,
// joints zero padded; out-of-image taps read 0 through a buffer descriptor's
// range check.
#pragma once

#include "fvp_device.h"

namespace fvp {

constexpr unsigned kOOB = 0x80000000u;  // beyond any descriptor range -> loads return 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void *base, unsigned bytes) {
    const unsigned long long p = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
    void *b = (void *)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// -- layout pass ----------------------------------------------------------------
// thread = (pixel, joint quad q): reads joints 4q..4q+3 of one pixel (the lanes
// of a wave cover 64/LPV consecutive pixels -> coalesced plane reads), writes
// one float4 (a wave writes a contiguous 1 KiB run).
template <int LPV, typename T>
__global__ __launch_bounds__(256) void heatmaps_to_cl_kernel(const T *__restrict__ hm, float4 *__restrict__ cl, int J,
                                                             int HW, long long total_px) {
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long pxg = gid / LPV;
    const int q = (int)(gid - pxg * LPV);
    if (pxg >= total_px) return;
    const long long bv = pxg / HW;
    const int pix = (int)(pxg - bv * HW);
    const T *__restrict__ src = hm + (size_t)bv * J * HW + pix;
    const int j = 4 * q;
    float4 o;
    o.x = (j + 0 < J) ? to_f32(src[(size_t)(j + 0) * HW]) : 0.f;
    o.y = (j + 1 < J) ? to_f32(src[(size_t)(j + 1) * HW]) : 0.f;
    o.z = (j + 2 < J) ? to_f32(src[(size_t)(j + 2) * HW]) : 0.f;
    o.w = (j + 3 < J) ? to_f32(src[(size_t)(j + 3) * HW]) : 0.f;
    cl[pxg * LPV + q] = o;
}

inline int lanes_per_voxel(int J) { return J <= 4 ? 1 : J <= 8 ? 2 : J <= 16 ? 4 : 8; }

inline size_t cl_frame_bytes(int V, int J, int H, int W) {
    return (size_t)V * H * W * 4 * lanes_per_voxel(J) * sizeof(float);
}

template <int LPV, typename T>
inline void launch_layout(const T *hm, int nb, int V, int J, int H, int W, float *cl, hipStream_t s) {
    const long long px = (long long)nb * V * H * W;
    const long long threads = px * LPV;
    hipLaunchKernelGGL((heatmaps_to_cl_kernel<LPV, T>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, hm,
                       reinterpret_cast<float4 *>(cl), J, H * W, px);
}

}  // namespace fvp
