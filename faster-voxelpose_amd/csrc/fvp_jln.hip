// JLN post-processing on device: soft-argmax of the
// per-plane joint maps, the offset shift and the three-plane fusion.
//
// Reference: SoftArgmaxLayer.forward (joint_localization_net.py:32-56),
// the offset additions of JointLocalizationNet.forward (:170-174) and
// fuse_pose_preds (:83-120).  The reference runs these per frame between the
// P2PNet / WeightNet CNNs with a host sync per frame (:148-151); here they are
// two launches for every proposal of a batch.
//
//   softargmax_kernel: one 256-thread block per (plane, proposal, joint):
//     y = beta * x; m = max y; e = exp(y - m); s = sum e
//     pose = sum(e * grid) / s + offset(plane);  maxprob = 1 / s  (= max softmax)
//   fuse_kernel: one block per proposal, thread per joint:
//     x = (w_xy, w_xz) / (w_xy + w_xz) . (xy.x, xz.x),  y, z likewise
//     conf = mean over planes and joints of maxprob
// Floating point: exp and the 4096-term sums differ from torch's CPU kernels
// in rounding only (parity is tolerance-based; see tests/test_jln_post.py).
#include "fvp_layout.h"

namespace fvp {

__device__ __forceinline__ float block_reduce_max(float v, float *red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) red[wave] = v;
    __syncthreads();
    v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    return v;
}

__device__ __forceinline__ float block_reduce_sum(float v, float *red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) red[wave] = v;
    __syncthreads();
    v = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return v;
}

// feat [3][P][J][S2], grids [3][S2][2], offset [P][3] (may be NULL)
// pose [3][P][J][2], maxprob [3][P][J]
// The row is read once: S2 <= 256*4*RV values stay in registers (float4 loads).
template <int RV>
__global__ __launch_bounds__(256) void softargmax_kernel(const float *__restrict__ feat,
                                                         const float *__restrict__ grids,
                                                         const float *__restrict__ offset, int P, int J, int S2,
                                                         float beta, float *__restrict__ pose,
                                                         float *__restrict__ maxprob) {
    __shared__ float red[4];
    const int row = blockIdx.x;  // (plane, p, j)
    const int plane = row / (P * J);
    const int p = (row / J) % P;
    const float *__restrict__ x = feat + (size_t)row * S2;
    const float *__restrict__ g = grids + (size_t)plane * S2 * 2;
    const bool vec = (S2 & 3) == 0;
    float y[RV][4];
    float m = -INFINITY;
#pragma unroll
    for (int r = 0; r < RV; ++r) {
        const int i = (r * 256 + threadIdx.x) * 4;
        if (vec && i < S2) {
            const float4 v = *reinterpret_cast<const float4 *>(x + i);
            y[r][0] = beta * v.x; y[r][1] = beta * v.y; y[r][2] = beta * v.z; y[r][3] = beta * v.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) y[r][k] = (i + k < S2) ? beta * x[i + k] : -INFINITY;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) m = fmaxf(m, y[r][k]);
    }
    m = block_reduce_max(m, red);
    float s = 0.f, sx = 0.f, sy = 0.f;
#pragma unroll
    for (int r = 0; r < RV; ++r) {
        const int i = (r * 256 + threadIdx.x) * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (i + k < S2) {
                const float e = expf(y[r][k] - m);
                const float2 c = reinterpret_cast<const float2 *>(g)[i + k];
                s += e;
                sx = __builtin_fmaf(e, c.x, sx);
                sy = __builtin_fmaf(e, c.y, sy);
            }
        }
    }
    s = block_reduce_sum(s, red);
    sx = block_reduce_sum(sx, red);
    sy = block_reduce_sum(sy, red);
    if (threadIdx.x == 0) {
        float ox = 0.f, oy = 0.f;
        if (offset) {  // xy: (x, y), xz: (x, z), yz: (y, z)   (:170-174)
            const float *o = offset + (size_t)p * 3;
            ox = plane == 2 ? o[1] : o[0];
            oy = plane == 0 ? o[1] : o[2];
        }
        pose[(size_t)row * 2 + 0] = sx / s + ox;
        pose[(size_t)row * 2 + 1] = sy / s + oy;
        maxprob[row] = 1.0f / s;
    }
}

// pose [3][P][J][2], weights [3P][J] (WeightNet output, plane-major), maxprob [3][P][J]
// fused [P][J][3], confs [P]
__global__ __launch_bounds__(64) void fuse_kernel(const float *__restrict__ pose, const float *__restrict__ weights,
                                                  const float *__restrict__ maxprob, int P, int J,
                                                  float *__restrict__ fused, float *__restrict__ confs) {
    const int p = blockIdx.x;
    const size_t PJ = (size_t)P * J;
    for (int j = threadIdx.x; j < J && fused; j += 64) {
        const size_t r = (size_t)p * J + j;
        const float wxy = weights[r], wxz = weights[PJ + r], wyz = weights[2 * PJ + r];
        const float *xy = pose + r * 2, *xz = pose + (PJ + r) * 2, *yz = pose + (2 * PJ + r) * 2;
        const float sx = wxy + wxz, sy = wxy + wyz, sz = wxz + wyz;
        float *o = fused + r * 3;
        o[0] = (wxy / sx) * xy[0] + (wxz / sx) * xz[0];
        o[1] = (wxy / sy) * xy[1] + (wyz / sy) * yz[0];
        o[2] = (wxz / sz) * xz[1] + (wyz / sz) * yz[1];
    }
    if (confs && threadIdx.x == 0) {
        float s = 0.f;
        for (int plane = 0; plane < 3; ++plane)
            for (int j = 0; j < J; ++j) s += maxprob[(size_t)plane * PJ + (size_t)p * J + j];
        confs[p] = s / (float)(3 * J);
    }
}

}  // namespace fvp

extern "C" int fvp_soft_argmax(const float *features, int P, int J, int S2, const float *center_grid,
                               const float *offset, float beta, float *pose, float *maxprob, void *stream) {
    if (P == 0) return FVP_OK;
    if (!features || !center_grid || !pose || !maxprob) return FVP_ERR_NULL;
    if (P < 0 || J <= 0 || S2 <= 0) return FVP_ERR_SHAPE;
    if ((long long)3 * P * J > 0x7fffffffLL) return FVP_ERR_SHAPE;
    if (S2 > 256 * 4 * 8) return FVP_ERR_SHAPE;  // up to 8192 cells per plane (64x64 = 4096)
    const dim3 grid((unsigned)(3 * P * J));
    if (S2 <= 256 * 4 * 4)
        hipLaunchKernelGGL(fvp::softargmax_kernel<4>, grid, dim3(256), 0, (hipStream_t)stream, features, center_grid,
                           offset, P, J, S2, beta, pose, maxprob);
    else
        hipLaunchKernelGGL(fvp::softargmax_kernel<8>, grid, dim3(256), 0, (hipStream_t)stream, features, center_grid,
                           offset, P, J, S2, beta, pose, maxprob);
    return (int)hipGetLastError();
}

extern "C" int fvp_fuse_poses(const float *pose, const float *weights, const float *maxprob, int P, int J,
                              float *fused, float *confs, void *stream) {
    if (P == 0) return FVP_OK;
    if (!pose || (fused && !weights) || (confs && !maxprob)) return FVP_ERR_NULL;
    if (P < 0 || J <= 0) return FVP_ERR_SHAPE;
    hipLaunchKernelGGL(fvp::fuse_kernel, dim3((unsigned)P), dim3(64), 0, (hipStream_t)stream, pose, weights, maxprob,
                       P, J, fused, confs);
    return (int)hipGetLastError();
}
