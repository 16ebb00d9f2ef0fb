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

// Rows longer than the register-resident kernel holds (person cubes beyond
// 90^3): the same arithmetic in two passes over the row (max, then exp sums).
__global__ __launch_bounds__(256) void softargmax_stream_kernel(const float *__restrict__ feat,
                                                                const float *__restrict__ grids,
                                                                const float *__restrict__ offset, int P, int J,
                                                                int S2, float beta, float *__restrict__ pose,
                                                                float *__restrict__ maxprob) {
    __shared__ float red[4];
    const int row = blockIdx.x;  // (plane, p, j)
    const int plane = row / (P * J);
    const int p = (row / J) % P;
    const float *__restrict__ x = feat + (size_t)row * S2;
    const float2 *__restrict__ g = reinterpret_cast<const float2 *>(grids + (size_t)plane * S2 * 2);
    float m = -INFINITY;
    for (int i = threadIdx.x; i < S2; i += 256) m = fmaxf(m, beta * x[i]);
    m = block_reduce_max(m, red);
    float s = 0.f, sx = 0.f, sy = 0.f;
    for (int i = threadIdx.x; i < S2; i += 256) {
        const float e = expf(beta * x[i] - m);
        const float2 c = g[i];
        s += e;
        sx = __builtin_fmaf(e, c.x, sx);
        sy = __builtin_fmaf(e, c.y, sy);
    }
    s = block_reduce_sum(s, red);
    sx = block_reduce_sum(sx, red);
    sy = block_reduce_sum(sy, red);
    if (threadIdx.x == 0) {
        float ox = 0.f, oy = 0.f;
        if (offset) {
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


// ---- WeightNet (weight_net.py:48-80): one block per joint map ---------------
// x [Nimg][H][W] (the [3P][J] joint maps, flattened as at weight_net.py:65-68)
//   -> conv3x3(1 -> C, pad 1) * scale + shift (conv bias and BatchNorm folded)
//   -> max_pool 2x2 (floor) -> ReLU -> mean over the pooled map
//   -> Linear(C -> Hd) -> ReLU -> Linear(Hd -> 1) -> sigmoid      -> out [Nimg]
// The [C][H][W] conv map the reference materialises (23.6 MB per proposal at
// 64x64, C = 32) never leaves registers: each thread owns pooled cells, reads
// their 4x4 input patch from the LDS copy of the map and keeps C running sums.
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int CMAX>
__global__ __launch_bounds__(256) void weight_net_kernel(const float *__restrict__ x, int H, int W,
                                                         const float *__restrict__ cw, const float *__restrict__ scale,
                                                         const float *__restrict__ shift, int C,
                                                         const float *__restrict__ w1, const float *__restrict__ b1,
                                                         int Hd, const float *__restrict__ w2,
                                                         const float *__restrict__ b2, float *__restrict__ out) {
    extern __shared__ float smem[];  // [(H+2)*(W+2)] zero-padded map | [4][CMAX] wave sums | [CMAX] means | [4]
    const int Wp = W + 2;
    const float *__restrict__ img = x + (size_t)blockIdx.x * H * W;
    for (int i = threadIdx.x; i < (H + 2) * Wp; i += 256) {
        const int yy = i / Wp - 1, xx = i - (yy + 1) * Wp - 1;
        smem[i] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? img[yy * W + xx] : 0.0f;
    }
    __syncthreads();
    float acc[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) acc[c] = 0.0f;
    const int Ho = H / 2, Wo = W / 2;
    for (int p = threadIdx.x; p < Ho * Wo; p += 256) {
        const int py = p / Wo, px = p - py * Wo;
        float t[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) t[r][q] = smem[(2 * py + r) * Wp + 2 * px + q];
#pragma unroll
        for (int c = 0; c < CMAX; ++c) {
            if (c < C) {  // uniform: the weights come in through scalar loads
                float k[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) k[i] = cw[c * 9 + i];
                const float sc = scale[c], sh = shift[c];
                // the two outputs of a pooled row as one packed pair (v_pk_fma_f32)
                f32x2 v[2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};
#pragma unroll
                for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                    for (int i = 0; i < 9; ++i) {
                        const f32x2 tap = {t[dy + i / 3][i % 3], t[dy + i / 3][1 + i % 3]};
                        v[dy] = __builtin_elementwise_fma((f32x2){k[i], k[i]}, tap, v[dy]);
                    }
                const f32x2 scv = {sc, sc}, shv = {sh, sh};
                v[0] = v[0] * scv + shv;
                v[1] = v[1] * scv + shv;
                // the 2x2 pool as two v_maximum3_f32 (IEEE maximum: NaN propagates as
                // in max_pool2d; +0 / -0 may differ from torch's pick, which the ReLU
                // and the +0-started sum below make invisible)
                const float m = __builtin_elementwise_maximum(
                    __builtin_elementwise_maximum(v[0][0], v[0][1]),
                    __builtin_elementwise_maximum(v[1][0], v[1][1]));
                acc[c] += m < 0.0f ? 0.0f : m;  // ReLU after the pool; NaN passes through as in torch
            }
        }
    }
    float *wsum = smem + (H + 2) * Wp, *mean = wsum + 4 * CMAX, *red = mean + CMAX;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
        if (c < C) {
            float v = acc[c];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) wsum[wave * CMAX + c] = v;
        }
    }
    __syncthreads();
    if (threadIdx.x < C) {
        const int c = threadIdx.x;
        mean[c] = ((wsum[c] + wsum[CMAX + c]) + (wsum[2 * CMAX + c] + wsum[3 * CMAX + c])) / (float)(Ho * Wo);
    }
    __syncthreads();
    float part = 0.0f;
    for (int h = threadIdx.x; h < Hd; h += 256) {
        float z = 0.0f;
        for (int c = 0; c < C; ++c) z = fmaf(w1[(size_t)h * C + c], mean[c], z);
        z += b1[h];
        part = fmaf(w2[h], z < 0.0f ? 0.0f : z, part);
    }
    part = block_reduce_sum(part, red);
    if (threadIdx.x == 0) out[blockIdx.x] = 1.0f / (1.0f + expf(-(part + b2[0])));
}

// torch.nonzero of a [rows][cols] bool mask in one launch (the JLN's one host sync reads `count`):
// idx[i] = (row, col) of the i-th true entry in row-major order, as nonzero returns them.  One
// 1,024-thread block: per 1,024-entry tile a wave-ballot prefix, the waves' totals in LDS, and a
// running base (rocprim's nonzero took 6 launches and a fill for the same, ~30 us at C3 B = 8).
// Optionally (the JLN's selection, so that nothing but views remains after the sync): frame_of[i] =
// row (int32) and rowdst[i][0..width) = rowsrc[row * rs0 + col * rs1 + 0..width).
__global__ __launch_bounds__(1024) void mask_nonzero_kernel(const unsigned char *__restrict__ mask, int n, int cols,
                                                            long long *__restrict__ idx, int *__restrict__ count,
                                                            int *__restrict__ frame_of,
                                                            const float *__restrict__ rowsrc, long long rs0,
                                                            long long rs1, int width, float *__restrict__ rowdst) {
    __shared__ int wtot[16];
    __shared__ int base_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) base_s = 0;
    __syncthreads();
    for (int t0 = 0; t0 < n; t0 += 1024) {
        const int e = t0 + tid;
        const bool on = e < n && mask[e] != 0;
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(on);
        const int before = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
        if (lane == 0) wtot[wave] = (int)__builtin_popcountll(bal);
        __syncthreads();
        int off = base_s;
        for (int w = 0; w < wave; ++w) off += wtot[w];
        if (on) {
            const int i = off + before, r = e / cols, c = e - r * cols;
            idx[2 * (size_t)i] = r;
            idx[2 * (size_t)i + 1] = c;
            if (frame_of) frame_of[i] = r;
            if (rowdst)
                for (int q = 0; q < width; ++q) rowdst[(size_t)i * width + q] = rowsrc[r * rs0 + c * rs1 + q];
        }
        __syncthreads();  // every wave has read base_s and wtot
        if (tid == 0) {
            int tot = 0;
            for (int w = 0; w < 16; ++w) tot += wtot[w];
            base_s += tot;
        }
        __syncthreads();
    }
    if (tid == 0) *count = base_s;
}

// The JLN's three boolean scatters (joint_localization_net.py:176-180) in one launch:
// all_fused[b,k] = fused[p], all_pose[:, b, k] = pose[:, p], centers[b, k, conf_col] = confs[p]
// for the P (b, k) pairs of idx; thread = (p, joint).
__global__ __launch_bounds__(256) void scatter_poses_kernel(const long long *__restrict__ idx, int P, int B, int K,
                                                            int J, const float *__restrict__ fused,
                                                            const float *__restrict__ pose,
                                                            const float *__restrict__ confs,
                                                            float *__restrict__ all_fused, float *__restrict__ all_pose,
                                                            float *__restrict__ centers, long long cs0, long long cs1,
                                                            int conf_col) {
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= (long long)P * J) return;
    const int p = (int)(gid / J), j = (int)(gid - (long long)p * J);
    const long long b = idx[2 * p], k = idx[2 * p + 1];
    const size_t bkj = ((size_t)b * K + k) * J + j;
#pragma unroll
    for (int c = 0; c < 3; ++c) all_fused[bkj * 3 + c] = fused[((size_t)p * J + j) * 3 + c];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int c = 0; c < 2; ++c)
            all_pose[(((size_t)pl * B * K) * J + bkj) * 2 + c] = pose[((((size_t)pl * P) + p) * J + j) * 2 + c];
    if (j == 0 && centers) centers[b * cs0 + k * cs1 + conf_col] = confs[p];
}

}  // namespace fvp

extern "C" int fvp_soft_argmax(const float *features, int P, int J, int S2, const float *center_grid,
                               const float *offset, float beta, float *pose, float *maxprob, void *stream) {
    if (P == 0) return FVP_OK;
    if (!features || !center_grid || !pose || !maxprob) return FVP_ERR_NULL;
    if (P < 0 || J <= 0 || S2 <= 0) return FVP_ERR_SHAPE;
    if ((long long)3 * P * J > 0x7fffffffLL) return FVP_ERR_SHAPE;
    const dim3 grid((unsigned)(3 * P * J));
    if (S2 > 256 * 4 * 8)  // beyond 8192 cells per plane (64x64 = 4096): two passes over the row
        hipLaunchKernelGGL(fvp::softargmax_stream_kernel, grid, dim3(256), 0, (hipStream_t)stream, features,
                           center_grid, offset, P, J, S2, beta, pose, maxprob);
    else if (S2 <= 256 * 4 * 4)
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

extern "C" int fvp_weight_net(const float *features, int Nimg, int H, int W, const float *conv_w,
                              const float *scale, const float *shift, int C, const float *fc1_w, const float *fc1_b,
                              int Hd, const float *fc2_w, const float *fc2_b, float *out, void *stream) {
    if (Nimg == 0) return FVP_OK;
    if (!features || !conv_w || !scale || !shift || !fc1_w || !fc1_b || !fc2_w || !fc2_b || !out)
        return FVP_ERR_NULL;
    if (Nimg < 0 || H < 2 || W < 2 || C <= 0 || C > 64 || Hd <= 0) return FVP_ERR_SHAPE;
    const int cmax = C <= 32 ? 32 : 64;
    const size_t lds = ((size_t)(H + 2) * (W + 2) + 5 * cmax + 4) * sizeof(float);
    if (lds > 64 * 1024) return FVP_ERR_SHAPE;  // maps up to ~124x124
    hipStream_t st = (hipStream_t)stream;
    if (cmax == 32)
        hipLaunchKernelGGL(fvp::weight_net_kernel<32>, dim3((unsigned)Nimg), dim3(256), lds, st, features, H, W,
                           conv_w, scale, shift, C, fc1_w, fc1_b, Hd, fc2_w, fc2_b, out);
    else
        hipLaunchKernelGGL(fvp::weight_net_kernel<64>, dim3((unsigned)Nimg), dim3(256), lds, st, features, H, W,
                           conv_w, scale, shift, C, fc1_w, fc1_b, Hd, fc2_w, fc2_b, out);
    return (int)hipGetLastError();
}

extern "C" int fvp_mask_select(const unsigned char *mask, int rows, int cols, long long *idx, int *count,
                               int *frame_of, const float *rowsrc, long long rs0, long long rs1, int width,
                               float *rowdst, void *stream);

extern "C" int fvp_mask_nonzero(const unsigned char *mask, int rows, int cols, long long *idx, int *count,
                                void *stream) {
    return fvp_mask_select(mask, rows, cols, idx, count, nullptr, nullptr, 0, 0, 0, nullptr, stream);
}

extern "C" int fvp_mask_select(const unsigned char *mask, int rows, int cols, long long *idx, int *count,
                               int *frame_of, const float *rowsrc, long long rs0, long long rs1, int width,
                               float *rowdst, void *stream) {
    if (!mask || !idx || !count || (rowdst && !rowsrc)) return FVP_ERR_NULL;
    if (rows < 0 || cols <= 0 || (long long)rows * cols > (1LL << 24) || (rowdst && width <= 0)) return FVP_ERR_SHAPE;
    hipLaunchKernelGGL(fvp::mask_nonzero_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, mask, rows * cols, cols,
                       idx, count, frame_of, rowsrc, rs0, rs1, width, rowdst);
    return (int)hipGetLastError();
}

extern "C" int fvp_scatter_poses(const long long *idx, int P, int B, int K, int J, const float *fused,
                                 const float *pose, const float *confs, float *all_fused, float *all_pose,
                                 float *centers, long long cs0, long long cs1, int conf_col, void *stream) {
    if (P == 0) return FVP_OK;
    if (!idx || !fused || !pose || !all_fused || !all_pose || (centers && !confs)) return FVP_ERR_NULL;
    if (P < 0 || B <= 0 || K <= 0 || J <= 0 || P > B * K) return FVP_ERR_SHAPE;
    const long long n = (long long)P * J;
    hipLaunchKernelGGL(fvp::scatter_poses_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       idx, P, B, K, J, fused, pose, confs, all_fused, all_pose, centers, cs0, cs1, conf_col);
    return (int)hipGetLastError();
}
