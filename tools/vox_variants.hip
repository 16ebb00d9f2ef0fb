// Experimental voxelize variants for A/B timing on the GPU (tools/microbench.py).
// Not part of the product library.  Each variant must produce the same cube /
// xy as the product kernel (bit-exact up to the sign of zero); microbench.py
// checks that before timing.
//
//   MAP  lane -> voxel mapping of a wave: (CX, CY, ZL) with CX*CY*ZL = 64
//   TAP  0: four buffer_load_dword per joint, out-of-image taps read as 0 via
//           the descriptor's range check (offset 0x80000000)
//        1: two buffer_load_dwordx2 per joint (horizontal tap pairs), rows
//           clamped, out-of-image taps get weight 0 (order of the non-zero
//           fma terms preserved -> same rounding as the reference)
#include "../faster-voxelpose_amd/csrc/fvp_device.h"

namespace fvpx {
using namespace fvp;

constexpr unsigned kOOB = 0x80000000u;

template <int MAP> struct Map;
template <> struct Map<0> { static constexpr int CX = 4, CY = 4, ZL = 4; };
template <> struct Map<1> { static constexpr int CX = 8, CY = 8, ZL = 1; };
template <> struct Map<2> { static constexpr int CX = 2, CY = 4, ZL = 8; };
template <> struct Map<3> { static constexpr int CX = 1, CY = 16, ZL = 4; };
template <> struct Map<4> { static constexpr int CX = 2, CY = 2, ZL = 16; };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_for(const float *base, unsigned bytes) {
    const unsigned long long p = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
    const float *b = (const float *)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc((void *)b, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                             0x00020000);
}

template <int MAP, int TAP, bool CUBE, int JT>
__global__ __launch_bounds__(256) void vox_var(const float *__restrict__ hm, const float2 *__restrict__ grids,
                                               float *__restrict__ cube, float *__restrict__ xy, int V, int J, int H,
                                               int W, int X, int Y, int Z, int tiles_y, int tiles_per_frame,
                                               int total_waves) {
    constexpr int CX = Map<MAP>::CX, CY = Map<MAP>::CY, ZL = Map<MAP>::ZL;
    const int lane = threadIdx.x & 63;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int wid = __builtin_amdgcn_readfirstlane(L * 4 + (threadIdx.x >> 6));
    if (wid >= total_waves) return;
    const int b = wid / tiles_per_frame;
    const int t = wid - b * tiles_per_frame;
    const int tx = t / tiles_y, ty = t - (t / tiles_y) * tiles_y;
    const int x = tx * CX + lane / (CY * ZL);
    const int y = ty * CY + (lane / ZL) % CY;
    const int zl = lane % ZL;
    const bool col_ok = (x < X) && (y < Y);
    const long long N = (long long)X * Y * Z;
    const unsigned HW = (unsigned)(H * W);
    const float fV = (float)V;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;

    for (int j0 = 0; j0 < J; j0 += JT) {
        const int jlast = min(JT, J - j0) - 1;
        float xymax[JT];
#pragma unroll
        for (int jj = 0; jj < JT; ++jj) xymax[jj] = -INFINITY;
        for (int z0 = 0; z0 < Z; z0 += ZL) {
            const int z = z0 + zl;
            const bool valid = col_ok && (z < Z);
            const long long n = ((long long)x * Y + y) * Z + z;
            float acc[JT];
#pragma unroll
            for (int jj = 0; jj < JT; ++jj) acc[jj] = 0.0f;
            for (int v = 0; v < V; ++v) {
                const float2 gg = valid ? grids[(size_t)v * N + n] : make_float2(-2.f, -2.f);
                const float ix = (gg.x + 1.0f) * sxs;
                const float iy = (gg.y + 1.0f) * sys;
                const float x0f = floorf(ix), y0f = floorf(iy);
                const float wx = ix - x0f, ex = 1.0f - wx;
                const float ny = iy - y0f, syw = 1.0f - ny;
                const float nw = syw * ex, ne = syw * wx, sw = ny * ex, se = ny * wx;
                const bool isnan_ = (ix != ix) || (iy != iy);
                const int x0 = isnan_ ? -4 : (int)x0f, y0 = isnan_ ? -4 : (int)y0f;
                const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
                const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
                const bool any = (vx0 | vx1) & (vy0 | vy1);
                if (isnan_) {
#pragma unroll
                    for (int jj = 0; jj < JT; ++jj) acc[jj] = acc[jj] + NAN;
                    continue;
                }
                if (!__builtin_amdgcn_ballot_w64(any)) continue;  // whole wave off-image for this camera
                const __amdgpu_buffer_rsrc_t rs =
                    rsrc_for(hm + ((size_t)b * V + v) * J * HW + (size_t)j0 * HW, (unsigned)((J - j0) * HW * 4));
                if (TAP == 0) {
                    const unsigned o00 = (vy0 & vx0) ? (unsigned)(y0 * W + x0) * 4u : kOOB;
                    const unsigned o01 = (vy0 & vx1) ? (unsigned)(y0 * W + x0 + 1) * 4u : kOOB;
                    const unsigned o10 = (vy1 & vx0) ? (unsigned)((y0 + 1) * W + x0) * 4u : kOOB;
                    const unsigned o11 = (vy1 & vx1) ? (unsigned)((y0 + 1) * W + x0 + 1) * 4u : kOOB;
                    float tv[JT][4];
#pragma unroll
                    for (int jj = 0; jj < JT; ++jj) {  // issue every tap load of the voxel-camera first
                        const int so = min(jj, jlast) * (int)HW * 4;  // padded joints re-read a valid plane
                        tv[jj][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o00, so, 0));
                        tv[jj][1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o01, so, 0));
                        tv[jj][2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o10, so, 0));
                        tv[jj][3] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o11, so, 0));
                    }
#pragma unroll
                    for (int jj = 0; jj < JT; ++jj)
                        acc[jj] = acc[jj] + __builtin_fmaf(tv[jj][3], se, __builtin_fmaf(tv[jj][2], sw,
                                                           __builtin_fmaf(tv[jj][1], ne, tv[jj][0] * nw)));
                } else {
                    const int xs = min(max(x0, 0), W - 2);
                    float w0, w1, u0, u1;  // top-row slot weights, bottom-row slot weights
                    if (x0 == xs) { w0 = nw; w1 = ne; u0 = sw; u1 = se; }
                    else if (x0 == -1) { w0 = ne; w1 = 0.f; u0 = se; u1 = 0.f; }
                    else if (x0 == W - 1) { w0 = 0.f; w1 = nw; u0 = 0.f; u1 = sw; }
                    else { w0 = w1 = u0 = u1 = 0.f; }
                    const unsigned ot = vy0 ? (unsigned)(y0 * W + xs) * 4u : kOOB;
                    const unsigned ob = vy1 ? (unsigned)((y0 + 1) * W + xs) * 4u : kOOB;
                    decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, ot, 0, 0)) tp[JT], bt[JT];
#pragma unroll
                    for (int jj = 0; jj < JT; ++jj) {
                        const int so = min(jj, jlast) * (int)HW * 4;
                        tp[jj] = __builtin_amdgcn_raw_buffer_load_b64(rs, ot, so, 0);
                        bt[jj] = __builtin_amdgcn_raw_buffer_load_b64(rs, ob, so, 0);
                    }
#pragma unroll
                    for (int jj = 0; jj < JT; ++jj) {
                        const float p0 = __builtin_bit_cast(float, (unsigned)tp[jj][0]);
                        const float p1 = __builtin_bit_cast(float, (unsigned)tp[jj][1]);
                        const float q0 = __builtin_bit_cast(float, (unsigned)bt[jj][0]);
                        const float q1 = __builtin_bit_cast(float, (unsigned)bt[jj][1]);
                        acc[jj] = acc[jj] + __builtin_fmaf(q1, u1, __builtin_fmaf(q0, u0, __builtin_fmaf(p1, w1, p0 * w0)));
                    }
                }
            }
#pragma unroll
            for (int jj = 0; jj < JT; ++jj) {
                if (j0 + jj < J) {
                    const float o = clampf(acc[jj] / fV, 0.0f, 1.0f);
                    if (valid) {
                        if (CUBE) cube[((size_t)b * J + j0 + jj) * N + n] = o;
                        xymax[jj] = nanmax(xymax[jj], o);
                    }
                }
            }
        }
#pragma unroll
        for (int jj = 0; jj < JT; ++jj) {
            float m = xymax[jj];
#pragma unroll
            for (int s = 1; s < ZL; s <<= 1) m = nanmax(m, __shfl_xor(m, s));
            if (j0 + jj < J && zl == 0 && col_ok) xy[(((size_t)b * J + j0 + jj) * X + x) * Y + y] = m;
        }
    }
}

template <int MAP, int TAP, bool CUBE>
int launch(const float *hm, int B, int V, int J, int H, int W, const float *grids, int X, int Y, int Z, float *cube,
           float *xy, hipStream_t s) {
    constexpr int CX = Map<MAP>::CX, CY = Map<MAP>::CY;
    const int tiles_y = (Y + CY - 1) / CY, tiles_x = (X + CX - 1) / CX;
    const int tpf = tiles_x * tiles_y;
    const int total = tpf * B;
    const int blocks = (total + 3) / 4;
#define VV_LAUNCH(JT_)                                                                                           \
    hipLaunchKernelGGL((vox_var<MAP, TAP, CUBE, JT_>), dim3(blocks), dim3(256), 0, s, hm,                          \
                       reinterpret_cast<const float2 *>(grids), cube, xy, V, J, H, W, X, Y, Z, tiles_y, tpf, total)
    if (J == 15) VV_LAUNCH(15);
    else if (J <= 8) VV_LAUNCH(8);
    else VV_LAUNCH(16);
#undef VV_LAUNCH
    return (int)hipGetLastError();
}

}  // namespace fvpx

#define VARIANT(M, T, C)                                                                                           \
    if (variant == (M) * 100 + (T) * 10 + (C))                                                                     \
        return fvpx::launch<M, T, (C) != 0>(hm, B, V, J, H, W, grids, X, Y, Z, cube, xy, (hipStream_t)stream);

extern "C" int voxvar_launch(int variant, const float *hm, int B, int V, int J, int H, int W, const float *grids,
                             int X, int Y, int Z, float *cube, float *xy, void *stream) {
    VARIANT(0, 0, 1) VARIANT(0, 1, 1) VARIANT(0, 1, 0) VARIANT(2, 1, 0) VARIANT(4, 1, 0)
    VARIANT(1, 0, 1) VARIANT(1, 1, 1)
    VARIANT(2, 0, 1) VARIANT(2, 1, 1)
    VARIANT(3, 0, 1) VARIANT(3, 1, 1)
    VARIANT(4, 1, 1)
    return -1;
}

// ---------------------------------------------------------------------------
// Channels-last experiment: heatmaps transposed to [B][V][H][W][JP] (JP = 4*LPV,
// zero padded), so the 4*LPV joints of one pixel are contiguous; LPV lanes
// (a quad for LPV = 4) share one voxel and each loads 16 B = 4 joints of a tap.
namespace fvpx {

template <int LPV>
__global__ __launch_bounds__(256) void to_cl(const float *__restrict__ hm, float *__restrict__ cl, int J, int HW,
                                             long long total_px) {
    constexpr int JP = 4 * LPV;
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long pxg = gid / LPV;  // global pixel over (bv, pix)
    const int q = (int)(gid % LPV);
    if (pxg >= total_px) return;
    const long long bv = pxg / HW;
    const int pix = (int)(pxg - bv * HW);
    const float *src = hm + (size_t)bv * J * HW + pix;
    float4 o;
    const int j = 4 * q;
    o.x = (j + 0 < J) ? src[(size_t)(j + 0) * HW] : 0.f;
    o.y = (j + 1 < J) ? src[(size_t)(j + 1) * HW] : 0.f;
    o.z = (j + 2 < J) ? src[(size_t)(j + 2) * HW] : 0.f;
    o.w = (j + 3 < J) ? src[(size_t)(j + 3) * HW] : 0.f;
    reinterpret_cast<float4 *>(cl)[pxg * LPV + q] = o;
}

template <int LPV, int COLS, bool CUBE>
__global__ __launch_bounds__(256) void vox_cl(const float *__restrict__ cl, const float2 *__restrict__ grids,
                                              float *__restrict__ cube, float *__restrict__ xy, int V, int J, int H,
                                              int W, int X, int Y, int Z, int col_blocks) {
    constexpr int JP = 4 * LPV;
    constexpr int VPP = 256 / LPV;  // voxels per pass
    extern __shared__ __attribute__((aligned(16))) float stage[];  // [JP][COLS*Z]
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int b = L / col_blocks;
    const int c0 = (L - b * col_blocks) * COLS;
    const int XY = X * Y;
    const int ncols = min(COLS, XY - c0);
    const int T = ncols * Z;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const unsigned HW = (unsigned)(H * W);
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int v = 0; v < V; ++v) {
            const float2 gg = valid ? grids[(size_t)v * N + n0 + i] : make_float2(-2.f, -2.f);
            const float ix = (gg.x + 1.0f) * sxs;
            const float iy = (gg.y + 1.0f) * sys;
            const float x0f = floorf(ix), y0f = floorf(iy);
            const float wx = ix - x0f, ex = 1.0f - wx;
            const float ny = iy - y0f, syw = 1.0f - ny;
            const float nw = syw * ex, ne = syw * wx, sw = ny * ex, se = ny * wx;
            const bool isnan_ = (ix != ix) || (iy != iy);
            const int x0 = isnan_ ? -4 : (int)x0f, y0 = isnan_ ? -4 : (int)y0f;
            const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
            const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
            const bool any = (vx0 | vx1) & (vy0 | vy1);
            if (isnan_) {
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] = acc[k] + NAN;
            }
            if (!__builtin_amdgcn_ballot_w64(any)) continue;
            const __amdgpu_buffer_rsrc_t rs = rsrc_for(cl + ((size_t)b * V + v) * HW * JP, HW * JP * 4u);
            const unsigned pix = (unsigned)(y0 * W + x0);
            const unsigned qo = (unsigned)q * 16u;
            const unsigned o00 = (vy0 & vx0) ? pix * (JP * 4u) + qo : kOOB;
            const unsigned o01 = (vy0 & vx1) ? (pix + 1u) * (JP * 4u) + qo : kOOB;
            const unsigned o10 = (vy1 & vx0) ? (pix + (unsigned)W) * (JP * 4u) + qo : kOOB;
            const unsigned o11 = (vy1 & vx1) ? (pix + (unsigned)W + 1u) * (JP * 4u) + qo : kOOB;
            const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, o00, 0, 0);
            const auto bq = __builtin_amdgcn_raw_buffer_load_b128(rs, o01, 0, 0);
            const auto c = __builtin_amdgcn_raw_buffer_load_b128(rs, o10, 0, 0);
            const auto d = __builtin_amdgcn_raw_buffer_load_b128(rs, o11, 0, 0);
            if (!isnan_) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float fa = __builtin_bit_cast(float, (unsigned)a[k]);
                    const float fb = __builtin_bit_cast(float, (unsigned)bq[k]);
                    const float fc = __builtin_bit_cast(float, (unsigned)c[k]);
                    const float fd = __builtin_bit_cast(float, (unsigned)d[k]);
                    acc[k] = acc[k] + __builtin_fmaf(fd, se, __builtin_fmaf(fc, sw, __builtin_fmaf(fb, ne, fa * nw)));
                }
            }
        }
        if (valid) {
#pragma unroll
            for (int k = 0; k < 4; ++k) stage[(4 * q + k) * (COLS * Z) + i] = clampf(acc[k] / fV, 0.f, 1.f);
        }
    }
    __syncthreads();
    // coalesced cube write: joint-major runs of T floats
    if (CUBE) {
        for (int j = 0; j < J; ++j)
            for (int e = threadIdx.x; e < T; e += 256) cube[((size_t)b * J + j) * N + n0 + e] = stage[j * (COLS * Z) + e];
    }
    // xy: max over z of each column
    for (int e = threadIdx.x; e < J * ncols; e += 256) {
        const int j = e / ncols, cc = e - (e / ncols) * ncols;
        float m = -INFINITY;
        const float *s = stage + j * (COLS * Z) + cc * Z;
        for (int z = 0; z < Z; ++z) m = nanmax(m, s[z]);
        xy[((size_t)b * J + j) * XY + c0 + cc] = m;
    }
}

}  // namespace fvpx

extern "C" int voxvar_to_cl(const float *hm, int B, int V, int J, int H, int W, float *cl, int lpv, void *stream) {
    const long long px = (long long)B * V * H * W;
    const long long threads = px * lpv;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    hipStream_t s = (hipStream_t)stream;
    if (lpv == 4) hipLaunchKernelGGL((fvpx::to_cl<4>), dim3(blocks), dim3(256), 0, s, hm, cl, J, H * W, px);
    else if (lpv == 8) hipLaunchKernelGGL((fvpx::to_cl<8>), dim3(blocks), dim3(256), 0, s, hm, cl, J, H * W, px);
    else return -1;
    return (int)hipGetLastError();
}

extern "C" int voxvar_cl(int cols, int cube_on, const float *cl, int B, int V, int J, int H, int W, const float *grids,
                         int X, int Y, int Z, float *cube, float *xy, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int XY = X * Y;
#define CL_LAUNCH(COLS, CUBE)                                                                                        \
    {                                                                                                                \
        const int cb = (XY + COLS - 1) / COLS;                                                                      \
        const size_t lds = (size_t)16 * COLS * Z * 4;                                                               \
        hipLaunchKernelGGL((fvpx::vox_cl<4, COLS, CUBE>), dim3(cb * B), dim3(256), lds, s, cl,                     \
                           reinterpret_cast<const float2 *>(grids), cube, xy, V, J, H, W, X, Y, Z, cb);              \
        return (int)hipGetLastError();                                                                               \
    }
    if (J > 16) return -1;
    if (cols == 16 && cube_on) CL_LAUNCH(16, true)
    if (cols == 16 && !cube_on) CL_LAUNCH(16, false)
    if (cols == 32 && cube_on) CL_LAUNCH(32, true)
    if (cols == 8 && cube_on) CL_LAUNCH(8, true)
#undef CL_LAUNCH
    return -2;
}

// v2: all cameras' grid reads, then all tap loads in flight at once (ILP), LDS-staged output.
namespace fvpx {
template <int VC, int COLS, bool CUBE>
__global__ __launch_bounds__(256) void vox_cl2(const float *__restrict__ cl, const float2 *__restrict__ grids,
                                               float *__restrict__ cube, float *__restrict__ xy, int V, int J, int H,
                                               int W, int X, int Y, int Z, int col_blocks) {
    constexpr int LPV = 4, JP = 16, VPP = 64;
    extern __shared__ __attribute__((aligned(16))) float stage[];  // [JP][COLS*Z + pad]
    const int SP = COLS * Z + 1;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int b = L / col_blocks;
    const int c0 = (L - b * col_blocks) * COLS;
    const int XY = X * Y;
    const int ncols = min(COLS, XY - c0);
    const int T = ncols * Z;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const unsigned HW = (unsigned)(H * W);
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int vb = 0; vb < V; vb += VC) {
            float2 g[VC];
#pragma unroll
            for (int u = 0; u < VC; ++u) {
                const int v = min(vb + u, V - 1);
                g[u] = grids[(size_t)v * N + n0 + min(i, T - 1)];  // unconditional (no branch): clamp index
                if (!valid) g[u] = make_float2(-2.f, -2.f);
            }
            float wt[VC][4];
            bool nanv[VC];
            using u32x4 = __attribute__((ext_vector_type(4))) unsigned; u32x4 d[VC][4];
#pragma unroll
            for (int u = 0; u < VC; ++u) {
                const int v = min(vb + u, V - 1);
                const float ix = (g[u].x + 1.0f) * sxs;
                const float iy = (g[u].y + 1.0f) * sys;
                const float x0f = floorf(ix), y0f = floorf(iy);
                const float wx = ix - x0f, ex = 1.0f - wx;
                const float ny = iy - y0f, syw = 1.0f - ny;
                wt[u][0] = syw * ex; wt[u][1] = syw * wx; wt[u][2] = ny * ex; wt[u][3] = ny * wx;
                nanv[u] = (ix != ix) || (iy != iy);
                const int x0 = nanv[u] ? -4 : (int)x0f, y0 = nanv[u] ? -4 : (int)y0f;
                const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
                const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
                const bool live = vb + u < V;
                const __amdgpu_buffer_rsrc_t rs = rsrc_for(cl + ((size_t)b * V + v) * HW * JP, HW * JP * 4u);
                const unsigned pix = (unsigned)(y0 * W + x0);
                const unsigned qo = (unsigned)q * 16u;
                d[u][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, (live & vy0 & vx0) ? pix * (JP * 4u) + qo : kOOB, 0, 0);
                d[u][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, (live & vy0 & vx1) ? (pix + 1u) * (JP * 4u) + qo : kOOB, 0, 0);
                d[u][2] = __builtin_amdgcn_raw_buffer_load_b128(rs, (live & vy1 & vx0) ? (pix + (unsigned)W) * (JP * 4u) + qo : kOOB, 0, 0);
                d[u][3] = __builtin_amdgcn_raw_buffer_load_b128(rs, (live & vy1 & vx1) ? (pix + (unsigned)W + 1u) * (JP * 4u) + qo : kOOB, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < VC; ++u) {
                if (vb + u < V) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const float fa = __builtin_bit_cast(float, (unsigned)d[u][0][k]);
                        const float fb = __builtin_bit_cast(float, (unsigned)d[u][1][k]);
                        const float fc = __builtin_bit_cast(float, (unsigned)d[u][2][k]);
                        const float fd = __builtin_bit_cast(float, (unsigned)d[u][3][k]);
                        const float val = nanv[u] ? NAN
                            : __builtin_fmaf(fd, wt[u][3], __builtin_fmaf(fc, wt[u][2], __builtin_fmaf(fb, wt[u][1], fa * wt[u][0])));
                        acc[k] = acc[k] + val;
                    }
                }
            }
        }
        if (valid) {
#pragma unroll
            for (int k = 0; k < 4; ++k) stage[(4 * q + k) * SP + i] = clampf(acc[k] / fV, 0.f, 1.f);
        }
    }
    __syncthreads();
    if (CUBE) {
        for (int j = 0; j < J; ++j)
            for (int e = threadIdx.x; e < T; e += 256) cube[((size_t)b * J + j) * N + n0 + e] = stage[j * SP + e];
    }
    for (int e = threadIdx.x; e < J * ncols; e += 256) {
        const int j = e / ncols, cc = e - (e / ncols) * ncols;
        float m = -INFINITY;
        const float *s = stage + j * SP + cc * Z;
        for (int z = 0; z < Z; ++z) m = nanmax(m, s[z]);
        xy[((size_t)b * J + j) * XY + c0 + cc] = m;
    }
}
}  // namespace fvpx

extern "C" int voxvar_cl2(int vc, int cols, const float *cl, int B, int V, int J, int H, int W, const float *grids,
                          int X, int Y, int Z, float *cube, float *xy, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int XY = X * Y;
#define CL2_LAUNCH(VC, COLS)                                                                                         \
    {                                                                                                                \
        const int cb = (XY + COLS - 1) / COLS;                                                                      \
        const size_t lds = (size_t)16 * (COLS * Z + 1) * 4;                                                         \
        hipLaunchKernelGGL((fvpx::vox_cl2<VC, COLS, true>), dim3(cb * B), dim3(256), lds, s, cl,                   \
                           reinterpret_cast<const float2 *>(grids), cube, xy, V, J, H, W, X, Y, Z, cb);              \
        return (int)hipGetLastError();                                                                               \
    }
    if (J > 16) return -1;
    if (vc == 5 && cols == 16) CL2_LAUNCH(5, 16)
    if (vc == 3 && cols == 16) CL2_LAUNCH(3, 16)
    if (vc == 1 && cols == 16) CL2_LAUNCH(1, 16)
    if (vc == 5 && cols == 8) CL2_LAUNCH(5, 8)
    if (vc == 5 && cols == 4) CL2_LAUNCH(5, 4)
#undef CL2_LAUNCH
    return -2;
}

// v3: one pass per workgroup (CT whole columns x Z), and an XCD-region mapping:
// the hardware deals blocks round-robin over the 8 XCDs, so block b runs on
// XCD (b % 8); XCD r is given region r (of an RX x RY split of the column
// grid) of every frame in turn, keeping the region's camera footprints in
// that XCD's L2.  Placement only affects speed.
namespace fvpx {
template <bool REGION>
__global__ __launch_bounds__(512) void vox_cl3(const float *__restrict__ cl, const float2 *__restrict__ grids,
                                               float *__restrict__ cube, float *__restrict__ xy, int V, int J, int H,
                                               int W, int X, int Y, int Z, int CT, int ytiles, int RX, int RY) {
    constexpr int LPV = 4, JP = 16;
    extern __shared__ __attribute__((aligned(16))) float stage[];  // [JP][CT*Z + 1]
    const int T = CT * Z;
    const int SP = T + 1;
    int b, x, yt;
    if (REGION) {
        const int xr = X / RX, yr = ytiles / RY, TR = xr * yr;
        const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
        b = k / TR;
        const int t = k - b * TR;
        x = (xcd / RY) * xr + t / yr;
        yt = (xcd % RY) * yr + t % yr;
    } else {
        const int L = xcd_remap(blockIdx.x, gridDim.x);
        const int TPF = X * ytiles;
        b = L / TPF;
        const int t = L - b * TPF;
        x = t / ytiles;
        yt = t - x * ytiles;
    }
    const int yb = yt * CT;
    const int ncols = min(CT, Y - yb);
    const int Tn = ncols * Z;
    const long long N = (long long)X * Y * Z;
    const long long n0 = ((long long)x * Y + yb) * Z;  // columns (x, yb..yb+ncols) are contiguous
    const int q = threadIdx.x % LPV;
    const int i = threadIdx.x / LPV;
    const bool valid = i < Tn;
    const unsigned HW = (unsigned)(H * W);
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int v = 0; v < V; ++v) {
        float2 gg = grids[(size_t)v * N + n0 + min(i, Tn - 1)];
        if (!valid) gg = make_float2(-2.f, -2.f);
        const float ix = (gg.x + 1.0f) * sxs;
        const float iy = (gg.y + 1.0f) * sys;
        const float x0f = floorf(ix), y0f = floorf(iy);
        const float wx = ix - x0f, ex = 1.0f - wx;
        const float ny = iy - y0f, syw = 1.0f - ny;
        const float nw = syw * ex, ne = syw * wx, sw = ny * ex, se = ny * wx;
        const bool isnan_ = (ix != ix) || (iy != iy);
        const int x0 = isnan_ ? -4 : (int)x0f, y0 = isnan_ ? -4 : (int)y0f;
        const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
        const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
        const bool any = (vx0 | vx1) & (vy0 | vy1);
        if (isnan_) {
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] = acc[k] + NAN;
        }
        if (!__builtin_amdgcn_ballot_w64(any)) continue;
        const __amdgpu_buffer_rsrc_t rs = rsrc_for(cl + ((size_t)b * V + v) * HW * JP, HW * JP * 4u);
        const unsigned pix = (unsigned)(y0 * W + x0);
        const unsigned qo = (unsigned)q * 16u;
        const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy0 & vx0) ? pix * (JP * 4u) + qo : kOOB, 0, 0);
        const auto bq = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy0 & vx1) ? (pix + 1u) * (JP * 4u) + qo : kOOB, 0, 0);
        const auto c = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy1 & vx0) ? (pix + (unsigned)W) * (JP * 4u) + qo : kOOB, 0, 0);
        const auto d = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy1 & vx1) ? (pix + (unsigned)W + 1u) * (JP * 4u) + qo : kOOB, 0, 0);
        if (!isnan_) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float fa = __builtin_bit_cast(float, (unsigned)a[k]);
                const float fb = __builtin_bit_cast(float, (unsigned)bq[k]);
                const float fc = __builtin_bit_cast(float, (unsigned)c[k]);
                const float fd = __builtin_bit_cast(float, (unsigned)d[k]);
                acc[k] = acc[k] + __builtin_fmaf(fd, se, __builtin_fmaf(fc, sw, __builtin_fmaf(fb, ne, fa * nw)));
            }
        }
    }
    const float fV = (float)V;
    if (valid) {
#pragma unroll
        for (int k = 0; k < 4; ++k) stage[(4 * q + k) * SP + i] = clampf(acc[k] / fV, 0.f, 1.f);
    }
    __syncthreads();
    for (int j = 0; j < J; ++j)
        for (int e = threadIdx.x; e < Tn; e += blockDim.x) cube[((size_t)b * J + j) * N + n0 + e] = stage[j * SP + e];
    for (int e = threadIdx.x; e < J * ncols; e += blockDim.x) {
        const int j = e / ncols, cc = e - (e / ncols) * ncols;
        float m = -INFINITY;
        const float *s = stage + j * SP + cc * Z;
        for (int z = 0; z < Z; ++z) m = nanmax(m, s[z]);
        xy[(((size_t)b * J + j) * X + x) * Y + yb + cc] = m;
    }
}
}  // namespace fvpx

extern "C" int voxvar_cl3(int region, int rx, int ry, const float *cl, int B, int V, int J, int H, int W,
                          const float *grids, int X, int Y, int Z, float *cube, float *xy, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (J > 16) return -1;
    const int CT = (80 / Z) > 1 ? (80 / Z) : 1;
    const int threads = ((CT * Z * 4 + 63) / 64) * 64;
    if (threads > 512) return -3;
    const int ytiles = (Y + CT - 1) / CT;
    const size_t lds = (size_t)16 * (CT * Z + 1) * 4;
    const long long blocks = (long long)B * X * ytiles;
    if (region) {
        if (rx * ry != 8 || X % rx || ytiles % ry) return -4;
        hipLaunchKernelGGL((fvpx::vox_cl3<true>), dim3((unsigned)blocks), dim3(threads), lds, s, cl,
                           reinterpret_cast<const float2 *>(grids), cube, xy, V, J, H, W, X, Y, Z, CT, ytiles, rx, ry);
    } else {
        hipLaunchKernelGGL((fvpx::vox_cl3<false>), dim3((unsigned)blocks), dim3(threads), lds, s, cl,
                           reinterpret_cast<const float2 *>(grids), cube, xy, V, J, H, W, X, Y, Z, CT, ytiles, rx, ry);
    }
    return (int)hipGetLastError();
}

// v4: camera-outer loop (all passes of a block for camera v, then v+1), so the
// blocks resident on an XCD tend to sample the same camera image at the same
// time (L2 working set ~ one camera instead of all V).  Accumulators for every
// pass live in registers; the per-voxel sum order over cameras is unchanged.
namespace fvpx {
template <int MAXP>
__global__ __launch_bounds__(256) void vox_cl4(const float *__restrict__ cl, const float2 *__restrict__ grids,
                                               float *__restrict__ cube, float *__restrict__ xy, int V, int J, int H,
                                               int W, int X, int Y, int Z, int cols, int col_blocks) {
    constexpr int LPV = 4, JP = 16, VPP = 64;
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int b = L / col_blocks;
    const int c0 = (L - b * col_blocks) * cols;
    const int XY = X * Y;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const int SP = cols * Z + 1;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const unsigned HW = (unsigned)(H * W);
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    float acc[MAXP][4];
#pragma unroll
    for (int p = 0; p < MAXP; ++p)
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[p][k] = 0.f;
    for (int v = 0; v < V; ++v) {
        const __amdgpu_buffer_rsrc_t rs = rsrc_for(cl + ((size_t)b * V + v) * HW * JP, HW * JP * 4u);
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
            const int i = p * VPP + threadIdx.x / LPV;
            const bool valid = i < T;
            float2 gg = grids[(size_t)v * N + n0 + min(i, T - 1)];
            if (!valid) gg = make_float2(-2.f, -2.f);
            const float ix = (gg.x + 1.0f) * sxs;
            const float iy = (gg.y + 1.0f) * sys;
            const float x0f = floorf(ix), y0f = floorf(iy);
            const float wx = ix - x0f, ex = 1.0f - wx;
            const float ny = iy - y0f, syw = 1.0f - ny;
            const float nw = syw * ex, ne = syw * wx, sw = ny * ex, se = ny * wx;
            const bool isnan_ = (ix != ix) || (iy != iy);
            const int x0 = isnan_ ? -4 : (int)x0f, y0 = isnan_ ? -4 : (int)y0f;
            const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
            const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
            const unsigned pix = (unsigned)(y0 * W + x0);
            const unsigned qo = (unsigned)q * 16u;
            const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy0 & vx0) ? pix * (JP * 4u) + qo : kOOB, 0, 0);
            const auto bq = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy0 & vx1) ? (pix + 1u) * (JP * 4u) + qo : kOOB, 0, 0);
            const auto c = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy1 & vx0) ? (pix + (unsigned)W) * (JP * 4u) + qo : kOOB, 0, 0);
            const auto d = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy1 & vx1) ? (pix + (unsigned)W + 1u) * (JP * 4u) + qo : kOOB, 0, 0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float fa = __builtin_bit_cast(float, (unsigned)a[k]);
                const float fb = __builtin_bit_cast(float, (unsigned)bq[k]);
                const float fc = __builtin_bit_cast(float, (unsigned)c[k]);
                const float fd = __builtin_bit_cast(float, (unsigned)d[k]);
                const float val = isnan_ ? NAN : __builtin_fmaf(fd, se, __builtin_fmaf(fc, sw, __builtin_fmaf(fb, ne, fa * nw)));
                acc[p][k] = acc[p][k] + val;
            }
        }
    }
    const float fV = (float)V;
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
        const int i = p * VPP + threadIdx.x / LPV;
        if (i < T) {
#pragma unroll
            for (int k = 0; k < 4; ++k) stage[(4 * q + k) * SP + i] = clampf(acc[p][k] / fV, 0.f, 1.f);
        }
    }
    __syncthreads();
    for (int j = 0; j < J; ++j)
        for (int e = threadIdx.x; e < T; e += 256) cube[((size_t)b * J + j) * N + n0 + e] = stage[j * SP + e];
    for (int e = threadIdx.x; e < J * ncols; e += 256) {
        const int j = e / ncols, cc = e - (e / ncols) * ncols;
        float m = -INFINITY;
        const float *s = stage + j * SP + cc * Z;
        for (int z = 0; z < Z; ++z) m = nanmax(m, s[z]);
        xy[((size_t)b * J + j) * XY + c0 + cc] = m;
    }
}
}  // namespace fvpx

extern "C" int voxvar_cl4(int cols, const float *cl, int B, int V, int J, int H, int W, const float *grids, int X,
                          int Y, int Z, float *cube, float *xy, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int XY = X * Y;
    const int cb = (XY + cols - 1) / cols;
    const size_t lds = (size_t)16 * (cols * Z + 1) * 4;
    const int passes = (cols * Z + 63) / 64;
    if (J > 16) return -1;
#define CL4(P) hipLaunchKernelGGL((fvpx::vox_cl4<P>), dim3(cb * B), dim3(256), lds, s, cl, \
                                  reinterpret_cast<const float2 *>(grids), cube, xy, V, J, H, W, X, Y, Z, cols, cb)
    if (passes <= 3) CL4(3);
    else if (passes <= 5) CL4(5);
    else if (passes <= 10) CL4(10);
    else return -2;
#undef CL4
    return (int)hipGetLastError();
}

// v5: cl + all cameras' grid coordinates loaded up front (one latency instead
// of V), tap loads of camera v+1 issued before camera v is consumed (2 deep),
// ballot skip kept.
namespace fvpx {
template <int VMAX>
__global__ __launch_bounds__(256) void vox_cl5(const float *__restrict__ cl, const float2 *__restrict__ grids,
                                               float *__restrict__ cube, float *__restrict__ xy, int V, int J, int H,
                                               int W, int X, int Y, int Z, int cols, int col_blocks) {
    constexpr int LPV = 4, JP = 16, VPP = 64;
    using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int b = L / col_blocks;
    const int c0 = (L - b * col_blocks) * cols;
    const int XY = X * Y;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const int SP = cols * Z + 1;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const unsigned HW = (unsigned)(H * W);
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    const unsigned qo = (unsigned)q * 16u;
    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        float2 g[VMAX];
#pragma unroll
        for (int u = 0; u < VMAX; ++u) {
            g[u] = grids[(size_t)min(u, V - 1) * N + n0 + min(i, T - 1)];
            if (!valid) g[u] = make_float2(-2.f, -2.f);
        }
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        // per camera: weights, tap data, flags
        float wt[2][4];
        u32x4 d[2][4];
        bool nanv[2], act[2];
        auto issue = [&](int u, int slot) {
            const float ix = (g[u].x + 1.0f) * sxs;
            const float iy = (g[u].y + 1.0f) * sys;
            const float x0f = floorf(ix), y0f = floorf(iy);
            const float wx = ix - x0f, ex = 1.0f - wx;
            const float ny = iy - y0f, syw = 1.0f - ny;
            wt[slot][0] = syw * ex; wt[slot][1] = syw * wx; wt[slot][2] = ny * ex; wt[slot][3] = ny * wx;
            nanv[slot] = (ix != ix) || (iy != iy);
            const int x0 = nanv[slot] ? -4 : (int)x0f, y0 = nanv[slot] ? -4 : (int)y0f;
            const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
            const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
            act[slot] = __builtin_amdgcn_ballot_w64((vx0 | vx1) & (vy0 | vy1)) != 0;
            if (act[slot]) {
                const __amdgpu_buffer_rsrc_t rs = rsrc_for(cl + ((size_t)b * V + u) * HW * JP, HW * JP * 4u);
                const unsigned pix = (unsigned)(y0 * W + x0);
                d[slot][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy0 & vx0) ? pix * (JP * 4u) + qo : kOOB, 0, 0);
                d[slot][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy0 & vx1) ? (pix + 1u) * (JP * 4u) + qo : kOOB, 0, 0);
                d[slot][2] = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy1 & vx0) ? (pix + (unsigned)W) * (JP * 4u) + qo : kOOB, 0, 0);
                d[slot][3] = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy1 & vx1) ? (pix + (unsigned)W + 1u) * (JP * 4u) + qo : kOOB, 0, 0);
            }
        };
        auto consume = [&](int slot) {
            if (nanv[slot]) {
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] = acc[k] + NAN;
            } else if (act[slot]) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float fa = __builtin_bit_cast(float, d[slot][0][k]);
                    const float fb = __builtin_bit_cast(float, d[slot][1][k]);
                    const float fc = __builtin_bit_cast(float, d[slot][2][k]);
                    const float fd = __builtin_bit_cast(float, d[slot][3][k]);
                    acc[k] = acc[k] + __builtin_fmaf(fd, wt[slot][3], __builtin_fmaf(fc, wt[slot][2],
                                                     __builtin_fmaf(fb, wt[slot][1], fa * wt[slot][0])));
                }
            }
        };
        issue(0, 0);
#pragma unroll
        for (int u = 0; u < VMAX; ++u) {
            if (u + 1 < VMAX && u + 1 < V) issue(u + 1, (u + 1) & 1);
            if (u < V) consume(u & 1);
        }
        if (valid) {
#pragma unroll
            for (int k = 0; k < 4; ++k) stage[(4 * q + k) * SP + i] = clampf(acc[k] / fV, 0.f, 1.f);
        }
    }
    __syncthreads();
    for (int j = 0; j < J; ++j)
        for (int e = threadIdx.x; e < T; e += 256) cube[((size_t)b * J + j) * N + n0 + e] = stage[j * SP + e];
    for (int e = threadIdx.x; e < J * ncols; e += 256) {
        const int j = e / ncols, cc = e - (e / ncols) * ncols;
        float m = -INFINITY;
        const float *s = stage + j * SP + cc * Z;
        for (int z = 0; z < Z; ++z) m = nanmax(m, s[z]);
        xy[((size_t)b * J + j) * XY + c0 + cc] = m;
    }
}
}  // namespace fvpx

extern "C" int voxvar_cl5(int cols, const float *cl, int B, int V, int J, int H, int W, const float *grids, int X,
                          int Y, int Z, float *cube, float *xy, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int XY = X * Y;
    const int cb = (XY + cols - 1) / cols;
    const size_t lds = (size_t)16 * (cols * Z + 1) * 4;
    if (J > 16 || V != 5) return -1;
    hipLaunchKernelGGL((fvpx::vox_cl5<5>), dim3(cb * B), dim3(256), lds, s, cl, reinterpret_cast<const float2 *>(grids),
                       cube, xy, V, J, H, W, X, Y, Z, cols, cb);
    return (int)hipGetLastError();
}
