// Whole-space voxelisation fused with the xy max-projection (A5-A7).
//
// Reference: project_whole.py:119-168 (grid_sample per frame, mean over all V
// cameras, clamp(0,1)) and cnns_2d.py:291 (max over z).
//
// Work decomposition (gfx950, wave64):
//   * a wave owns a 4x4 block of (x,y) voxel columns; its 64 lanes are
//     (x4, y4, z4) so one load instruction touches a compact 3-D voxel block,
//     whose projections are a compact pixel patch (L1/L2 line reuse between
//     the four bilinear taps and between neighbouring lanes);
//   * the wave walks the z axis in steps of 4; each lane accumulates all J
//     joints of its voxel in registers (coordinates and weights computed once
//     per voxel-camera, reused for every joint plane);
//   * the xy max over z is a running register max per lane plus two
//     cross-lane steps (lanes differing in z4) at the end -- no LDS, no atomics;
//   * a 256-thread block = 2x2 waves = an 8x8 column tile of one frame; the
//     blockIdx is remapped so each XCD processes whole frames (its L2 holds the
//     frame's heatmap planes while its tiles sample them).
// Voxel-cameras whose four taps are all outside the image (clamped +-1.1
// coordinates) contribute exactly 0 and issue no loads.
#include "fvp_device.h"

namespace fvp {

template <int JT, typename T>
__global__ __launch_bounds__(256) void voxelize_kernel(const T *__restrict__ hm, const float2 *__restrict__ grids,
                                                       const int32_t *__restrict__ grid_index,
                                                       float *__restrict__ cube, float *__restrict__ xy, int V,
                                                       int J, int H, int W, int X, int Y, int Z, int tiles_y,
                                                       int tiles_per_frame) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int b = L / tiles_per_frame;
    const int t = L - b * tiles_per_frame;
    const int tx = t / tiles_y, ty = t - (t / tiles_y) * tiles_y;
    const int x = tx * 8 + (wave >> 1) * 4 + (lane >> 4);
    const int y = ty * 8 + (wave & 1) * 4 + ((lane >> 2) & 3);
    const int zi = lane & 3;
    const bool col_ok = (x < X) && (y < Y);

    const long long N = (long long)X * Y * Z;
    const size_t HW = (size_t)H * W;
    const int gsel = grid_index ? grid_index[b] : 0;
    const float2 *__restrict__ g = grids + (size_t)gsel * V * N;
    const T *__restrict__ hmb = hm + (size_t)b * V * J * HW;
    const float fV = (float)V;

    for (int j0 = 0; j0 < J; j0 += JT) {
        float xymax[JT];
#pragma unroll
        for (int jj = 0; jj < JT; ++jj) xymax[jj] = -INFINITY;

        for (int z0 = 0; z0 < Z; z0 += 4) {
            const int z = z0 + zi;
            const bool valid = col_ok && (z < Z);
            const long long n = ((long long)x * Y + y) * Z + z;
            float acc[JT];
#pragma unroll
            for (int jj = 0; jj < JT; ++jj) acc[jj] = 0.0f;
            if (valid) {
                for (int v = 0; v < V; ++v) {
                    const float2 gg = g[(size_t)v * N + n];
                    const Taps tp = make_taps(gg.x, gg.y, H, W);
                    if (tp.nan) {
#pragma unroll
                        for (int jj = 0; jj < JT; ++jj) acc[jj] = acc[jj] + NAN;
                    } else if (tp.any) {
                        const T *__restrict__ base = hmb + ((size_t)v * J + j0) * HW;
#pragma unroll
                        for (int jj = 0; jj < JT; ++jj) {
                            if (j0 + jj < J) acc[jj] = acc[jj] + sample(base + (size_t)jj * HW, tp);
                        }
                    }
                }
            }
#pragma unroll
            for (int jj = 0; jj < JT; ++jj) {
                if (j0 + jj < J) {
                    const float o = clampf(acc[jj] / fV, 0.0f, 1.0f);
                    if (valid) {
                        if (cube) cube[((size_t)b * J + j0 + jj) * N + n] = o;
                        xymax[jj] = nanmax(xymax[jj], o);
                    }
                }
            }
        }
        if (xy) {
#pragma unroll
            for (int jj = 0; jj < JT; ++jj) {
                float m = xymax[jj];
                m = nanmax(m, __shfl_xor(m, 1));
                m = nanmax(m, __shfl_xor(m, 2));
                if (j0 + jj < J && zi == 0 && col_ok) xy[(((size_t)b * J + j0 + jj) * X + x) * Y + y] = m;
            }
        }
    }
}

template <typename T>
static int launch_voxelize(const T *hm, int B, int V, int J, int H, int W, const float *grids,
                           const int32_t *grid_index, int X, int Y, int Z, float *cube, float *xy, hipStream_t s) {
    const int tiles_x = (X + 7) / 8, tiles_y = (Y + 7) / 8;
    const long long tiles = (long long)tiles_x * tiles_y;
    const long long blocks = tiles * B;
    if (blocks > 0x7fffffffLL) return FVP_ERR_SHAPE;
    hipLaunchKernelGGL((voxelize_kernel<16, T>), dim3((unsigned)blocks), dim3(256), 0, s, hm,
                       reinterpret_cast<const float2 *>(grids), grid_index, cube, xy, V, J, H, W, X, Y, Z, tiles_y,
                       (int)tiles);
    return (int)hipGetLastError();
}

}  // namespace fvp

extern "C" int fvp_voxelize(const float *heatmaps, int B, int V, int J, int H, int W, const float *sample_grids,
                            const int32_t *grid_index, int X, int Y, int Z, float *cube, float *xy, void *stream) {
    if (!heatmaps || !sample_grids) return FVP_ERR_NULL;
    if (B <= 0 || V <= 0 || J <= 0 || H < 2 || W < 2 || X <= 0 || Y <= 0 || Z <= 0) return FVP_ERR_SHAPE;
    if (!cube && !xy) return FVP_OK;
    return fvp::launch_voxelize<float>(heatmaps, B, V, J, H, W, sample_grids, grid_index, X, Y, Z, cube, xy,
                                       (hipStream_t)stream);
}
