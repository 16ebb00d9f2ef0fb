// Whole-space voxelisation fused with the xy max-projection (A5-A7).
//
// Reference: project_whole.py:119-168 (grid_sample per frame, mean over all V
// cameras, clamp(0,1)) and cnns_2d.py:291 (max over z).
//
// Why two kernels.  A bilinear tap of all J joints touches J separate
// [H][W] planes in the reference layout.  On gfx950 the texture addresser
// only merges ADJACENT lanes that fall in one 128-B line (a quad per clock);
// scattered per-joint taps cost ~64 clocks per wave load (tools/ta_probe.py),
// and a voxel-camera needs 2 rows x J planes of lines.  So each chunk of
// frames is first re-laid out channels-last:
//   heatmaps_to_cl : [B][V][J][H][W]  ->  [b][V][H][W][JP]   (JP = 4*LPV >= J, zero padded)
// a pure streaming pass, then
//   voxelize_cl    : LPV lanes share one voxel; lane q loads 16 B = joints
//                    4q..4q+3 of each tap with one buffer_load_dwordx4, so a
//                    quad reads one 64-B pixel in one clock; out-of-image taps
//                    use an out-of-range offset and read 0 through the buffer
//                    descriptor's range check (= grid_sample's zero padding).
// The chunk's channels-last copy is sized to stay in the 256 MB Infinity
// Cache between the two launches.
//
// voxelize_cl work decomposition: a 256-thread block owns COLS whole voxel
// columns (x, y..y+COLS, all z) of one frame -- a contiguous range of the
// cube -- processed in passes of 256/LPV voxels; results are staged in LDS
// so the cube is written as contiguous runs per joint and the xy max over z
// is read back from LDS.  Arithmetic per tap and the camera/sum order are the
// reference's (fvp_device.h), so the result is bit-exact.
#include "fvp_layout.h"

namespace fvp {

// -- gather pass ----------------------------------------------------------------
template <int LPV>
__global__ __launch_bounds__(256) void voxelize_cl_kernel(const float *__restrict__ cl, const float2 *__restrict__ grids,
                                                          const int32_t *__restrict__ grid_index, int frame0,
                                                          float *__restrict__ cube, float *__restrict__ xy, int V,
                                                          int J, int H, int W, int X, int Y, int Z, int cols,
                                                          int col_blocks) {
    constexpr int JP = 4 * LPV;
    constexpr int VPP = 256 / LPV;  // voxels per pass
    extern __shared__ __attribute__((aligned(16))) float stage[];  // [JP][SP]
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int bl = L / col_blocks;   // frame within the chunk
    const int b = frame0 + bl;       // frame within the batch (outputs, grid_index)
    const int XY = X * Y;
    const int c0 = (L - bl * col_blocks) * cols;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const int SP = cols * Z + 1;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const unsigned HW = (unsigned)(H * W);
    const unsigned pix_bytes = JP * 4u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    const int gsel = grid_index ? grid_index[b] : 0;
    const float2 *__restrict__ g = grids + (size_t)gsel * V * N + n0;

    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int v = 0; v < V; ++v) {
            float2 gg = g[(size_t)v * N + min(i, T - 1)];
            if (!valid) gg = make_float2(-2.f, -2.f);
            const float ix = (gg.x + 1.0f) * sxs;
            const float iy = (gg.y + 1.0f) * sys;
            const bool isnan_ = (ix != ix) || (iy != iy);
            if (isnan_) {  // grid_sample of a NaN coordinate is NaN (0 * NaN weights)
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] = acc[k] + NAN;
            }
            const float x0f = floorf(ix), y0f = floorf(iy);
            const float wx = ix - x0f, ex = 1.0f - wx;
            const float ny = iy - y0f, syw = 1.0f - ny;
            const float nw = syw * ex, ne = syw * wx, sw = ny * ex, se = ny * wx;
            const int x0 = isnan_ ? -4 : (int)x0f, y0 = isnan_ ? -4 : (int)y0f;
            const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
            const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
            const bool any = (vx0 | vx1) & (vy0 | vy1);
            if (!__builtin_amdgcn_ballot_w64(any)) continue;  // whole wave off-image: contributes exactly 0
            const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(cl + ((size_t)bl * V + v) * HW * JP, HW * pix_bytes);
            const unsigned pix = (unsigned)(y0 * W + x0);
            const unsigned qo = (unsigned)q * 16u;
            const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, (vy0 & vx0) ? pix * pix_bytes + qo : kOOB, 0, 0);
            const auto bq =
                __builtin_amdgcn_raw_buffer_load_b128(rs, (vy0 & vx1) ? (pix + 1u) * pix_bytes + qo : kOOB, 0, 0);
            const auto c = __builtin_amdgcn_raw_buffer_load_b128(
                rs, (vy1 & vx0) ? (pix + (unsigned)W) * pix_bytes + qo : kOOB, 0, 0);
            const auto d = __builtin_amdgcn_raw_buffer_load_b128(
                rs, (vy1 & vx1) ? (pix + (unsigned)W + 1u) * pix_bytes + qo : kOOB, 0, 0);
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
            for (int k = 0; k < 4; ++k) stage[(4 * q + k) * SP + i] = clampf(acc[k] / fV, 0.0f, 1.0f);
        }
    }
    __syncthreads();
    if (cube) {
        for (int j = 0; j < J; ++j) {
            float *__restrict__ dst = cube + ((size_t)b * J + j) * N + n0;
            for (int e = threadIdx.x; e < T; e += 256) dst[e] = stage[j * SP + e];
        }
    }
    if (xy) {
        for (int e = threadIdx.x; e < J * ncols; e += 256) {
            const int j = e / ncols, cc = e - (e / ncols) * ncols;
            const float *s = stage + j * SP + cc * Z;
            float m = -INFINITY;
            for (int z = 0; z < Z; ++z) m = nanmax(m, s[z]);
            xy[((size_t)b * J + j) * XY + c0 + cc] = m;
        }
    }
}


static int cols_per_block(int Z) { return Z >= 320 ? 1 : 320 / Z; }


// Frames per chunk: keep the channels-last copy of a chunk well inside the
// 256 MB Infinity Cache (measured best at ~64-80 MB for C2: 8 frames).
static int chunk_frames(int B, int V, int J, int H, int W) {
    const size_t per = cl_frame_bytes(V, J, H, W);
    long long c = (long long)((80ull << 20) / (per ? per : 1));
    if (c < 1) c = 1;
    if (c > B) c = B;
    return (int)c;
}

template <int LPV, typename T>
static int run_chunks(const T *hm, int B, int V, int J, int H, int W, const float *grids, const int32_t *grid_index,
                      int X, int Y, int Z, float *cube, float *xy, float *ws, hipStream_t s) {
    const int chunk = chunk_frames(B, V, J, H, W);
    const int cols = cols_per_block(Z);
    const int col_blocks = (X * Y + cols - 1) / cols;
    const size_t lds = (size_t)4 * LPV * (cols * Z + 1) * sizeof(float);
    const size_t frame_elems = (size_t)V * J * H * W;
    for (int f0 = 0; f0 < B; f0 += chunk) {
        const int nb = min(chunk, B - f0);
        const long long px = (long long)nb * V * H * W;
        const long long threads = px * LPV;
        hipLaunchKernelGGL((heatmaps_to_cl_kernel<LPV, T>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                           hm + (size_t)f0 * frame_elems, reinterpret_cast<float4 *>(ws), J, H * W, px);
        hipLaunchKernelGGL((voxelize_cl_kernel<LPV>), dim3((unsigned)(nb * col_blocks)), dim3(256), lds, s, ws,
                           reinterpret_cast<const float2 *>(grids), grid_index, f0, cube, xy, V, J, H, W, X, Y, Z,
                           cols, col_blocks);
    }
    return (int)hipGetLastError();
}

template <typename T>
static int voxelize_any(const T *hm, int B, int V, int J, int H, int W, const float *grids, const int32_t *grid_index,
                        int X, int Y, int Z, float *cube, float *xy, void *ws, size_t ws_bytes, hipStream_t s) {
    const size_t need = (size_t)chunk_frames(B, V, J, H, W) * cl_frame_bytes(V, J, H, W);
    if (!ws || ws_bytes < need) return FVP_ERR_WORKSPACE;
    if ((long long)V * H * W * 4 * lanes_per_voxel(J) * 4 > 0x7fffffffLL) return FVP_ERR_SHAPE;  // 32-bit offsets
    float *w = reinterpret_cast<float *>(ws);
    switch (lanes_per_voxel(J)) {
        case 1: return run_chunks<1, T>(hm, B, V, J, H, W, grids, grid_index, X, Y, Z, cube, xy, w, s);
        case 2: return run_chunks<2, T>(hm, B, V, J, H, W, grids, grid_index, X, Y, Z, cube, xy, w, s);
        case 4: return run_chunks<4, T>(hm, B, V, J, H, W, grids, grid_index, X, Y, Z, cube, xy, w, s);
        default: return run_chunks<8, T>(hm, B, V, J, H, W, grids, grid_index, X, Y, Z, cube, xy, w, s);
    }
}

static int check_args(const void *heatmaps, int B, int V, int J, int H, int W, const float *grids, int X, int Y, int Z) {
    if (!heatmaps || !grids) return FVP_ERR_NULL;
    if (B <= 0 || V <= 0 || J <= 0 || J > FVP_MAX_JOINTS || H < 2 || W < 2 || X <= 0 || Y <= 0 || Z <= 0)
        return FVP_ERR_SHAPE;
    if ((long long)X * Y * Z > 0x7fffffffLL) return FVP_ERR_SHAPE;
    return FVP_OK;
}

}  // namespace fvp

extern "C" size_t fvp_voxelize_workspace_bytes(int B, int V, int J, int H, int W) {
    if (B <= 0 || V <= 0 || J <= 0 || J > FVP_MAX_JOINTS || H <= 0 || W <= 0) return 0;
    return (size_t)fvp::chunk_frames(B, V, J, H, W) * fvp::cl_frame_bytes(V, J, H, W);
}

extern "C" int fvp_voxelize(const float *heatmaps, int B, int V, int J, int H, int W, const float *sample_grids,
                            const int32_t *grid_index, int X, int Y, int Z, float *cube, float *xy, void *workspace,
                            size_t workspace_bytes, void *stream) {
    const int st = fvp::check_args(heatmaps, B, V, J, H, W, sample_grids, X, Y, Z);
    if (st != FVP_OK) return st;
    if (!cube && !xy) return FVP_OK;
    return fvp::voxelize_any<float>(heatmaps, B, V, J, H, W, sample_grids, grid_index, X, Y, Z, cube, xy, workspace,
                                    workspace_bytes, (hipStream_t)stream);
}

extern "C" int fvp_voxelize_f16(const void *heatmaps, int B, int V, int J, int H, int W, const float *sample_grids,
                                const int32_t *grid_index, int X, int Y, int Z, float *cube, float *xy,
                                void *workspace, size_t workspace_bytes, void *stream) {
    const int st = fvp::check_args(heatmaps, B, V, J, H, W, sample_grids, X, Y, Z);
    if (st != FVP_OK) return st;
    if (!cube && !xy) return FVP_OK;
    return fvp::voxelize_any<_Float16>(reinterpret_cast<const _Float16 *>(heatmaps), B, V, J, H, W, sample_grids,
                                       grid_index, X, Y, Z, cube, xy, workspace, workspace_bytes, (hipStream_t)stream);
}
