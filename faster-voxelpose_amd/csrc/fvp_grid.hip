// Per-sequence sample grid (A1-A4 of SURVEY.md §8(a)).
//
// One thread per (camera, voxel): rebuild the voxel centre from the linspace
// axes (project_whole.py:43-79), project it (cameras.py:30-56), clamp, apply
// the resize affine (transforms.py:59-63), scale and normalise
// (project_whole.py:96-117).  Bit-exact with the reference CPU path (see
// fvp_device.h).  Runs once per sequence; HBM-bound on the V*N*8-byte write.
#include "fvp_device.h"

namespace fvp {

__global__ __launch_bounds__(256) void project_grid_kernel(
    const float *__restrict__ cams, const float *__restrict__ resize_t, fvp_grid_spec g, ImageConsts im,
    float2 *__restrict__ out, int V, long long N) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int v = blockIdx.y;
    if (gid >= N || v >= V) return;
    const int Z = g.bins[2], Y = g.bins[1];
    const int iz = (int)(gid % Z);
    const long long r = gid / Z;
    const int iy = (int)(r % Y);
    const int ix = (int)(r / Y);
    const float x = axis_coord(g.start[0], g.end[0], g.bins[0], ix, g.center[0]);
    const float y = axis_coord(g.start[1], g.end[1], g.bins[1], iy, g.center[1]);
    const float z = axis_coord(g.start[2], g.end[2], g.bins[2], iz, g.center[2]);
    const Cam c = load_cam(cams + (size_t)v * FVP_CAM_STRIDE);
    float px, py, gx, gy;
    project_point(c, x, y, z, px, py);
    pixel_to_sample(px, py, resize_t, im, gx, gy);
    out[(size_t)v * N + gid] = make_float2(gx, gy);
}

}  // namespace fvp

extern "C" int fvp_project_grid(const float *cams, int V, const float *resize_t, const fvp_grid_spec *grid,
                                const fvp_image_spec *img, float *sample_grid, void *stream) {
    if (!cams || !resize_t || !grid || !img || !sample_grid) return FVP_ERR_NULL;
    if (V <= 0 || V > 65535 || grid->bins[0] <= 0 || grid->bins[1] <= 0 || grid->bins[2] <= 0 || img->hm_w < 2 ||
        img->hm_h < 2)
        return FVP_ERR_SHAPE;
    const long long N = (long long)grid->bins[0] * grid->bins[1] * grid->bins[2];
    const long long blocks = (N + 255) / 256;
    if (blocks > 0x7fffffffLL) return FVP_ERR_SHAPE;
    dim3 gdim((unsigned)blocks, (unsigned)V);
    hipLaunchKernelGGL(fvp::project_grid_kernel, gdim, dim3(256), 0, (hipStream_t)stream, cams, resize_t, *grid,
                       fvp::image_consts(*img), reinterpret_cast<float2 *>(sample_grid), V, N);
    return (int)hipGetLastError();
}
