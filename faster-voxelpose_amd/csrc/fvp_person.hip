// Per-person voxel cubes from the cached fine sample grid (A11-A13) and the
// JLN xy/xz/yz max-projections (A8).
//
// person_cubes replaces project_individual.ProjectLayer.forward
// (project_individual.py:222-293) without its host syncs: every block
// recomputes its proposal's window (centers_tl, margins, start/end, skip
// flag, :255-275) from the proposal row, so no per-proposal launch or
// torch.sum(...) readback is needed.  One thread per output voxel (x, y, z),
// all joints in registers; lanes run along z so grid reads and cube writes
// are contiguous.
//
// max_planes replaces torch.cat([max(c,4), max(c,3), max(c,2)])
// (joint_localization_net.py:158-160): one block per (person, joint) reads the
// S^3 cube once; lane = z, each wave owns S/4 y-rows; yz is a register max
// over x, xz a register + LDS max over y, xy a wave reduction over z.
#include "fvp_device.h"

namespace fvp {

struct Window {
    int ctl[3], start[3], end[3];
    bool skip;
};

__device__ __forceinline__ Window person_window(const float *__restrict__ pc, const fvp_person_spec &s) {
    Window w;
    // centers_tl = round(center * scale + bias).int()   (:255, round half to even)
#pragma unroll
    for (int a = 0; a < 3; ++a) w.ctl[a] = (int)rintf(pc[a] * s.scale[a] + s.bias[a]);
    // mask = ((1 - bbox) / 2 * (vpa[0:2] - 1)).int(), negatives -> 0, z margin 0  (:262-265)
    int m[3];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const float f = ((1.0f - pc[5 + a]) / 2.0f) * (float)(s.bins[a] - 1);
        int mi = (int)f;  // trunc toward zero, as .int()
        m[a] = mi < 0 ? 0 : mi;
    }
    m[2] = 0;
    w.skip = false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int lo = w.ctl[a] + m[a];
        const int hi = w.ctl[a] + s.bins[a] - m[a];
        w.start[a] = lo >= 0 ? lo : 0;                   // :268
        w.end[a] = hi <= s.fine[a] ? hi : s.fine[a];     // :269
        w.skip |= (w.start[a] >= w.end[a]);              // :274-275
    }
    return w;
}

template <int JT>
__global__ __launch_bounds__(256) void person_cubes_kernel(const float *__restrict__ hm,
                                                           const float2 *__restrict__ fgrid,
                                                           const float *__restrict__ props, fvp_person_spec s,
                                                           float *__restrict__ cubes, float *__restrict__ offset,
                                                           int V, int J, int H, int W) {
    const int p = blockIdx.z;
    const int SX = s.bins[0], SY = s.bins[1], SZ = s.bins[2];
    const int ox = blockIdx.y;
    const int oz = threadIdx.x % SZ;  // SZ <= 256 and divides blockDim handled below
    const int oy = blockIdx.x * (blockDim.x / SZ) + threadIdx.x / SZ;
    const bool inside = (oy < SY) && (threadIdx.x < (blockDim.x / SZ) * SZ);
    const Window w = person_window(props + (size_t)p * 7, s);

    if (offset && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 3) {
        const int a = threadIdx.x;
        // offset = ctl.float() / (fine - 1) * ws - ws / 2 + isz / 2   (:258)
        offset[(size_t)p * 3 + a] =
            ((float)w.ctl[a] / (float)(s.fine[a] - 1)) * s.whole_size[a] - s.whole_size[a] / 2.0f +
            s.ind_size[a] / 2.0f;
    }
    if (!inside) return;

    const int gx = w.ctl[0] + ox, gy = w.ctl[1] + oy, gz = w.ctl[2] + oz;
    const bool valid = !w.skip && gx >= w.start[0] && gx < w.end[0] && gy >= w.start[1] && gy < w.end[1] &&
                       gz >= w.start[2] && gz < w.end[2];
    const size_t HW = (size_t)H * W;
    const long long FN = (long long)s.fine[0] * s.fine[1] * s.fine[2];
    const long long gn = valid ? ((long long)gx * s.fine[1] + gy) * s.fine[2] + gz : 0;
    const size_t S3 = (size_t)SX * SY * SZ;
    const size_t cell = ((size_t)ox * SY + oy) * SZ + oz;
    const float fV = (float)V;

    for (int j0 = 0; j0 < J; j0 += JT) {
        float acc[JT];
#pragma unroll
        for (int jj = 0; jj < JT; ++jj) acc[jj] = 0.0f;
        if (valid) {
            for (int v = 0; v < V; ++v) {
                const float2 gg = fgrid[(size_t)v * FN + gn];
                const Taps tp = make_taps(gg.x, gg.y, H, W);
                if (tp.nan) {
#pragma unroll
                    for (int jj = 0; jj < JT; ++jj) acc[jj] = acc[jj] + NAN;
                } else if (tp.any) {
                    const float *__restrict__ base = hm + ((size_t)v * J + j0) * HW;
#pragma unroll
                    for (int jj = 0; jj < JT; ++jj)
                        if (j0 + jj < J) acc[jj] = acc[jj] + sample(base + (size_t)jj * HW, tp);
                }
            }
        }
#pragma unroll
        for (int jj = 0; jj < JT; ++jj) {
            if (j0 + jj < J) {
                const float o = valid ? clampf(acc[jj] / fV, 0.0f, 1.0f) : 0.0f;
                cubes[((size_t)p * J + j0 + jj) * S3 + cell] = o;
            }
        }
    }
}

// planes: [3P][J][S][S]; block (p, j); 256 threads = 4 waves, lane = z.
__global__ __launch_bounds__(256) void max_planes_kernel(const float *__restrict__ cubes, float *__restrict__ planes,
                                                         int P, int J, int S) {
    __shared__ float xz_part[4][64];
    const int p = blockIdx.x / J, j = blockIdx.x % J;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool zok = lane < S;
    const size_t SS = (size_t)S * S;
    const float *__restrict__ c = cubes + ((size_t)p * J + j) * SS * S;
    float *__restrict__ pxy = planes + ((size_t)(0 * P + p) * J + j) * SS;
    float *__restrict__ pxz = planes + ((size_t)(1 * P + p) * J + j) * SS;
    float *__restrict__ pyz = planes + ((size_t)(2 * P + p) * J + j) * SS;
    constexpr int kRows = 16;  // y rows per wave (S <= 64)
    float yz[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) yz[r] = -INFINITY;

    for (int x = 0; x < S; ++x) {
        float xzm = -INFINITY;
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            const int y = wave + 4 * r;
            const bool ok = zok && y < S;
            const float v = ok ? c[((size_t)x * S + y) * S + lane] : -INFINITY;
            yz[r] = nanmax(yz[r], v);
            xzm = nanmax(xzm, v);
            // xy[x][y] = max over z (wave reduction; y is wave-uniform)
            float m = v;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) m = nanmax(m, __shfl_xor(m, off));
            if (lane == 0 && y < S) pxy[(size_t)x * S + y] = m;
        }
        xz_part[wave][lane] = xzm;
        __syncthreads();
        if (wave == 0 && zok) {
            float m = xz_part[0][lane];
            m = nanmax(m, xz_part[1][lane]);
            m = nanmax(m, xz_part[2][lane]);
            m = nanmax(m, xz_part[3][lane]);
            pxz[(size_t)x * S + lane] = m;
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int y = wave + 4 * r;
        if (zok && y < S) pyz[(size_t)y * S + lane] = yz[r];
    }
}

}  // namespace fvp

extern "C" int fvp_person_cubes(const float *heatmaps, int V, int J, int H, int W, const float *fine_grid,
                                const fvp_person_spec *spec, const float *proposals, int P, float *cubes,
                                float *offset, void *stream) {
    if (!heatmaps || !fine_grid || !spec || !cubes) return FVP_ERR_NULL;
    if (P <= 0) return FVP_OK;
    if (!proposals) return FVP_ERR_NULL;
    if (V <= 0 || J <= 0 || H < 2 || W < 2) return FVP_ERR_SHAPE;
    const int SX = spec->bins[0], SY = spec->bins[1], SZ = spec->bins[2];
    if (SX <= 0 || SY <= 0 || SZ <= 0 || SZ > 256 || spec->fine[0] <= 1 || spec->fine[1] <= 1 ||
        spec->fine[2] <= 1)
        return FVP_ERR_SHAPE;
    const int rows = 256 / SZ;  // y rows per block
    dim3 grid((SY + rows - 1) / rows, SX, P);
    hipLaunchKernelGGL((fvp::person_cubes_kernel<16>), grid, dim3(256), 0, (hipStream_t)stream, heatmaps,
                       reinterpret_cast<const float2 *>(fine_grid), proposals, *spec, cubes, offset, V, J, H, W);
    return (int)hipGetLastError();
}

extern "C" int fvp_max_planes(const float *cubes, int P, int J, int S, float *planes, void *stream) {
    if (!cubes || !planes) return FVP_ERR_NULL;
    if (P <= 0) return FVP_OK;
    if (J <= 0 || S <= 0 || S > 64) return FVP_ERR_SHAPE;
    hipLaunchKernelGGL(fvp::max_planes_kernel, dim3(P * J), dim3(256), 0, (hipStream_t)stream, cubes, planes, P, J,
                       S);
    return (int)hipGetLastError();
}
