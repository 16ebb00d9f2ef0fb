// Experimental gather variants for A/B against the product fvp_voxelize
// (tools/microbench2.py).  Not part of libfvp.so.
//
// qg ("quad grid"): the sample grid is re-laid out voxel-major, [N][GV][2]
// with GV = 2*LPV*ceil(V/(2*LPV)), so the LPV lanes that share a voxel load
// the coordinates of 2*LPV cameras with ONE buffer_load_dwordx4 (one 128-B
// line per quad) instead of one broadcast load per camera; each lane computes
// the bilinear offsets/weights of its two cameras once, and the voxel's
// lanes pick them up per camera through DPP quad broadcasts.  Per
// voxel-camera this removes a grid load and 3/4 of the coordinate VALU.
#include <utility>

#include "../faster-voxelpose_amd/csrc/fvp_voxelize.hip"

namespace fvp {
namespace next {

// broadcast lane S of each LPV-lane voxel group to the whole group
template <int LPV, int S>
__device__ __forceinline__ unsigned bcast(unsigned x) {
    if constexpr (LPV == 1) {
        return x;
    } else if constexpr (LPV == 2) {  // quad_perm [S, S, 2+S, 2+S]
        return (unsigned)__builtin_amdgcn_mov_dpp((int)x, S | (S << 2) | ((2 + S) << 4) | ((2 + S) << 6), 0xf, 0xf,
                                                  false);
    } else if constexpr (LPV == 4) {  // quad_perm [S, S, S, S]
        return (unsigned)__builtin_amdgcn_mov_dpp((int)x, S | (S << 2) | (S << 4) | (S << 6), 0xf, 0xf, false);
    } else {  // 8-lane groups: ds_swizzle bit mode, lane' = (lane & 0x18) | S
        return (unsigned)__builtin_amdgcn_ds_swizzle((int)x, 0x18 | (S << 5));
    }
}


struct Tap {
    unsigned o[4];  // byte offsets of the 4 taps' pixels (kOOB when outside)
    float w[4];     // nw, ne, sw, se
};

// grid_sample unnormalise + bilinear setup for one camera (project_whole.py:162
// through aten grid_sampler_2d, align_corners=True, zeros padding).
__device__ __forceinline__ Tap make_tap(float gx, float gy, float sxs, float sys, int W, int H, unsigned pb) {
    Tap t;
    const float ix = (gx + 1.0f) * sxs;
    const float iy = (gy + 1.0f) * sys;
    const bool nan_ = (ix != ix) || (iy != iy);
    const float x0f = floorf(ix), y0f = floorf(iy);
    const float wx = ix - x0f, ex = 1.0f - wx;
    const float ny = iy - y0f, syw = 1.0f - ny;
    t.w[0] = syw * ex;
    t.w[1] = syw * wx;
    t.w[2] = ny * ex;
    t.w[3] = ny * wx;
    // NaN coordinates: all four taps read in-image pixels so the NaN weights
    // propagate (grid_sample returns NaN); far-away coordinates are clamped
    // before the int conversion.
    const int x0 = nan_ ? 0 : (int)fminf(fmaxf(x0f, -4.0f), (float)W + 4.0f);
    const int y0 = nan_ ? 0 : (int)fminf(fmaxf(y0f, -4.0f), (float)H + 4.0f);
    const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
    const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
    const unsigned p = (unsigned)(y0 * W + x0) * pb;
    t.o[0] = (vy0 & vx0) ? p : kOOB;
    t.o[1] = (vy0 & vx1) ? p + pb : kOOB;
    t.o[2] = (vy1 & vx0) ? p + (unsigned)W * pb : kOOB;
    t.o[3] = (vy1 & vx1) ? p + (unsigned)(W + 1) * pb : kOOB;
    return t;
}

template <int LPV, int MODE, int PF>
__global__ __launch_bounds__(256) void gather_qg(const float *__restrict__ cl, const float4 *__restrict__ gq,
                                                 int GV, const int32_t *__restrict__ grid_index, int frame0,
                                                 float *__restrict__ cube, float *__restrict__ xy, int V, int J, int H,
                                                 int W, int X, int Y, int Z, int cols, int col_blocks) {
    constexpr int JP = 4 * LPV;
    constexpr int VPP = 256 / LPV;
    constexpr int CPG = 2 * LPV;  // cameras per grid load
    static_assert(CPG % PF == 0, "batch must divide the camera group");
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int bl = L / col_blocks;
    const int b = frame0 + bl;
    const int XY = X * Y;
    const int c0 = (L - bl * col_blocks) * cols;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const int SP = cols * Z + 1;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const unsigned HW = (unsigned)(H * W);
    const unsigned pb = JP * 4u;
    const unsigned qo = (unsigned)q * 16u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    const int gsel = grid_index ? grid_index[b] : 0;
    const int G4 = GV / 2;  // float4 per voxel
    const float4 *__restrict__ g = gq + ((size_t)gsel * N + n0) * G4;
    const float *__restrict__ clf = cl + (size_t)bl * V * HW * JP;

    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        const int ii = min(i, T - 1);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int v0 = 0; v0 < V; v0 += CPG) {
            float4 gg;
            if constexpr (MODE == 3 || MODE == 4) {  // timing probe: synthetic in-image coordinates
                const float t = (float)((ii * 7 + q * 13) & 255) * (1.0f / 256.0f) - 0.5f;
                gg = make_float4(t, -t, t * 0.5f, t * 0.25f);
            } else {
                gg = g[(size_t)ii * G4 + v0 / 2 + q];
            }
            if (!valid) gg = make_float4(-2.f, -2.f, -2.f, -2.f);
            const Tap t0 = make_tap(gg.x, gg.y, sxs, sys, W, H, pb);
            const Tap t1 = make_tap(gg.z, gg.w, sxs, sys, W, H, pb);
            static_for(std::make_integer_sequence<int, CPG / PF>{}, [&](auto bc) {
                constexpr int kb = decltype(bc)::value * PF;
                if (v0 + kb >= V) return;
                unsigned o[PF][4];
                float w[PF][4];
                bool any = false;
                static_for(std::make_integer_sequence<int, PF>{}, [&](auto pc) {
                    constexpr int k = kb + decltype(pc)::value;
                    const Tap &src = (k & 1) ? t1 : t0;
                    const bool live = v0 + k < V;
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        o[pc][m] = live ? bcast<LPV, (k >> 1)>(src.o[m]) : kOOB;
                        w[pc][m] = __builtin_bit_cast(float, bcast<LPV, (k >> 1)>(__builtin_bit_cast(unsigned, src.w[m])));
                        if constexpr (MODE == 1) o[pc][m] &= (kOOB | 0xFFFu);
                        if constexpr (MODE == 2 || MODE == 4) o[pc][m] = kOOB;
                    }
                    any |= ((o[pc][0] & o[pc][1] & o[pc][2] & o[pc][3]) & kOOB) == 0u;
                });
                if (!__builtin_amdgcn_ballot_w64(any)) return;
                typedef unsigned u4 __attribute__((ext_vector_type(4)));
                u4 t[PF][4];
                static_for(std::make_integer_sequence<int, PF>{}, [&](auto pc) {
                    constexpr int k = kb + decltype(pc)::value;
                    const int v = min(v0 + k, V - 1);
                    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(clf + (size_t)v * HW * JP, HW * pb);
#pragma unroll
                    for (int m = 0; m < 4; ++m) t[pc][m] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[pc][m] + qo, 0, 0);
                });
                static_for(std::make_integer_sequence<int, PF>{}, [&](auto pc) {
                    constexpr int k = kb + decltype(pc)::value;
                    if (v0 + k >= V) return;
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const float fa = __builtin_bit_cast(float, (unsigned)t[pc][0][m]);
                        const float fb = __builtin_bit_cast(float, (unsigned)t[pc][1][m]);
                        const float fc = __builtin_bit_cast(float, (unsigned)t[pc][2][m]);
                        const float fd = __builtin_bit_cast(float, (unsigned)t[pc][3][m]);
                        acc[m] = acc[m] + __builtin_fmaf(fd, w[pc][3],
                                                         __builtin_fmaf(fc, w[pc][2],
                                                                        __builtin_fmaf(fb, w[pc][1], fa * w[pc][0])));
                    }
                });
            });
        }
        if (valid) {
#pragma unroll
            for (int m = 0; m < 4; ++m) stage[(4 * q + m) * SP + i] = clampf(acc[m] / fV, 0.0f, 1.0f);
        }
    }
    __syncthreads();
    if (cube && MODE != 5) {
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

// Multi-frame variant: a block gathers the same COLS columns for F frames of
// the chunk, so each grid load and each camera's tap setup (make_tap + DPP
// broadcasts) serves F frames.  The grid is read with a ranged buffer load, so
// GV may be any even count >= V (lanes past the row read the next voxel or 0).
template <int LPV, int PF, int F>
__global__ __launch_bounds__(256) void gather_mf(const float *__restrict__ cl, const float *__restrict__ gq, int GV,
                                                 unsigned grid_bytes, int nb, int frame0, float *__restrict__ cube,
                                                 float *__restrict__ xy, int V, int J, int H, int W, int X, int Y,
                                                 int Z, int cols, int col_blocks) {
    constexpr int JP = 4 * LPV;
    constexpr int VPP = 256 / LPV;
    constexpr int CPG = 2 * LPV;
    static_assert(CPG % PF == 0, "batch must divide the camera group");
    extern __shared__ __attribute__((aligned(16))) float stage[];  // [F][JP][SP]
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int fb = L / col_blocks;  // frame group within the chunk
    const int XY = X * Y;
    const int c0 = (L - fb * col_blocks) * cols;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const int SP = cols * Z + 1;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const unsigned HW = (unsigned)(H * W);
    const unsigned pb = JP * 4u;
    const unsigned qo = (unsigned)q * 16u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(gq, grid_bytes);
    const int nf = min(F, nb - fb * F);  // frames of this group that exist
    const float *__restrict__ clf = cl + (size_t)fb * F * V * HW * JP;

    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        const int ii = min(i, T - 1);
        float acc[F][4];
#pragma unroll
        for (int f = 0; f < F; ++f)
#pragma unroll
            for (int m = 0; m < 4; ++m) acc[f][m] = 0.f;
        for (int v0 = 0; v0 < V; v0 += CPG) {
            const unsigned goff = (unsigned)(((n0 + ii) * GV + v0 + 2 * q) * 8);
            const auto graw = __builtin_amdgcn_raw_buffer_load_b128(grs, goff, 0, 0);
            float4 gg = make_float4(__builtin_bit_cast(float, (unsigned)graw[0]), __builtin_bit_cast(float, (unsigned)graw[1]),
                                    __builtin_bit_cast(float, (unsigned)graw[2]), __builtin_bit_cast(float, (unsigned)graw[3]));
            if (!valid) gg = make_float4(-2.f, -2.f, -2.f, -2.f);
            const Tap t0 = make_tap(gg.x, gg.y, sxs, sys, W, H, pb);
            const Tap t1 = make_tap(gg.z, gg.w, sxs, sys, W, H, pb);
            static_for(std::make_integer_sequence<int, CPG / PF>{}, [&](auto bc) {
                constexpr int kb = decltype(bc)::value * PF;
                if (v0 + kb >= V) return;
                unsigned o[PF][4];
                float w[PF][4];
                bool any = false;
                static_for(std::make_integer_sequence<int, PF>{}, [&](auto pc) {
                    constexpr int k = kb + decltype(pc)::value;
                    const Tap &src = (k & 1) ? t1 : t0;
                    const bool live = v0 + k < V;
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        o[pc][m] = live ? bcast<LPV, (k >> 1)>(src.o[m]) : kOOB;
                        w[pc][m] = __builtin_bit_cast(float, bcast<LPV, (k >> 1)>(__builtin_bit_cast(unsigned, src.w[m])));
                    }
                    any |= ((o[pc][0] & o[pc][1] & o[pc][2] & o[pc][3]) & kOOB) == 0u;
                });
                if (!__builtin_amdgcn_ballot_w64(any)) return;
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    if (f >= nf) break;
                    typedef unsigned u4 __attribute__((ext_vector_type(4)));
                    u4 t[PF][4];
                    static_for(std::make_integer_sequence<int, PF>{}, [&](auto pc) {
                        constexpr int k = kb + decltype(pc)::value;
                        const int v = min(v0 + k, V - 1);
                        const __amdgpu_buffer_rsrc_t rs =
                            uniform_rsrc(clf + ((size_t)f * V + v) * HW * JP, HW * pb);
#pragma unroll
                        for (int m = 0; m < 4; ++m)
                            t[pc][m] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[pc][m] + qo, 0, 0);
                    });
                    static_for(std::make_integer_sequence<int, PF>{}, [&](auto pc) {
                        constexpr int k = kb + decltype(pc)::value;
                        if (v0 + k >= V) return;
#pragma unroll
                        for (int m = 0; m < 4; ++m) {
                            const float fa = __builtin_bit_cast(float, (unsigned)t[pc][0][m]);
                            const float fb_ = __builtin_bit_cast(float, (unsigned)t[pc][1][m]);
                            const float fc = __builtin_bit_cast(float, (unsigned)t[pc][2][m]);
                            const float fd = __builtin_bit_cast(float, (unsigned)t[pc][3][m]);
                            acc[f][m] = acc[f][m] + __builtin_fmaf(fd, w[pc][3],
                                                                   __builtin_fmaf(fc, w[pc][2],
                                                                                  __builtin_fmaf(fb_, w[pc][1], fa * w[pc][0])));
                        }
                    });
                }
            });
        }
        if (valid) {
#pragma unroll
            for (int f = 0; f < F; ++f)
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    stage[((size_t)f * JP + 4 * q + m) * SP + i] = clampf(acc[f][m] / fV, 0.0f, 1.0f);
        }
    }
    __syncthreads();
    for (int f = 0; f < nf; ++f) {
        const int b = frame0 + fb * F + f;
        const float *st = stage + (size_t)f * JP * SP;
        if (cube) {
            for (int j = 0; j < J; ++j) {
                float *__restrict__ dst = cube + ((size_t)b * J + j) * N + n0;
                for (int e = threadIdx.x; e < T; e += 256) dst[e] = st[j * SP + e];
            }
        }
        if (xy) {
            for (int e = threadIdx.x; e < J * ncols; e += 256) {
                const int j = e / ncols, cc = e - (e / ncols) * ncols;
                const float *s = st + j * SP + cc * Z;
                float m = -INFINITY;
                for (int z = 0; z < Z; ++z) m = nanmax(m, s[z]);
                xy[((size_t)b * J + j) * XY + c0 + cc] = m;
            }
        }
    }
}

// ---- fp16 pair table (C5: fp16 heatmaps) -------------------------------------
// Entry (y, e) of camera v holds, for x0 = e-1, the pixels x0 and x0+1 of row y:
// lane q's 16 B = [x0: joints 4q..4q+3 | x0+1: joints 4q..4q+3] as fp16
// (zeros outside the image).  A voxel-camera then needs 2 aligned 64-B quad
// loads (rows y0, y1) instead of 4, and fp16 -> fp32 is exact.
__global__ __launch_bounds__(256) void layout_pair_h(const _Float16 *__restrict__ hm, uint4 *__restrict__ tab, int J,
                                                     int H, int W, long long total) {
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;  // total = nbV * H * (W+1) * 4
    const int q = (int)(gid & 3);
    const long long ent = gid >> 2;
    const int W1 = W + 1;
    const long long row = ent / W1;
    const int e = (int)(ent - row * W1);
    const long long bv = row / H;
    const int y = (int)(row - bv * H);
    const _Float16 *__restrict__ src = hm + (size_t)bv * J * H * W + (size_t)y * W;
    const size_t HW = (size_t)H * W;
    unsigned short h[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = 4 * q + k;
        const int x0 = e - 1, x1 = e;
        const _Float16 z = (_Float16)0.0f;
        const _Float16 a = (j < J && x0 >= 0) ? src[j * HW + x0] : z;
        const _Float16 b = (j < J && x1 < W) ? src[j * HW + x1] : z;
        h[k] = __builtin_bit_cast(unsigned short, a);
        h[4 + k] = __builtin_bit_cast(unsigned short, b);
    }
    uint4 o;
    o.x = h[0] | ((unsigned)h[1] << 16);
    o.y = h[2] | ((unsigned)h[3] << 16);
    o.z = h[4] | ((unsigned)h[5] << 16);
    o.w = h[6] | ((unsigned)h[7] << 16);
    tab[gid] = o;
}

__device__ __forceinline__ float h_lo(unsigned u) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(u & 0xffffu)); }
__device__ __forceinline__ float h_hi(unsigned u) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(u >> 16)); }

// product-style per-camera loop (grid [V][N][2], one broadcast load per camera)
__global__ __launch_bounds__(256) void gather_h(const uint4 *__restrict__ tab, const float2 *__restrict__ grids,
                                                int frame0, float *__restrict__ cube, float *__restrict__ xy, int V,
                                                int J, int H, int W, int X, int Y, int Z, int cols, int col_blocks) {
    constexpr int LPV = 4, JP = 16, VPP = 64;
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int bl = L / col_blocks;
    const int b = frame0 + bl;
    const int XY = X * Y;
    const int c0 = (L - bl * col_blocks) * cols;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const int SP = cols * Z + 1;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const int W1 = W + 1;
    const unsigned ents = (unsigned)(H * W1);
    const unsigned eb = 64u;  // bytes per entry
    const unsigned qo = (unsigned)q * 16u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    const float2 *__restrict__ g = grids + n0;

    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int v = 0; v < V; ++v) {
            float2 gg = g[(size_t)v * N + min(i, T - 1)];
            if (!valid) gg = make_float2(-2.f, -2.f);
            const float ix = (gg.x + 1.0f) * sxs;
            const float iy = (gg.y + 1.0f) * sys;
            const bool nan_ = (ix != ix) || (iy != iy);
            const float x0f = floorf(ix), y0f = floorf(iy);
            const float wx = ix - x0f, ex = 1.0f - wx;
            const float ny = iy - y0f, syw = 1.0f - ny;
            const float nw = syw * ex, ne = syw * wx, sw = ny * ex, se = ny * wx;
            const int x0 = nan_ ? 0 : (int)fminf(fmaxf(x0f, -4.0f), (float)W + 4.0f);
            const int y0 = nan_ ? 0 : (int)fminf(fmaxf(y0f, -4.0f), (float)H + 4.0f);
            const bool vx = (x0 >= -1) & (x0 < W);
            const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
            const bool any = vx & (vy0 | vy1);
            if (!__builtin_amdgcn_ballot_w64(any)) continue;
            const __amdgpu_buffer_rsrc_t rs =
                uniform_rsrc(tab + ((size_t)bl * V + v) * ents * 4, ents * eb);
            const unsigned e0 = (unsigned)(y0 * W1 + x0 + 1) * eb + qo;
            const auto r0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (vx & vy0) ? e0 : kOOB, 0, 0);
            const auto r1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (vx & vy1) ? e0 + (unsigned)W1 * eb : kOOB, 0, 0);
            // r0 = [a j0 j1 | a j2 j3 | b j0 j1 | b j2 j3], r1 likewise for c, d
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const unsigned ua = (unsigned)r0[m >> 1], ub = (unsigned)r0[2 + (m >> 1)];
                const unsigned uc = (unsigned)r1[m >> 1], ud = (unsigned)r1[2 + (m >> 1)];
                const float fa = (m & 1) ? h_hi(ua) : h_lo(ua);
                const float fb = (m & 1) ? h_hi(ub) : h_lo(ub);
                const float fc = (m & 1) ? h_hi(uc) : h_lo(uc);
                const float fd = (m & 1) ? h_hi(ud) : h_lo(ud);
                acc[m] = acc[m] + __builtin_fmaf(fd, se, __builtin_fmaf(fc, sw, __builtin_fmaf(fb, ne, fa * nw)));
            }
        }
        if (valid) {
#pragma unroll
            for (int m = 0; m < 4; ++m) stage[(4 * q + m) * SP + i] = clampf(acc[m] / fV, 0.0f, 1.0f);
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

// fp16 pair table + quad-shared grid ([N][GV][2], GV even >= V)
__global__ __launch_bounds__(256) void gather_hq(const uint4 *__restrict__ tab, const float *__restrict__ gq, int GV,
                                                 unsigned grid_bytes, int frame0, float *__restrict__ cube,
                                                 float *__restrict__ xy, int V, int J, int H, int W, int X, int Y,
                                                 int Z, int cols, int col_blocks) {
    constexpr int LPV = 4, VPP = 64, CPG = 8;
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int bl = L / col_blocks;
    const int b = frame0 + bl;
    const int XY = X * Y;
    const int c0 = (L - bl * col_blocks) * cols;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const int SP = cols * Z + 1;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const int W1 = W + 1;
    const unsigned ents = (unsigned)(H * W1);
    const unsigned eb = 64u;
    const unsigned qo = (unsigned)q * 16u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(gq, grid_bytes);
    const uint4 *__restrict__ tabf = tab + (size_t)bl * V * ents * 4;

    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        const int ii = min(i, T - 1);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int v0 = 0; v0 < V; v0 += CPG) {
            const unsigned goff = (unsigned)(((n0 + ii) * GV + v0 + 2 * q) * 8);
            const auto graw = __builtin_amdgcn_raw_buffer_load_b128(grs, goff, 0, 0);
            float4 gg = make_float4(__builtin_bit_cast(float, (unsigned)graw[0]), __builtin_bit_cast(float, (unsigned)graw[1]),
                                    __builtin_bit_cast(float, (unsigned)graw[2]), __builtin_bit_cast(float, (unsigned)graw[3]));
            if (!valid) gg = make_float4(-2.f, -2.f, -2.f, -2.f);
            unsigned eo[2][2];
            float wt[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float ix = ((h ? gg.z : gg.x) + 1.0f) * sxs;
                const float iy = ((h ? gg.w : gg.y) + 1.0f) * sys;
                const bool nan_ = (ix != ix) || (iy != iy);
                const float x0f = floorf(ix), y0f = floorf(iy);
                const float wx = ix - x0f, ex = 1.0f - wx;
                const float ny = iy - y0f, syw = 1.0f - ny;
                wt[h][0] = syw * ex;
                wt[h][1] = syw * wx;
                wt[h][2] = ny * ex;
                wt[h][3] = ny * wx;
                const int x0 = nan_ ? 0 : (int)fminf(fmaxf(x0f, -4.0f), (float)W + 4.0f);
                const int y0 = nan_ ? 0 : (int)fminf(fmaxf(y0f, -4.0f), (float)H + 4.0f);
                const bool vx = (x0 >= -1) & (x0 < W);
                const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
                const unsigned e0 = (unsigned)(y0 * W1 + x0 + 1) * eb;
                eo[h][0] = (vx & vy0) ? e0 : kOOB;
                eo[h][1] = (vx & vy1) ? e0 + (unsigned)W1 * eb : kOOB;
            }
            static_for(std::make_integer_sequence<int, CPG>{}, [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                const int v = v0 + k;
                if (v >= V) return;
                const unsigned o0 = bcast<LPV, (k >> 1)>(eo[k & 1][0]);
                const unsigned o1 = bcast<LPV, (k >> 1)>(eo[k & 1][1]);
                const bool any = ((o0 & o1) & kOOB) == 0u;
                if (!__builtin_amdgcn_ballot_w64(any)) return;
                float w[4];
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    w[m] = __builtin_bit_cast(float, bcast<LPV, (k >> 1)>(__builtin_bit_cast(unsigned, wt[k & 1][m])));
                const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(tabf + (size_t)v * ents * 4, ents * eb);
                const auto r0 = __builtin_amdgcn_raw_buffer_load_b128(rs, o0 + qo, 0, 0);
                const auto r1 = __builtin_amdgcn_raw_buffer_load_b128(rs, o1 + qo, 0, 0);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const unsigned ua = (unsigned)r0[m >> 1], ub = (unsigned)r0[2 + (m >> 1)];
                    const unsigned uc = (unsigned)r1[m >> 1], ud = (unsigned)r1[2 + (m >> 1)];
                    const float fa = (m & 1) ? h_hi(ua) : h_lo(ua);
                    const float fb = (m & 1) ? h_hi(ub) : h_lo(ub);
                    const float fc = (m & 1) ? h_hi(uc) : h_lo(uc);
                    const float fd = (m & 1) ? h_hi(ud) : h_lo(ud);
                    acc[m] = acc[m] + __builtin_fmaf(fd, w[3], __builtin_fmaf(fc, w[2], __builtin_fmaf(fb, w[1], fa * w[0])));
                }
            });
        }
        if (valid) {
#pragma unroll
            for (int m = 0; m < 4; ++m) stage[(4 * q + m) * SP + i] = clampf(acc[m] / fV, 0.0f, 1.0f);
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

// On-the-fly projection: no grid read.  Lane q of a voxel group projects the
// voxel centre into cameras v0+2q, v0+2q+1 (camera records staged in LDS) with
// the exact fp32 sequence of project_grid_kernel, then the product's tap code.
template <int LPV, bool PAIR>
__global__ __launch_bounds__(256) void gather_otf(const void *__restrict__ tab, const float *__restrict__ cams,
                                                  const float *__restrict__ resize_t, fvp_grid_spec gs,
                                                  fvp_image_spec im, int frame0, float *__restrict__ cube,
                                                  float *__restrict__ xy, int V, int J, int H, int W, int X, int Y,
                                                  int Z, int cols, int col_blocks) {
    constexpr int JP = 4 * LPV;
    constexpr int VPP = 256 / LPV;
    constexpr int CPG = 2 * LPV;
    extern __shared__ __attribute__((aligned(16))) float stage[];  // [JP][SP] then cams [GV][24], rt[6]
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int bl = L / col_blocks;
    const int b = frame0 + bl;
    const int XY = X * Y;
    const int c0 = (L - bl * col_blocks) * cols;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const int SP = cols * Z + 1;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const int GV = V + (V & 1);
    const unsigned qo = (unsigned)q * 16u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    float *lcam = stage + JP * SP + 3;  // 16-B aligned enough for float reads
    for (int e = threadIdx.x; e < GV * FVP_CAM_STRIDE; e += 256)
        lcam[e] = e < V * FVP_CAM_STRIDE ? cams[e] : 0.0f;
    float rt[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) rt[k] = resize_t[k];
    __syncthreads();
    const unsigned unit = PAIR ? 64u : JP * 4u;
    const unsigned img = PAIR ? (unsigned)(H * (W + 1)) * 64u : (unsigned)(H * W) * unit;
    const char *__restrict__ frame_tab = (const char *)tab + (size_t)bl * V * img;

    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        const int ii = min(i, T - 1);
        const long long n = n0 + ii;
        const int iz = (int)(n % Z);
        const long long r = n / Z;
        const int iy = (int)(r % Y), ix = (int)(r / Y);
        const float wx_ = axis_coord(gs.start[0], gs.end[0], gs.bins[0], ix, gs.center[0]);
        const float wy_ = axis_coord(gs.start[1], gs.end[1], gs.bins[1], iy, gs.center[1]);
        const float wz_ = axis_coord(gs.start[2], gs.end[2], gs.bins[2], iz, gs.center[2]);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int v0 = 0; v0 < V; v0 += CPG) {
            float g[4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int vc = min(v0 + 2 * q + h, GV - 1);
                const Cam c = load_cam(lcam + vc * FVP_CAM_STRIDE);
                float px, py;
                project_point(c, wx_, wy_, wz_, px, py);
                pixel_to_sample(px, py, rt, im.ori_max, im.img_w, im.img_h, (float)im.hm_w, (float)im.hm_h, g[2 * h],
                                g[2 * h + 1]);
            }
            if (!valid) g[0] = g[1] = g[2] = g[3] = -2.0f;
            const Taps4<PAIR> t0 = setup_taps<PAIR>(g[0], g[1], sxs, sys, W, H, unit);
            const Taps4<PAIR> t1 = setup_taps<PAIR>(g[2], g[3], sxs, sys, W, H, unit);
            static_for(std::make_integer_sequence<int, CPG>{}, [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = k >> 1;
                const int v = v0 + k;
                if (v >= V) return;
                const Taps4<PAIR> &src = (k & 1) ? t1 : t0;
                unsigned o[Taps4<PAIR>::NO];
                unsigned all = kOOB;
#pragma unroll
                for (int m = 0; m < Taps4<PAIR>::NO; ++m) {
                    o[m] = group_bcast<LPV, S>(src.o[m]);
                    all &= o[m];
                }
                if (!__builtin_amdgcn_ballot_w64((all & kOOB) == 0u)) return;
                float w[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) w[m] = group_bcast<LPV, S>(src.w[m]);
                const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(frame_tab + (size_t)v * img, img);
                if constexpr (PAIR) {
                    const u32x4 r0 = __builtin_amdgcn_raw_buffer_load_b128(rs, o[0] + qo, 0, 0);
                    const u32x4 r1 = __builtin_amdgcn_raw_buffer_load_b128(rs, o[1] + qo, 0, 0);
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const unsigned ua = r0[m >> 1], ub = r0[2 + (m >> 1)];
                        const unsigned uc = r1[m >> 1], ud = r1[2 + (m >> 1)];
                        const float fa = (m & 1) ? h_hi(ua) : h_lo(ua);
                        const float fb = (m & 1) ? h_hi(ub) : h_lo(ub);
                        const float fc = (m & 1) ? h_hi(uc) : h_lo(uc);
                        const float fd = (m & 1) ? h_hi(ud) : h_lo(ud);
                        acc[m] = acc[m] +
                                 __builtin_fmaf(fd, w[3], __builtin_fmaf(fc, w[2], __builtin_fmaf(fb, w[1], fa * w[0])));
                    }
                } else {
                    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, o[0] + qo, 0, 0);
                    const u32x4 bq = __builtin_amdgcn_raw_buffer_load_b128(rs, o[1] + qo, 0, 0);
                    const u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(rs, o[2] + qo, 0, 0);
                    const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(rs, o[3] + qo, 0, 0);
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const float fa = __builtin_bit_cast(float, (unsigned)a[m]);
                        const float fb = __builtin_bit_cast(float, (unsigned)bq[m]);
                        const float fc = __builtin_bit_cast(float, (unsigned)c[m]);
                        const float fd = __builtin_bit_cast(float, (unsigned)d[m]);
                        acc[m] = acc[m] +
                                 __builtin_fmaf(fd, w[3], __builtin_fmaf(fc, w[2], __builtin_fmaf(fb, w[1], fa * w[0])));
                    }
                }
            });
        }
        if (valid) {
#pragma unroll
            for (int m = 0; m < 4; ++m) stage[(4 * q + m) * SP + i] = clampf(acc[m] / fV, 0.0f, 1.0f);
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

// Camera-outer C5 variant: fp16 pair table, on-the-fly coordinates; each block
// keeps the accumulators of its NP passes (NP*64 voxels) in registers and walks
// camera groups outermost, so concurrently resident blocks sweep the cameras
// roughly in lockstep (L2 working set = a few cameras' footprints).
template <int NP>
__global__ __launch_bounds__(256) void gather_co(const void *__restrict__ tab, CoordSource src_, int frame0,
                                                 float *__restrict__ cube, float *__restrict__ xy, int V, int J, int H,
                                                 int W, int X, int Y, int Z, int cols, int col_blocks, int SP) {
    constexpr int LPV = 4, JP = 16, VPP = 64, CPG = 8;
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int bl = L / col_blocks;
    const int b = frame0 + bl;
    const int XY = X * Y;
    const int c0 = (L - bl * col_blocks) * cols;
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const int GV = V + (V & 1);
    const unsigned qo = (unsigned)q * 16u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    float *lcam = stage + ((JP * SP + 3) & ~3);
    for (int e = threadIdx.x; e < GV * FVP_CAM_STRIDE; e += 256) lcam[e] = e < V * FVP_CAM_STRIDE ? src_.cams[e] : 0.0f;
    float rt[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) rt[k] = src_.resize_t[k];
    __syncthreads();
    const unsigned img = (unsigned)(H * (W + 1)) * 64u;
    const char *__restrict__ frame_tab = (const char *)tab + (size_t)bl * V * img;
    float acc[NP][4];
    float wc[NP][3];
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[pp][m] = 0.f;
        const int i = pp * VPP + threadIdx.x / LPV;
        const long long n = n0 + min(i, T - 1);
        const int iz = (int)(n % Z);
        const long long r = n / Z;
        wc[pp][0] = axis_coord(src_.gs.start[0], src_.gs.end[0], X, (int)(r / Y), src_.gs.center[0]);
        wc[pp][1] = axis_coord(src_.gs.start[1], src_.gs.end[1], Y, (int)(r % Y), src_.gs.center[1]);
        wc[pp][2] = axis_coord(src_.gs.start[2], src_.gs.end[2], Z, iz, src_.gs.center[2]);
    }
    for (int v0 = 0; v0 < V; v0 += CPG) {
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) {
            const int i = pp * VPP + threadIdx.x / LPV;
            const bool valid = i < T;
            float g[4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const Cam c = load_cam(lcam + min(v0 + 2 * q + h, GV - 1) * FVP_CAM_STRIDE);
                float px, py;
                project_point(c, wc[pp][0], wc[pp][1], wc[pp][2], px, py);
                pixel_to_sample(px, py, rt, src_.im.ori_max, src_.im.img_w, src_.im.img_h, (float)src_.im.hm_w,
                                (float)src_.im.hm_h, g[2 * h], g[2 * h + 1]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) g[k] = valid ? g[k] : -2.0f;
            const Taps4<true> t0 = setup_taps<true>(g[0], g[1], sxs, sys, W, H, 64u);
            const Taps4<true> t1 = setup_taps<true>(g[2], g[3], sxs, sys, W, H, 64u);
            static_for(std::make_integer_sequence<int, CPG>{}, [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = k >> 1;
                const int v = v0 + k;
                if (v >= V) return;
                const Taps4<true> &src = (k & 1) ? t1 : t0;
                const unsigned o0 = group_bcast<LPV, S>(src.o[0]);
                const unsigned o1 = group_bcast<LPV, S>(src.o[1]);
                if (!__builtin_amdgcn_ballot_w64(((o0 & o1) & kOOB) == 0u)) return;
                float w[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) w[m] = group_bcast<LPV, S>(src.w[m]);
                const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(frame_tab + (size_t)v * img, img);
                const u32x4 r0 = __builtin_amdgcn_raw_buffer_load_b128(rs, o0 + qo, 0, 0);
                const u32x4 r1 = __builtin_amdgcn_raw_buffer_load_b128(rs, o1 + qo, 0, 0);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const unsigned ua = r0[m >> 1], ub = r0[2 + (m >> 1)];
                    const unsigned uc = r1[m >> 1], ud = r1[2 + (m >> 1)];
                    const float fa = (m & 1) ? h_hi(ua) : h_lo(ua);
                    const float fb = (m & 1) ? h_hi(ub) : h_lo(ub);
                    const float fc = (m & 1) ? h_hi(uc) : h_lo(uc);
                    const float fd = (m & 1) ? h_hi(ud) : h_lo(ud);
                    acc[pp][m] = acc[pp][m] +
                                 __builtin_fmaf(fd, w[3], __builtin_fmaf(fc, w[2], __builtin_fmaf(fb, w[1], fa * w[0])));
                }
            });
        }
    }
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
        const int i = pp * VPP + threadIdx.x / LPV;
        if (i < T) {
#pragma unroll
            for (int m = 0; m < 4; ++m) stage[(4 * q + m) * SP + i] = clampf(acc[pp][m] / fV, 0.0f, 1.0f);
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
            const float *sp = stage + j * SP + cc * Z;
            float m = -INFINITY;
            for (int z = 0; z < Z; ++z) m = nanmax(m, sp[z]);
            xy[((size_t)b * J + j) * XY + c0 + cc] = m;
        }
    }
}

// [V][N][2] -> [N][GV][2], padded cameras (-2,-2) (off-image)
__global__ void regrid_kernel(const float2 *__restrict__ g, float2 *__restrict__ out, int V, int GV, long long N) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= N * GV) return;
    const long long n = t / GV;
    const int v = (int)(t - n * GV);
    out[t] = v < V ? g[(size_t)v * N + n] : make_float2(-2.f, -2.f);
}

}  // namespace next
}  // namespace fvp

using namespace fvp;

extern "C" int voxnext_regrid(const float *g, float *out, int V, int GV, long long N, void *stream) {
    const long long tot = N * GV;
    hipLaunchKernelGGL(next::regrid_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float2 *)g, (float2 *)out, V, GV, N);
    return (int)hipGetLastError();
}

// Full op: per chunk of `chunk` frames, layout then the qg gather.
template <int MODE, int PF>
static void launch_qg(dim3 grid, size_t lds, hipStream_t s, const float *ws, const float *gq, int GV, int f0,
                      float *cube, float *xy, int V, int J, int H, int W, int X, int Y, int Z, int cols,
                      int col_blocks) {
    hipLaunchKernelGGL((next::gather_qg<4, MODE, PF>), grid, dim3(256), lds, s, ws, (const float4 *)gq, GV, nullptr,
                       f0, cube, xy, V, J, H, W, X, Y, Z, cols, col_blocks);
}

// Full op: per chunk of `chunk` frames, layout then the qg gather.
extern "C" int voxnext_qg(const void *hm, int half, int B, int V, int J, int H, int W, const float *gq, int GV, int X,
                          int Y, int Z, float *cube, float *xy, float *ws, int chunk, int cols, int mode, int pf,
                          void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int LPV = lanes_per_voxel(J);
    if (LPV != 4) return -1;
    const int col_blocks = (X * Y + cols - 1) / cols;
    const size_t lds = (size_t)4 * LPV * (cols * Z + 1) * sizeof(float);
    const size_t frame_elems = (size_t)V * J * H * W;
    for (int f0 = 0; f0 < B; f0 += chunk) {
        const int nb = min(chunk, B - f0);
        if (half)
            launch_layout<4, _Float16>((const _Float16 *)hm + (size_t)f0 * frame_elems, nb, V, J, H, W, ws, s);
        else
            launch_layout<4, float>((const float *)hm + (size_t)f0 * frame_elems, nb, V, J, H, W, ws, s);
        const dim3 grid((unsigned)(nb * col_blocks));
#define QG(M, P) launch_qg<M, P>(grid, lds, s, ws, gq, GV, f0, cube, xy, V, J, H, W, X, Y, Z, cols, col_blocks)
        const int key = mode * 10 + pf;
        switch (key) {
            case 1: QG(0, 1); break;
            case 2: QG(0, 2); break;
            case 4: QG(0, 4); break;
            case 8: QG(0, 8); break;
            case 11: QG(1, 1); break;
            case 12: QG(1, 2); break;
            case 21: QG(2, 1); break;
            case 22: QG(2, 2); break;
            case 31: QG(3, 1); break;
            case 41: QG(4, 1); break;
            case 42: QG(4, 2); break;
            case 51: QG(5, 1); break;
            default: return -2;
        }
#undef QG
    }
    return (int)hipGetLastError();
}

// Split entry points for stream-overlap experiments.
extern "C" int voxnext_layout(const void *hm, int half, int nb, int V, int J, int H, int W, float *ws, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (half)
        launch_layout<4, _Float16>((const _Float16 *)hm, nb, V, J, H, W, ws, s);
    else
        launch_layout<4, float>((const float *)hm, nb, V, J, H, W, ws, s);
    return (int)hipGetLastError();
}

template <int PF, int F>
static void launch_mf(int nb, size_t lds0, hipStream_t s, const float *ws, const float *gq, int GV, unsigned gbytes,
                      int f0, float *cube, float *xy, int V, int J, int H, int W, int X, int Y, int Z, int cols,
                      int col_blocks) {
    const dim3 grid((unsigned)(((nb + F - 1) / F) * col_blocks));
    hipLaunchKernelGGL((next::gather_mf<4, PF, F>), grid, dim3(256), lds0 * F, s, ws, gq, GV, gbytes, nb, f0, cube, xy,
                       V, J, H, W, X, Y, Z, cols, col_blocks);
}

extern "C" int voxnext_mf(const void *hm, int half, int B, int V, int J, int H, int W, const float *gq, int GV, int X,
                          int Y, int Z, float *cube, float *xy, float *ws, int chunk, int cols, int F, int pf,
                          void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (lanes_per_voxel(J) != 4) return -1;
    const int col_blocks = (X * Y + cols - 1) / cols;
    const size_t lds0 = (size_t)16 * (cols * Z + 1) * sizeof(float);
    const size_t frame_elems = (size_t)V * J * H * W;
    const unsigned gbytes = (unsigned)((size_t)X * Y * Z * GV * 8);
    for (int f0 = 0; f0 < B; f0 += chunk) {
        const int nb = min(chunk, B - f0);
        if (half)
            launch_layout<4, _Float16>((const _Float16 *)hm + (size_t)f0 * frame_elems, nb, V, J, H, W, ws, s);
        else
            launch_layout<4, float>((const float *)hm + (size_t)f0 * frame_elems, nb, V, J, H, W, ws, s);
#define MF(P, FF) launch_mf<P, FF>(nb, lds0, s, ws, gq, GV, gbytes, f0, cube, xy, V, J, H, W, X, Y, Z, cols, col_blocks)
        switch (F * 10 + pf) {
            case 11: MF(1, 1); break;
            case 12: MF(2, 1); break;
            case 21: MF(1, 2); break;
            case 22: MF(2, 2); break;
            case 41: MF(1, 4); break;
            default: return -2;
        }
#undef MF
    }
    return (int)hipGetLastError();
}

// fp16 pair-table op: per chunk, layout_pair_h then gather_h.  ws must hold
// chunk * V * H * (W+1) * 64 bytes.
extern "C" int voxnext_h(const void *hm, int B, int V, int J, int H, int W, const float *grids, int X, int Y, int Z,
                         float *cube, float *xy, void *ws, int chunk, int cols, const float *gq, int GV, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (J > 16) return -1;
    const int col_blocks = (X * Y + cols - 1) / cols;
    const size_t lds = (size_t)16 * (cols * Z + 1) * sizeof(float);
    const size_t frame_elems = (size_t)V * J * H * W;
    for (int f0 = 0; f0 < B; f0 += chunk) {
        const int nb = min(chunk, B - f0);
        const long long total = (long long)nb * V * H * (W + 1) * 4;
        hipLaunchKernelGGL(next::layout_pair_h, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                           (const _Float16 *)hm + (size_t)f0 * frame_elems, (uint4 *)ws, J, H, W, total);
        if (gq)
            hipLaunchKernelGGL(next::gather_hq, dim3((unsigned)(nb * col_blocks)), dim3(256), lds, s,
                               (const uint4 *)ws, gq, GV, (unsigned)((size_t)X * Y * Z * GV * 8), f0, cube, xy, V, J,
                               H, W, X, Y, Z, cols, col_blocks);
        else
            hipLaunchKernelGGL(next::gather_h, dim3((unsigned)(nb * col_blocks)), dim3(256), lds, s, (const uint4 *)ws,
                               (const float2 *)grids, f0, cube, xy, V, J, H, W, X, Y, Z, cols, col_blocks);
    }
    return (int)hipGetLastError();
}

// On-the-fly op (fp32 CL or fp16 pairs per input dtype), per chunk.
extern "C" int voxnext_otf(const void *hm, int half, int B, int V, int J, int H, int W, const float *cams,
                           const float *rt, const fvp_grid_spec *gs, const fvp_image_spec *im, float *cube, float *xy,
                           void *ws, int chunk, int cols, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (J > 16 || J < 9) return -1;
    const int X = gs->bins[0], Y = gs->bins[1], Z = gs->bins[2];
    const int col_blocks = (X * Y + cols - 1) / cols;
    const size_t lds = ((size_t)16 * (cols * Z + 1) + 3 + (size_t)(V + 1) * FVP_CAM_STRIDE) * sizeof(float);
    const size_t frame_elems = (size_t)V * J * H * W;
    for (int f0 = 0; f0 < B; f0 += chunk) {
        const int nb = min(chunk, B - f0);
        const dim3 grid((unsigned)(nb * col_blocks));
        if (half) {
            const long long total = (long long)nb * V * H * (W + 1) * 4;
            hipLaunchKernelGGL(heatmaps_to_pairs_kernel<_Float16>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                               s, (const _Float16 *)hm + (size_t)f0 * frame_elems, (uint4 *)ws, J, H, W, total);
            hipLaunchKernelGGL((next::gather_otf<4, true>), grid, dim3(256), lds, s, ws, cams, rt, *gs, *im, f0, cube,
                               xy, V, J, H, W, X, Y, Z, cols, col_blocks);
        } else {
            launch_layout<4, float>((const float *)hm + (size_t)f0 * frame_elems, nb, V, J, H, W, (float *)ws, s);
            hipLaunchKernelGGL((next::gather_otf<4, false>), grid, dim3(256), lds, s, ws, cams, rt, *gs, *im, f0,
                               cube, xy, V, J, H, W, X, Y, Z, cols, col_blocks);
        }
    }
    return (int)hipGetLastError();
}

// Product kernel with a chosen dynamic-LDS size (occupancy limiter), chunk and cols.
extern "C" int voxnext_occ(const float *hm, int B, int V, int J, int H, int W, const float *packed, int X, int Y, int Z,
                           float *cube, float *xy, void *ws, int chunk, int cols, int lds_bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (lanes_per_voxel(J) != 4) return -1;
    const int col_blocks = (X * Y + cols - 1) / cols;
    const int SP = lds_bytes < 0 ? cols * Z : cols * Z + 1;
    size_t lds = (size_t)16 * SP * sizeof(float);
    if (lds_bytes > 0 && (size_t)lds_bytes > lds) lds = lds_bytes;
    CoordSource src{};
    src.grids = packed;
    const size_t frame_elems = (size_t)V * J * H * W;
    for (int f0 = 0; f0 < B; f0 += chunk) {
        const int nb = min(chunk, B - f0);
        launch_layout<4, float>(hm + (size_t)f0 * frame_elems, nb, V, J, H, W, (float *)ws, s);
        hipLaunchKernelGGL((voxelize_kernel<4, false, false>), dim3((unsigned)(nb * col_blocks)), dim3(256), lds, s,
                           ws, src, nullptr, f0, cube, xy, V, J, H, W, X, Y, Z, cols, col_blocks, SP);
    }
    return (int)hipGetLastError();
}

// camera-outer C5 op (fp16 pairs + on-the-fly), NP = cols*Z/64 passes
extern "C" int voxnext_co(const void *hm, int B, int V, int J, int H, int W, const float *cams, const float *rt,
                          const fvp_grid_spec *gs, const fvp_image_spec *im, float *cube, float *xy, void *ws,
                          int chunk, int cols, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (J > 16 || J < 9) return -1;
    const int X = gs->bins[0], Y = gs->bins[1], Z = gs->bins[2];
    const int T = cols * Z;
    if (T % 64) return -3;
    const int NP = T / 64;
    const int col_blocks = (X * Y + cols - 1) / cols;
    const int SP = T + 1;
    const size_t lds = (((size_t)16 * SP + 3) & ~(size_t)3) * 4 + (size_t)(V + 1) * FVP_CAM_STRIDE * 4;
    CoordSource src{};
    src.cams = cams;
    src.resize_t = rt;
    src.gs = *gs;
    src.im = *im;
    const size_t frame_elems = (size_t)V * J * H * W;
    for (int f0 = 0; f0 < B; f0 += chunk) {
        const int nb = min(chunk, B - f0);
        const long long total = (long long)nb * V * H * (W + 1) * 4;
        hipLaunchKernelGGL(heatmaps_to_pairs_kernel<_Float16>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                           (const _Float16 *)hm + (size_t)f0 * frame_elems, (uint4 *)ws, J, H, W, total);
        const dim3 grid((unsigned)(nb * col_blocks));
#define CO(NPV) hipLaunchKernelGGL((next::gather_co<NPV>), grid, dim3(256), lds, s, ws, src, f0, cube, xy, V, J, H, W, X, Y, Z, cols, col_blocks, SP)
        switch (NP) {
            case 1: CO(1); break;
            case 2: CO(2); break;
            case 3: CO(3); break;
            case 4: CO(4); break;
            case 5: CO(5); break;
            case 8: CO(8); break;
            case 10: CO(10); break;
            default: return -4;
        }
#undef CO
    }
    return (int)hipGetLastError();
}
