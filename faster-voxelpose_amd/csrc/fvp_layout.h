// Channels-last heatmap layout shared by the whole-space and per-person
// gathers (see fvp_voxelize.hip for why): [b][V][H*W][JP] fp32, JP = 4*LPV,
// joints zero padded; out-of-image taps read 0 through a buffer descriptor's
// range check.
#pragma once

#include <utility>

#include "fvp_device.h"

namespace fvp {

constexpr unsigned kOOB = 0x80000000u;  // beyond any descriptor range -> loads return 0

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void *base, unsigned bytes) {
    const unsigned long long p = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
    void *b = (void *)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// The same descriptor as four SGPR words, for the inline-asm LDS-DMA below.
__device__ __forceinline__ u32x4 uniform_rsrc4(const void *base, unsigned bytes) {
    const unsigned long long p = (unsigned long long)base;
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((unsigned)p);
    r.y = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32)) & 0xffffu;  // stride 0
    r.z = __builtin_amdgcn_readfirstlane(bytes);
    r.w = 0x00020000u;
    return r;
}

// One 16-B piece per lane of a global -> LDS copy (buffer_load_dwordx4 ... lds) into the wave's
// 1-KiB run at LDS byte address lds_base (M0; wave-uniform).  Inline asm rather than
// __builtin_amdgcn_raw_ptr_buffer_load_lds: the compiler then does not track the copy as an LDS
// write, so it puts no s_waitcnt vmcnt(0) before the LDS reads of the OTHER stage buffer (with
// the builtin it drained the next stage's copies before every step's reads: a double buffer
// with no overlap).  The caller orders it with counted vmcnt waits and barriers.
__device__ __forceinline__ void lds_dma16(u32x4 rsrc, unsigned lds_base, unsigned voffset) {
    asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voffset), "s"(rsrc), "{m0}"(lds_base) : "memory");
}

// -- layout pass ----------------------------------------------------------------
// thread = (pixel, joint quad q): reads joints 4q..4q+3 of one pixel (the lanes
// of a wave cover 64/LPV consecutive pixels -> coalesced plane reads), writes
// one float4 (a wave writes a contiguous 1 KiB run; NF > 1: runs of JP*4 B,
// the NF frames of a group interleaved per pixel: [b/NF][V][H*W][NF][JP]).
// (J joints of a slice; Jst = the planes per (frame, view) of the source)
template <int LPV, typename T, int NF = 1>
__global__ __launch_bounds__(256) void heatmaps_to_cl_kernel(const T *__restrict__ hm, float4 *__restrict__ cl, int J,
                                                             int Jst, int HW, int V, long long total_px) {
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long pxg = gid / LPV;
    const int q = (int)(gid - pxg * LPV);
    if (pxg >= total_px) return;
    const long long bv = pxg / HW;
    const int pix = (int)(pxg - bv * HW);
    const T *__restrict__ src = hm + (size_t)bv * Jst * HW + pix;
    const int j = 4 * q;
    float4 o;
    o.x = (j + 0 < J) ? to_f32(src[(size_t)(j + 0) * HW]) : 0.f;
    o.y = (j + 1 < J) ? to_f32(src[(size_t)(j + 1) * HW]) : 0.f;
    o.z = (j + 2 < J) ? to_f32(src[(size_t)(j + 2) * HW]) : 0.f;
    o.w = (j + 3 < J) ? to_f32(src[(size_t)(j + 3) * HW]) : 0.f;
    if constexpr (NF == 1) {
        cl[pxg * LPV + q] = o;
    } else {
        const long long fr = bv / V;  // frame within the chunk
        const long long g = fr / NF, f = fr - (fr / NF) * NF, v = bv - fr * V;
        cl[(((g * V + v) * HW + pix) * NF + f) * LPV + q] = o;
    }
}

// -- fp16 pixel-pair table ------------------------------------------------------
// [b][V][H][W+1] entries of 64 B; entry (y, e) holds pixels x0 = e-1 and x0+1
// of row y, lane q's 16 B = [x0: joints 4q..4q+3 | x0+1: joints 4q..4q+3] fp16,
// zeros outside the image (J <= 16).  One thread per (entry, q).
template <typename T, int NF = 1>  // T = _Float16; NF frames per entry: [b/NF][V][H][W+1][NF] x 64 B
__global__ __launch_bounds__(256) void heatmaps_to_pairs_kernel(const T *__restrict__ hm,
                                                                uint4 *__restrict__ tab, int J, int H, int W, int V,
                                                                long long total) {
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int q = (int)(gid & 3);
    const long long ent = gid >> 2;
    const int W1 = W + 1;
    const long long row = ent / W1;
    const int e = (int)(ent - row * W1);
    const long long bv = row / H;
    const int y = (int)(row - bv * H);
    const size_t HW = (size_t)H * W;
    const T *__restrict__ src = hm + (size_t)bv * J * HW + (size_t)y * W;
    unsigned short h[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = 4 * q + k;
        const T z = (T)0.0f;
        const T a = (j < J && e >= 1) ? src[j * HW + e - 1] : z;
        const T b = (j < J && e < W) ? src[j * HW + e] : z;
        h[k] = __builtin_bit_cast(unsigned short, a);
        h[4 + k] = __builtin_bit_cast(unsigned short, b);
    }
    const uint4 val = make_uint4(h[0] | ((unsigned)h[1] << 16), h[2] | ((unsigned)h[3] << 16),
                                 h[4] | ((unsigned)h[5] << 16), h[6] | ((unsigned)h[7] << 16));
    if constexpr (NF == 1) {
        tab[gid] = val;
    } else {
        const long long fr = bv / V, v = bv - fr * V;
        const long long g = fr / NF, f = fr - (fr / NF) * NF;
        tab[(((((g * V + v) * H + y) * W1 + e) * NF) + f) * 4 + q] = val;
    }
}

// The same table, one block per (frame group, view, row): the NF frames' J
// joint rows are read with coalesced 4-B loads (a wave covers 256 B of one
// row) into LDS as [NF][16][W+4] halves (pixel x at x+2, zeros at x = -1, W
// and for joints >= J), then the row's (W+1) x NF entries go out as one
// contiguous run of 16-B stores.  The per-entry kernel above reads 2-B values
// per lane (8 loads per 16-B store) and writes 64-B pieces NF*64 B apart:
// C5, 4 frames per entry, 132 -> 97.5 us per launch (profiles/round3/c5/pairs_layout.txt).
// Needs W even (4-B aligned rows); LDS NF*16*(W/2+2)*4 B.
template <int NF>
__global__ __launch_bounds__(256) void pairs_rows_kernel(const _Float16 *__restrict__ hm, uint4 *__restrict__ tab,
                                                         int J, int H, int W, int V) {
    extern __shared__ unsigned s32[];
    const int P2 = W / 2 + 2;  // words per staged joint row
    const int row = blockIdx.x;  // (g * V + v) * H + y
    const int gv = row / H, y = row - gv * H;
    const int g = gv / V, v = gv - g * V;
    const size_t HW = (size_t)H * W;
    for (int t = threadIdx.x; t < NF * 16 * P2; t += 256) {  // the zero borders and padding joints
        const int jr = t / P2, w = t - jr * P2;
        if ((jr & 15) >= J || w == 0 || w == P2 - 1) s32[t] = 0u;
    }
    // all U loads of a lane issued before their LDS writes (clamped, always
    // legal addresses): a row is one dependent HBM round trip per block
    constexpr int U = 16;
    const int HWc = W / 2, total = NF * J * HWc;
    for (int t0 = threadIdx.x; t0 < total; t0 += 256 * U) {
        unsigned val[U];
        int at[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = min(t0 + u * 256, total - 1);
            const int fj = t / HWc, c = t - fj * HWc;
            const int f = fj / J, j = fj - f * J;
            val[u] = reinterpret_cast<const unsigned *>(hm + (((size_t)(g * NF + f) * V + v) * J + j) * HW +
                                                        (size_t)y * W)[c];
            at[u] = (f * 16 + j) * P2 + 1 + c;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + u * 256 < total) s32[at[u]] = val[u];
    }
    __syncthreads();
    const unsigned short *s16 = reinterpret_cast<const unsigned short *>(s32);
    const int W1 = W + 1;
    uint4 *__restrict__ dst = tab + (size_t)row * W1 * NF * 4;
    for (int t = threadIdx.x; t < W1 * NF * 4; t += 256) {  // t = (e * NF + f) * 4 + q
        const int q = t & 3, ef = t >> 2;
        const int e = ef / NF, f = ef - e * NF;
        const unsigned short *r = s16 + (f * 16 + 4 * q) * (2 * P2) + e + 1;  // pixel e-1, then pixel e
        unsigned h[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            h[k] = r[k * 2 * P2];
            h[4 + k] = r[k * 2 * P2 + 1];
        }
        dst[t] = make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16));
    }
}

// The same table without LDS, 8 entries per thread (W % 8 == 0, 16-B aligned
// rows): thread = (row, 8-pixel group m, frame f, joint quad q) loads pixels
// 8m .. 8m+7 of its 4 joint rows with one 16-B load each (+ pixel 8m-1), and
// writes entries 8m .. 8m+7 (pixels e-1, e) -- and entry W for the last group.
// A wave's 16 (f, q) lanes of one m write 256 contiguous bytes per entry.
template <int NF>
__global__ __launch_bounds__(256) void pairs_vec8_kernel(const _Float16 *__restrict__ hm, uint4 *__restrict__ tab,
                                                         int J, int H, int W, int V, long long total) {
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int M = W / 8;
    const int q = (int)(gid & 3);
    const long long r1 = gid >> 2;
    const int f = (int)(r1 % NF);
    const long long r2 = r1 / NF;
    const int m = (int)(r2 % M);
    const long long row = r2 / M;  // (g * V + v) * H + y
    const long long gv = row / H;
    const int y = (int)(row - gv * H);
    const long long g = gv / V, v = gv - g * V;
    const size_t HW = (size_t)H * W;
    unsigned px[4][4], prev[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = 4 * q + k;
        const unsigned short *src = reinterpret_cast<const unsigned short *>(hm) +
                                    (((size_t)(g * NF + f) * V + v) * J + j) * HW + (size_t)y * W;
        uint4 a = make_uint4(0u, 0u, 0u, 0u);
        unsigned b = 0u;
        if (j < J) {
            a = *reinterpret_cast<const uint4 *>(src + 8 * m);
            b = m > 0 ? src[8 * m - 1] : 0u;
        }
        px[k][0] = a.x; px[k][1] = a.y; px[k][2] = a.z; px[k][3] = a.w;
        prev[k] = b;
    }
    auto pix = [&](int k, int i) -> unsigned { return (px[k][i >> 1] >> (16 * (i & 1))) & 0xffffu; };
    const int W1 = W + 1;
    uint4 *__restrict__ dst = tab + ((size_t)row * W1 * NF + f) * 4 + q;
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // entry e = 8m + i: pixels e - 1 and e
        unsigned lo[4], hi[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            lo[k] = i == 0 ? prev[k] : pix(k, i - 1);
            hi[k] = pix(k, i);
        }
        dst[(size_t)(8 * m + i) * NF * 4] =
            make_uint4(lo[0] | (lo[1] << 16), lo[2] | (lo[3] << 16), hi[0] | (hi[1] << 16), hi[2] | (hi[3] << 16));
    }
    if (m == M - 1) {  // entry W: pixel W - 1 and the zero past the row
        dst[(size_t)W * NF * 4] = make_uint4(pix(0, 7) | (pix(1, 7) << 16), pix(2, 7) | (pix(3, 7) << 16), 0u, 0u);
    }
}

inline size_t pair_frame_bytes(int V, int H, int W) { return (size_t)V * H * (W + 1) * 64; }

// Launch the pair-table layout for nb frames (a multiple of NF).
template <int NF>
inline void launch_pairs(const _Float16 *hm, int nb, int V, int J, int H, int W, uint4 *tab, hipStream_t s) {
    const size_t lds = (size_t)NF * 16 * (W / 2 + 2) * 4;
    // 8 entries a thread wherever rows are 16-B aligned: C5, 4 frames per entry
    // 98.2 -> 72.5 us, one frame 20.4 -> 15.9 us (profiles/round4/pairs8/).
    // Otherwise row blocks for frame groups (a 15 KB row per block leaves its
    // load / store phases exposed at one frame: 40.8 vs 20.8 us per entry), and
    // the per-entry kernel for single frames, odd widths and 2-B-aligned pointers.
    const bool aligned = ((unsigned long long)hm & 3ull) == 0;  // 4-B row loads (a C-ABI caller may pass any fp16 pointer)
    if (W % 8 == 0 && ((unsigned long long)hm & 15ull) == 0) {
        const long long total = (long long)nb / NF * V * H * (W / 8) * NF * 4;
        hipLaunchKernelGGL((pairs_vec8_kernel<NF>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, hm, tab,
                           J, H, W, V, total);
    } else if (NF > 1 && aligned && W % 2 == 0 && lds <= 64 * 1024) {
        hipLaunchKernelGGL((pairs_rows_kernel<NF>), dim3((unsigned)((long long)nb / NF * V * H)), dim3(256), lds, s, hm,
                           tab, J, H, W, V);
    } else {
        const long long total = (long long)nb * V * H * (W + 1) * 4;
        hipLaunchKernelGGL((heatmaps_to_pairs_kernel<_Float16, NF>), dim3((unsigned)((total + 255) / 256)), dim3(256),
                           0, s, hm, tab, J, H, W, V, total);
    }
}

// -- lane-group helpers -----------------------------------------------------------
// Broadcast lane S of each LPV-lane voxel group to the whole group (DPP quad
// permutes for LPV <= 4, ds_swizzle bit mode for 8-lane groups).
template <int LPV, int S>
__device__ __forceinline__ unsigned group_bcast(unsigned x) {
    if constexpr (LPV == 1) {
        return x;
    } else if constexpr (LPV == 2) {
        return (unsigned)__builtin_amdgcn_mov_dpp((int)x, S | (S << 2) | ((2 + S) << 4) | ((2 + S) << 6), 0xf, 0xf,
                                                  false);
    } else if constexpr (LPV == 4) {
        return (unsigned)__builtin_amdgcn_mov_dpp((int)x, S | (S << 2) | (S << 4) | (S << 6), 0xf, 0xf, false);
    } else {
        static_assert(LPV == 8, "voxel groups of 1, 2, 4 or 8 lanes");
        return (unsigned)__builtin_amdgcn_ds_swizzle((int)x, 0x18 | (S << 5));
    }
}

// Unsigned maximum over the lanes of the wave that hold the same group slot
// (lane mod LPV), all in VALU: DPP row rotations by LPV, 2 LPV, .. 8 within each
// 16-lane row, then v_permlane16_swap / v_permlane32_swap (gfx950) across the
// rows.  Every lane ends with its slot's maximum.  (A __shfl_xor chain compiles
// to ds_bpermute, an LDS round trip and an lgkmcnt(0) wait per step.)
template <int LPV>
__device__ __forceinline__ unsigned slot_umax(unsigned m) {
    static_assert(LPV == 1 || LPV == 2 || LPV == 4 || LPV == 8, "voxel groups of 1, 2, 4 or 8 lanes");
    // row_ror:s = DPP control 0x120 + s
    auto ror = [](unsigned v, auto sc) {
        return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x120 + decltype(sc)::value, 0xf, 0xf, false);
    };
    unsigned r;
    if constexpr (LPV <= 1) { r = ror(m, std::integral_constant<int, 1>{}); m = m > r ? m : r; }
    if constexpr (LPV <= 2) { r = ror(m, std::integral_constant<int, 2>{}); m = m > r ? m : r; }
    if constexpr (LPV <= 4) { r = ror(m, std::integral_constant<int, 4>{}); m = m > r ? m : r; }
    r = ror(m, std::integral_constant<int, 8>{});
    m = m > r ? m : r;
    const auto h = __builtin_amdgcn_permlane16_swap(m, m, false, false);
    m = h[0] > h[1] ? h[0] : h[1];
    const auto w = __builtin_amdgcn_permlane32_swap(m, m, false, false);
    return w[0] > w[1] ? w[0] : w[1];
}

template <int LPV, int S>
__device__ __forceinline__ float group_bcast(float x) {
    return __builtin_bit_cast(float, group_bcast<LPV, S>(__builtin_bit_cast(unsigned, x)));
}

// Compile-time loop: f(std::integral_constant<int, K>) for K in the sequence.
template <int... K, typename F>
__device__ __forceinline__ void static_for(std::integer_sequence<int, K...>, F &&f) {
    (f(std::integral_constant<int, K>{}), ...);
}


__device__ __forceinline__ float h_lo(unsigned u) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(u & 0xffffu));
}
__device__ __forceinline__ float h_hi(unsigned u) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(u >> 16)); }

// fmaf(h, b, c) with h the fp16 in half HI of u, as one v_fma_mix_f32: the
// fp16 -> fp32 conversion is exact and the fma rounds once, so this equals
// fmaf(HI ? h_hi(u) : h_lo(u), b, c) bit for bit -- without the separate
// v_cvt_f32_f16 (the compiler packs the fp32 fmas instead and keeps the
// conversions).  With c = -0.0f it is the product h * b exactly (x + -0 = x,
// signed zeros included).
template <int HI>
__device__ __forceinline__ float fma_h(unsigned u, float b, float c) {
    float d;
    if constexpr (HI)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(u), "v"(b), "v"(c));
    else
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(u), "v"(b), "v"(c));
    return d;
}

// Bilinear setup of one voxel-camera (aten grid_sampler_2d, align_corners=True,
// zeros padding): weights nw, ne, sw, se and the byte offsets of the taps
// (kOOB when outside).  CL: 4 pixel offsets.  PAIR: 2 row-entry offsets.
template <bool PAIR>
struct Taps4 {
    static constexpr int NO = PAIR ? 2 : 4;
    unsigned o[NO];
    float w[4];
};

// Top-left tap (x0, y0) of a sample at heatmap pixel (ix, iy).  NaN
// coordinates read in-image taps so the NaN weights propagate (as in
// grid_sample); far-off coordinates are clamped before the int conversion.
__device__ __forceinline__ void tap_origin(float ix, float iy, int W, int H, int &x0, int &y0) {
    const bool nan_ = (ix != ix) || (iy != iy);
    x0 = nan_ ? 0 : (int)fminf(fmaxf(floorf(ix), -4.0f), (float)W + 4.0f);
    y0 = nan_ ? 0 : (int)fminf(fmaxf(floorf(iy), -4.0f), (float)H + 4.0f);
}

template <bool PAIR>
__device__ __forceinline__ Taps4<PAIR> setup_taps(float gx, float gy, float sxs, float sys, int W, int H,
                                                  unsigned unit) {
    Taps4<PAIR> t;
    const float ix = (gx + 1.0f) * sxs;
    const float iy = (gy + 1.0f) * sys;
    const float x0f = floorf(ix), y0f = floorf(iy);
    const float wx = ix - x0f, ex = 1.0f - wx;
    const float ny = iy - y0f, syw = 1.0f - ny;
    t.w[0] = syw * ex;
    t.w[1] = syw * wx;
    t.w[2] = ny * ex;
    t.w[3] = ny * wx;
    int x0, y0;
    tap_origin(ix, iy, W, H, x0, y0);
    const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)(y0 + 1) < (unsigned)H;
    if constexpr (PAIR) {
        const bool vx = (x0 >= -1) & (x0 < W);
        const unsigned e0 = (unsigned)(y0 * (W + 1) + x0 + 1) * unit;
        t.o[0] = (vx & vy0) ? e0 : kOOB;
        t.o[1] = (vx & vy1) ? e0 + (unsigned)(W + 1) * unit : kOOB;
    } else {
        const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)(x0 + 1) < (unsigned)W;
        const unsigned p = (unsigned)(y0 * W + x0) * unit;
        t.o[0] = (vy0 & vx0) ? p : kOOB;
        t.o[1] = (vy0 & vx1) ? p + unit : kOOB;
        t.o[2] = (vy1 & vx0) ? p + (unsigned)W * unit : kOOB;
        t.o[3] = (vy1 & vx1) ? p + (unsigned)(W + 1) * unit : kOOB;
    }
    return t;
}

inline int lanes_per_voxel(int J) { return J <= 4 ? 1 : J <= 8 ? 2 : J <= 16 ? 4 : 8; }

inline size_t cl_frame_bytes(int V, int J, int H, int W) {
    return (size_t)V * H * W * 4 * lanes_per_voxel(J) * sizeof(float);
}

template <int LPV, typename T, int NF = 1>
inline void launch_layout(const T *hm, int nb, int V, int J, int Jst, int H, int W, float *cl, hipStream_t s) {
    const long long px = (long long)nb * V * H * W;
    const long long threads = px * LPV;
    hipLaunchKernelGGL((heatmaps_to_cl_kernel<LPV, T, NF>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                       hm, reinterpret_cast<float4 *>(cl), J, Jst, H * W, V, px);
}

}  // namespace fvp
