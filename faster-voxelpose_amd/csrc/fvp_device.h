// Device-side helpers shared by the fvp kernels (gfx950 / CDNA4).
//
// Floating-point contract: every expression below reproduces the fp32
// operation sequence of the reference's PyTorch CPU path, which the oracle
// (oracle/fvp_oracle.py) pins bit-exactly against reference-generated vectors:
//   * separate torch ops are separately rounded   -> contraction is OFF here
//   * torch.mm with K=3 accumulates fma(a2,b2, fma(a1,b1, a0*b0))
//   * torch.linspace is fma(step,i,start) / fma(-step,n-1-i,end)
//   * grid_sample accumulates fma(se_v,se, fma(sw_v,sw, fma(ne_v,ne, nw_v*nw)))
//   * torch.mean(dim=0) over the V views (project_whole.py:162,
//     project_individual.py:283) is sum / V, the sum in ATen's cascade order
//     (SumKernel.cpp multi_row_sum, level step 16): views accumulate
//     sequentially from 0 in blocks of 16; each complete block is folded into
//     a second accumulator (itself a sequential sum of block sums from 0); the
//     total is remainder + blocks.  V <= 16 is a plain sequential sum.
//     (Verified against torch here for V = 5..100; the last < 64 output
//     elements of a tensor -- never a whole-space cube -- take ATen's ILP-4
//     tail order instead, machine-dependent, at most 1 ulp apart.)
// Compile with -ffp-contract=off and correctly rounded fp32 division.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fvp.h"

#pragma clang fp contract(off)

namespace fvp {

constexpr int kWave = 64;

struct Cam {
    float R[9], T[3], f[2], c[2], k[3], p[2];
};

__device__ __forceinline__ Cam load_cam(const float *__restrict__ rec) {
    Cam c;
#pragma unroll
    for (int i = 0; i < 9; ++i) c.R[i] = rec[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) c.T[i] = rec[9 + i];
    c.f[0] = rec[12]; c.f[1] = rec[13];
    c.c[0] = rec[14]; c.c[1] = rec[15];
    c.k[0] = rec[16]; c.k[1] = rec[17]; c.k[2] = rec[18];
    c.p[0] = rec[19]; c.p[1] = rec[20];
    return c;
}

// torch.linspace(start, end, n)[i] (fp32 CPU kernel), then + centre.
__device__ __forceinline__ float axis_coord(float start, float end, int n, int i, float centre) {
    float v;
    if (n == 1) {
        v = start;
    } else {
        const float step = (end - start) / (float)(n - 1);
        v = (i < n / 2) ? __builtin_fmaf(step, (float)i, start)
                        : __builtin_fmaf(-step, (float)(n - 1 - i), end);
    }
    return v + centre;
}

// torch.clamp: NaN propagates.
__device__ __forceinline__ float clampf(float x, float lo, float hi) {
    return (x != x) ? x : fminf(fmaxf(x, lo), hi);
}

// torch.max reduction: NaN propagates.
__device__ __forceinline__ float nanmax(float a, float b) {
    return (b > a || b != b) ? b : a;
}

// a0 / b and a1 / b, correctly rounded, for the two quotients of one divisor in
// project_point (y = xcam[:2] / (xcam[2] + 1e-5), cameras.py:44).  The IEEE
// division the compiler emits (-fhip-fp32-correctly-rounded-divide-sqrt) is
// v_div_scale x2, v_rcp, fma(-d, r, 1), fma(e, r, r), n * r, then two
// remainder steps fma(-d, q, n) / fma(e, r, q), v_div_fmas and v_div_fixup.
// When |a0|, |a1| and |b| lie in [2^-40, 2^40] none of its scaling or fixup
// cases can trigger (v_div_scale scales only for an exponent gap >= 96, a
// denormal divisor, reciprocal or quotient, or a numerator below 2^-103;
// v_div_fixup acts only on NaN / inf / zero operands and out-of-range
// quotients), so that sequence is exactly the unscaled core below -- whose
// reciprocal refinement depends on b alone and is shared by both numerators:
// 3 + 2 x 5 VALU ops (plus the range test) against 2 x ~12.  Outside the range
// (zero numerators, divisors near 0) the lanes take the IEEE division itself.
// Bit-identity is also checked on the host for reciprocal seeds 1 ulp either
// side of RN(1/b) (tests/test_div_const.py::test_div_pair_*) and by the C1-C5
// sample-grid and on-the-fly cube digests.
__device__ __forceinline__ void div_pair(float a0, float a1, float b, float &q0, float &q1) {
    const float r0 = __builtin_amdgcn_rcpf(b);
    const float r = __builtin_fmaf(__builtin_fmaf(-b, r0, 1.0f), r0, r0);
    const float lo = fminf(fminf(fabsf(a0), fabsf(a1)), fabsf(b));
    const float hi = fmaxf(fmaxf(fabsf(a0), fabsf(a1)), fabsf(b));
    if (lo >= 0x1p-40f && hi <= 0x1p40f) {
        float q = a0 * r;
        q = __builtin_fmaf(__builtin_fmaf(-b, q, a0), r, q);
        q0 = __builtin_fmaf(__builtin_fmaf(-b, q, a0), r, q);
        q = a1 * r;
        q = __builtin_fmaf(__builtin_fmaf(-b, q, a1), r, q);
        q1 = __builtin_fmaf(__builtin_fmaf(-b, q, a1), r, q);
    } else {
        q0 = a0 / b;
        q1 = a1 / b;
    }
}

// lib/utils/cameras.py:30-56 project_point for one world point -> pixel.
__device__ __forceinline__ void project_point(const Cam &c, float x, float y, float z, float &px, float &py) {
    const float dx = x - c.T[0], dy = y - c.T[1], dz = z - c.T[2];
    const float xc0 = __builtin_fmaf(c.R[2], dz, __builtin_fmaf(c.R[1], dy, c.R[0] * dx));
    const float xc1 = __builtin_fmaf(c.R[5], dz, __builtin_fmaf(c.R[4], dy, c.R[3] * dx));
    const float xc2 = __builtin_fmaf(c.R[8], dz, __builtin_fmaf(c.R[7], dy, c.R[6] * dx));
    const float den = xc2 + 1e-5f;
    float y0, y1;
    div_pair(xc0, xc1, den, y0, y1);
    const float r = y0 * y0 + y1 * y1;
    float d = (1.0f + c.k[0] * r) + (c.k[1] * r) * r;
    d = d + ((c.k[2] * r) * r) * r;
    const float u = (y0 * d + ((2.0f * c.p[0]) * y0) * y1) + c.p[1] * (r + (2.0f * y0) * y0);
    const float v = (y1 * d + ((2.0f * c.p[1]) * y0) * y1) + c.p[0] * (r + (2.0f * y1) * y1);
    px = c.f[0] * u + c.c[0];
    py = c.f[1] * v + c.c[1];
}

// a / b for a divisor fixed per launch, rb = 1.0f / b (correctly rounded; the
// callers' loop-invariant division, hoisted out of their loops): q = a*rb,
// the exact remainder a - q*b by one fma, one correction step.  Three VALU
// ops against ~10 for an IEEE division (v_div_scale / v_rcp / v_div_fmas /
// v_div_fixup).  Equal to the correctly rounded a / b for every integer
// divisor b in [1, 65535] whenever the quotient is a normal float: checked
// for every odd b in that range over all 2^23 mantissas of a in [1, 2)
// (tools/div_const_sweep.c; the three operations and a / b scale exactly by
// powers of two in a and in b while everything stays normal, and are odd in
// a), and over whole fp32 exponent ranges for the BASELINE divisors
// (tests/test_div_const.py).  Only subnormal quotients (|a| < ~1e-36 here)
// and a = -0 (gives +0) can differ.  Markstein's theorem alone does not
// cover it (RN(a * RN(1/b)) can be 1.5 ulp off), so the fast path is taken
// only for divisors the sweep covers (ImageConsts::exact, set on the host);
// any other divisor takes the IEEE division.
__device__ __forceinline__ float div_const(float a, float b, float rb) {
    const float q = a * rb;
    return __builtin_fmaf(__builtin_fmaf(-q, b, a), rb, q);
}

// The launch constants of pixel_to_sample: fvp_image_spec plus which of the
// four divisors div_const serves exactly (bit 0 img_w, 1 img_h, 2 hm_w - 1,
// 3 hm_h - 1; image_consts() on the host).
struct ImageConsts {
    float ori_max, img_w, img_h, hm_w, hm_h;
    unsigned exact;
};

// Host: an integer divisor in [1, 4095] -- the range tests/test_div_const.py sweeps
// with tools/div_const_sweep.c on every CPU run (every image and heatmap size of
// the reference's configs); any other divisor takes the IEEE division.
inline bool div_const_covered(float b) {
    return b >= 1.0f && b <= 4095.0f && (float)(int)b == b;
}

inline ImageConsts image_consts(const fvp_image_spec &im) {
    ImageConsts c{im.ori_max, im.img_w, im.img_h, (float)im.hm_w, (float)im.hm_h, 0u};
    c.exact = (div_const_covered(im.img_w) ? 1u : 0u) | (div_const_covered(im.img_h) ? 2u : 0u) |
              (div_const_covered((float)im.hm_w - 1.0f) ? 4u : 0u) |
              (div_const_covered((float)im.hm_h - 1.0f) ? 8u : 0u);
    return c;
}

__device__ __forceinline__ float div_launch(float a, float b, bool exact) {
    return exact ? div_const(a, b, 1.0f / b) : a / b;
}

// project_whole.py:96-117 after project_pose: pixel -> normalised sample coords.
// The four divisions by launch constants use div_const where it is exact
// (ImageConsts::exact): where it could differ from an IEEE division (a
// subnormal or -0 quotient) the value next goes through `* 2 - 1` (directly,
// or after a second division that keeps it below 2^-100), which rounds it to
// -1 either way, so gx / gy are bit-identical to the reference's (and the
// sample-grid digests of C1-C5 pin it).
__device__ __forceinline__ void pixel_to_sample(float px, float py, const float *__restrict__ t,
                                                const ImageConsts &c, float &gx, float &gy) {
    px = clampf(px, -1.0f, c.ori_max);
    py = clampf(py, -1.0f, c.ori_max);
    // transforms.py:59-63: torch.mm(t, [x, y, 1]^T)
    const float ax = __builtin_fmaf(t[2], 1.0f, __builtin_fmaf(t[1], py, t[0] * px));
    const float ay = __builtin_fmaf(t[5], 1.0f, __builtin_fmaf(t[4], py, t[3] * px));
    const float sw = c.hm_w - 1.0f, sh = c.hm_h - 1.0f;
    const float hx = div_launch(ax * c.hm_w, c.img_w, c.exact & 1u);
    const float hy = div_launch(ay * c.hm_h, c.img_h, c.exact & 2u);
    gx = clampf(div_launch(hx, sw, c.exact & 4u) * 2.0f - 1.0f, -1.1f, 1.1f);
    gy = clampf(div_launch(hy, sh, c.exact & 8u) * 2.0f - 1.0f, -1.1f, 1.1f);
}

// Bilinear tap set of F.grid_sample(align_corners=True, padding zeros) at a
// normalised coordinate; offsets are clamped into the plane so loads are
// always legal, and the in-bounds mask selects 0 for outside taps.
struct Taps {
    int o00, o01, o10, o11;   // plane offsets (y*W + x), clamped
    bool m00, m01, m10, m11;  // in-bounds flags
    float nw, ne, sw, se;     // weights
    bool any;                 // at least one tap inside
    bool nan;                 // coordinate is NaN -> result NaN
};

__device__ __forceinline__ Taps make_taps(float gx, float gy, int H, int W) {
    Taps t;
    const float ix = (gx + 1.0f) * ((float)(W - 1) * 0.5f);
    const float iy = (gy + 1.0f) * ((float)(H - 1) * 0.5f);
    t.nan = (ix != ix) || (iy != iy);
    const float x0f = floorf(ix), y0f = floorf(iy);
    const float wx = ix - x0f, ex = 1.0f - wx;
    const float ny = iy - y0f, sy = 1.0f - ny;
    t.nw = sy * ex; t.ne = sy * wx; t.sw = ny * ex; t.se = ny * wx;
    const int x0 = t.nan ? -2 : (int)x0f, y0 = t.nan ? -2 : (int)y0f;
    const int x1 = x0 + 1, y1 = y0 + 1;
    const bool vx0 = (x0 >= 0) & (x0 < W), vx1 = (x1 >= 0) & (x1 < W);
    const bool vy0 = (y0 >= 0) & (y0 < H), vy1 = (y1 >= 0) & (y1 < H);
    t.m00 = vy0 & vx0; t.m01 = vy0 & vx1; t.m10 = vy1 & vx0; t.m11 = vy1 & vx1;
    t.any = t.m00 | t.m01 | t.m10 | t.m11;
    const int cx0 = min(max(x0, 0), W - 1), cx1 = min(max(x1, 0), W - 1);
    const int cy0 = min(max(y0, 0), H - 1), cy1 = min(max(y1, 0), H - 1);
    t.o00 = cy0 * W + cx0; t.o01 = cy0 * W + cx1; t.o10 = cy1 * W + cx0; t.o11 = cy1 * W + cx1;
    return t;
}

template <typename T>
__device__ __forceinline__ float to_f32(T v) { return (float)v; }

template <typename T>
__device__ __forceinline__ float sample(const T *__restrict__ plane, const Taps &t) {
    const float a = t.m00 ? to_f32(plane[t.o00]) : 0.0f;
    const float b = t.m01 ? to_f32(plane[t.o01]) : 0.0f;
    const float c = t.m10 ? to_f32(plane[t.o10]) : 0.0f;
    const float d = t.m11 ? to_f32(plane[t.o11]) : 0.0f;
    return __builtin_fmaf(d, t.se, __builtin_fmaf(c, t.sw, __builtin_fmaf(b, t.ne, a * t.nw)));
}

// Bijective XCD-aware block remap: the hardware deals blocks round-robin over
// the 8 XCDs; give each XCD a contiguous range of logical blocks so the tiles
// of one frame share an L2.  Speed only -- any placement stays correct.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int nx = 8;
    const int xcd = bid % nx, k = bid / nx;
    const int q = nblk / nx, r = nblk % nx;
    return xcd * q + min(xcd, r) + k;
}

}  // namespace fvp
