// 3x3 stride-1 "same" convolutions by Winograd F(2x2, 3x3) on the fp32
// matrix cores (the Basic2DBlock / Res2DBlock 3x3
// layers of P2PNet and CenterNet, cnns_2d.py:12-125; the 3x3 layers of the
// PoseResNet Bottlenecks, resnet.py:60-95).
//
// out = A^T [ sum_ci (G g G^T) . (B^T d B) ] A over 2x2 output tiles, d the
// 4x4 input patch: 16 products per 4 outputs and input channel instead of 36
// -- 2.25x fewer MFMA operations than the direct (implicit GEMM) kernels of
// fvp_conv.hip.  Every other step is an exact fp32 operation sequence: the
// input transform B^T d B and the output transform A^T m A are sums and
// differences, the weight transform G g G^T is computed once on the host in
// fp64 and rounded to fp32.  The result differs from the direct convolution by
// the transforms' rounding (a few ulp of the partial sums; tests/test_cnn.py
// bounds it with the other fp32 kernels).
//
// Block = 256 threads, an 8 x 16 output tile (32 Winograd tiles) of one image
// x NB*32 output channels.  Per 16-channel K step:
//   1. the 10 x 18 x 16 input halo -> LDS (float4 loads issued a step ahead,
//      zero outside the image)
//   2. input transform: thread (tile, channel) -> V[xi][c mod 4][tile][c / 4]
//   3. v_mfma_f32_16x16x4f32 (16 tiles x 16 columns x 4 channels): A = V (one
//      ds_read_b128 per lane and 4 channels), B = the transformed weights
//      straight from global memory (one 16-B load per lane, 4 xi in flight)
// All 16 xi accumulators of a (tile, column) sit in one lane, so after the K
// loop the output transform runs in registers and the epilogue of
// fvp_conv2d_nhwc_ex is applied: acc * scale + shift (+ res_pre), ReLU,
// (+ res_post), NHWC stores.
#include "fvp_layout.h"

namespace fvp {

typedef float wf32x16 __attribute__((ext_vector_type(16)));

struct WinoArgs {
    const float *in;        // [N][H][W][Cpi]
    const float *u;         // [16][Cpi/16][4][Cpo][4]: U = G g G^T per (xi, 16-channel step, c mod 4, co, c/4 mod 4)
    const float *scale;     // [Cpo]
    const float *shift;     // [Cpo]
    const float *res_pre;   // [N][H][W][Cpo] or null
    const float *res_post;  // [N][H][W][Cpo] or null
    float *out;             // [N][H][W][Cpo]
    int N, H, W, Cpi, Cpo, relu;
    int tiles_y, tiles_x;   // ceil(H / 8), ceil(W / 16)
};

constexpr int kWinoTH = 8, kWinoTW = 16;                  // output pixels per block
constexpr int kWinoHH = kWinoTH + 2, kWinoHW = kWinoTW + 2;  // input halo
constexpr int kWinoHP = 20;                                // halo LDS floats per pixel (16 + pad, 16-B aligned)
constexpr int kWinoHalo = kWinoHH * kWinoHW * kWinoHP;     // 3,600 floats

// The MFMA tile is 16 tiles x 16 columns and all 16 xi accumulators of a lane
// stay in registers (no LDS exchange, no barrier after the K loop, 46 KB of
// LDS per block).  NB = 2 (64 columns per block): wave w owns the 16 columns
// 16 w .. and both 16-tile halves, so every wave loads different weights (no B
// fragment is fetched twice per block); NB = 1 (32 columns): wave w owns tile
// half w & 1 of column block w >> 1.
// V in LDS: [xi][c mod 4][tile ^ 2 (c mod 4)][c / 4] (the XOR keeps the
// transform's stores conflict-free, the MFMA reads stay 16 contiguous tiles);
// U: [16][Cpi/16][c mod 4][Cpo][c/4 (4)].
constexpr int kWinoRV = 16 * 4 * 32 * 4;                    // 8,192 floats
constexpr int kWinoRLds = kWinoHalo + kWinoRV;

template <int NB>
__global__ __launch_bounds__(256, 2) void conv_wino_kernel(WinoArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *halo = lds, *vt = lds + kWinoHalo;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int bid = blockIdx.x;
    const int nblk = a.Cpo / (32 * NB);
    const int cbk = bid % nblk;
    bid /= nblk;
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int img = bid / a.tiles_y;
    const int y0 = ty * kWinoTH, x0 = tx * kWinoTW;
    const int th0 = NB == 2 ? 0 : (wave & 1);                                   // first tile half
    const int nw = cbk * 32 * NB + 16 * (NB == 2 ? wave : (wave >> 1));          // this wave's 16 columns
    const float *__restrict__ src = a.in + (size_t)img * a.H * a.W * a.Cpi;
    const int ksteps = a.Cpi / 16;
    const int l16 = lane & 15, cm = lane >> 4;

    f32x4 acc[16][NB];  // [xi][tile half]
#pragma unroll
    for (int x = 0; x < 16; ++x)
#pragma unroll
        for (int h = 0; h < NB; ++h) acc[x][h] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto halo_load = [&](int ks, f32x4 (&hl)[3]) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int s = tid + 256 * u;
            const int p = s >> 2, q = s & 3;
            const int hy = p / kWinoHW, hx = p - hy * kWinoHW;
            const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (s < kWinoHH * kWinoHW * 4 && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)
                v = *reinterpret_cast<const f32x4 *>(src + ((size_t)gy * a.W + gx) * a.Cpi + ks * 16 + 4 * q);
            hl[u] = v;
        }
    };
    // B fragment of (xi, step ks): U[xi][ks][cm][co][0..3], co = nw + l16
    const float *__restrict__ ub = a.u + ((size_t)cm * a.Cpo + nw + l16) * 4;
    auto b_at = [&](int xi, int ks) {
        return *reinterpret_cast<const f32x4 *>(ub + ((size_t)xi * ksteps + ks) * 16 * a.Cpo);
    };
    f32x4 hnext[3];
    halo_load(0, hnext);
    for (int ks = 0; ks < ksteps; ++ks) {
        __syncthreads();  // the previous step's transform has read the halo
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int s = tid + 256 * u;
            if (s < kWinoHH * kWinoHW * 4)
                *reinterpret_cast<f32x4 *>(halo + (s >> 2) * kWinoHP + 4 * (s & 3)) = hnext[u];
        }
        if (ks + 1 < ksteps) halo_load(ks + 1, hnext);
        f32x4 bq[2][4];  // B of 4 xi at a time, the next group loading while one is used
#pragma unroll
        for (int x = 0; x < 4; ++x) bq[0][x] = b_at(x, ks);
        __syncthreads();  // halo written; the previous step's MFMAs have read V
#pragma unroll
        for (int it = 0; it < 2; ++it) {  // input transform: item = tile * 16 + c
            const int item = tid + 256 * it;
            const int t = item >> 4, c = item & 15;
            const int ti = t >> 3, tj = t & 7;
            const float *hp = halo + ((2 * ti) * kWinoHW + 2 * tj) * kWinoHP + c;
            float d[4][4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) d[r][s2] = hp[(r * kWinoHW + s2) * kWinoHP];
            float e[4][4];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                e[0][s2] = d[0][s2] - d[2][s2];
                e[1][s2] = d[1][s2] + d[2][s2];
                e[2][s2] = d[2][s2] - d[1][s2];
                e[3][s2] = d[1][s2] - d[3][s2];
            }
            const int cmod = c & 3;
            float *vp = vt + (cmod * 32 + (t ^ (2 * cmod))) * 4 + (c >> 2);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                vp[(r * 4 + 0) * 4 * 32 * 4] = e[r][0] - e[r][2];
                vp[(r * 4 + 1) * 4 * 32 * 4] = e[r][1] + e[r][2];
                vp[(r * 4 + 2) * 4 * 32 * 4] = e[r][2] - e[r][1];
                vp[(r * 4 + 3) * 4 * 32 * 4] = e[r][1] - e[r][3];
            }
        }
        __syncthreads();
        // MFMAs: 16 xi x NB tile halves x 4 channel quads
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (g < 3) {
#pragma unroll
                for (int x = 0; x < 4; ++x) bq[(g + 1) & 1][x] = b_at(4 * (g + 1) + x, ks);
            }
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const int xi = 4 * g + x;
#pragma unroll
                for (int h = 0; h < NB; ++h) {
                    const int ta = (16 * (th0 + h) + l16) ^ (2 * cm);
                    const f32x4 av = *reinterpret_cast<const f32x4 *>(vt + ((xi * 4 + cm) * 32 + ta) * 4);
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        acc[xi][h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[k], bq[g & 1][x][k], acc[xi][h], 0, 0, 0);
                }
            }
        }
    }
    // output transform in registers: lane holds tiles 16 (th0 + h) + 4 cm + r (r < 4), column nw + l16
    const float *__restrict__ rpre_p = a.res_pre;
    const float *__restrict__ rpost_p = a.res_post;
    const float *__restrict__ rfirst = rpre_p ? rpre_p : rpost_p;
    auto out_off = [&](int t, int q, int co, bool &ok) {
        const int oy = y0 + 2 * (t >> 3) + (q >> 1), ox = x0 + 2 * (t & 7) + (q & 1);
        ok = oy < a.H && ox < a.W;
        return (((size_t)img * a.H + oy) * a.W + ox) * a.Cpo + co;
    };
    const int co = nw + l16;
    const float sc = a.scale[co], sh = a.shift[co];
#pragma unroll
    for (int h = 0; h < NB; ++h) {
        float rv[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                bool ok;
                const size_t off = out_off(16 * (th0 + h) + 4 * cm + r, q, co, ok);
                rv[r][q] = (rfirst && ok) ? rfirst[off] : 0.0f;
            }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = 16 * (th0 + h) + 4 * cm + r;
            float f[2][4];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                f[0][s2] = (acc[s2][h][r] + acc[4 + s2][h][r]) + acc[8 + s2][h][r];
                f[1][s2] = (acc[4 + s2][h][r] - acc[8 + s2][h][r]) - acc[12 + s2][h][r];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int dy = q >> 1, dx = q & 1;
                bool ok;
                const size_t off = out_off(t, q, co, ok);
                if (!ok) continue;
                float v = dx == 0 ? (f[dy][0] + f[dy][1]) + f[dy][2] : (f[dy][1] - f[dy][2]) - f[dy][3];
                v = v * sc + sh;
                if (rpre_p) v = v + rv[r][q];
                if (a.relu) v = fmaxf(v, 0.0f);
                if (rpost_p) v = v + (rpre_p ? rpost_p[off] : rv[r][q]);
                a.out[off] = v;
            }
        }
    }
}

}  // namespace fvp

extern "C" int fvp_conv3x3_wino_nhwc(const float *in, int N, int H, int W, int Cpi, const float *u, int Cpo,
                                     const float *scale, const float *shift, const float *res_pre,
                                     const float *res_post, int relu, float *out, void *stream) {
    if (!in || !u || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || Cpi <= 0 || Cpi % 16 || Cpo <= 0 || Cpo % 32) return FVP_ERR_SHAPE;
    fvp::WinoArgs a{in, u, scale, shift, res_pre, res_post, out, N, H, W, Cpi, Cpo, relu,
                    (H + fvp::kWinoTH - 1) / fvp::kWinoTH, (W + fvp::kWinoTW - 1) / fvp::kWinoTW};
    const int nb = Cpo % 64 == 0 ? 2 : 1;
    const long long blocks = (long long)N * a.tiles_y * a.tiles_x * (Cpo / (32 * nb));
    if (blocks > 0x7fffffffLL) return FVP_ERR_SHAPE;
    hipStream_t s = (hipStream_t)stream;
    const size_t lds = (size_t)fvp::kWinoRLds * sizeof(float);
    if (nb == 2)
        hipLaunchKernelGGL(fvp::conv_wino_kernel<2>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL(fvp::conv_wino_kernel<1>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    return (int)hipGetLastError();
}
