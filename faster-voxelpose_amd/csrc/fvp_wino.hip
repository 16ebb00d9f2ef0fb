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
//   1. the 10 x 18 x 16 input halo -> LDS (float4 loads, zero outside the image)
//   2. input transform: thread (tile, channel) -> V[xi][c parity][tile][c/2]
//   3. wave w owns xi = 4w .. 4w+3: per xi and 32 columns, 8 v_mfma_f32_32x32x2f32
//      with A = V (two ds_read_b128 per lane) and B = the transformed weights
//      straight from global memory (two 16-B loads per lane, k-contiguous)
// After the K loop the 16 xi accumulators of each (tile, channel) meet in LDS,
// the output transform makes the 2x2 outputs and the epilogue of
// fvp_conv2d_nhwc_ex is applied: acc * scale + shift (+ res_pre), ReLU,
// (+ res_post), NHWC stores.
#include "fvp_layout.h"

// (probe builds: FVP_WINO_MODE 1 = no MFMAs, 2 = no input transform, 3 = no output phase)
#ifndef FVP_WINO_MODE
#define FVP_WINO_MODE 0
#endif
#ifndef FVP_WINO_R
#define FVP_WINO_R 1
#endif

namespace fvp {

typedef float wf32x16 __attribute__((ext_vector_type(16)));

struct WinoArgs {
    const float *in;        // [N][H][W][Cpi]
    const float *u;         // [16][Cpi/16][Cpo][2][8]: U = G g G^T per (xi, 16-channel step, co, c parity, c/2)
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
constexpr int kWinoVT = 12;                                // V LDS floats per (xi, parity, tile) (8 + pad)
constexpr int kWinoHalo = kWinoHH * kWinoHW * kWinoHP;     // 3,600 floats
constexpr int kWinoV = 16 * 2 * 32 * kWinoVT;              // 12,288 floats
constexpr int kWinoX = 16 * 32 * 32;                       // 16,384 floats: [xi][tile][32 columns]
constexpr int kWinoLds = (kWinoHalo + kWinoV > kWinoX ? kWinoHalo + kWinoV : kWinoX);

template <int NB>
__global__ __launch_bounds__(256, 2) void conv_wino_kernel(WinoArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *halo = lds, *vt = lds + kWinoHalo, *xch = lds;  // xch reuses the K-loop region after the loop
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int bid = blockIdx.x;
    const int nblk = a.Cpo / (32 * NB);
    const int cb = bid % nblk;
    bid /= nblk;
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int img = bid / a.tiles_y;
    const int y0 = ty * kWinoTH, x0 = tx * kWinoTW;
    const int n0 = cb * 32 * NB;
    const float *__restrict__ src = a.in + (size_t)img * a.H * a.W * a.Cpi;
    const int ksteps = a.Cpi / 16;

    wf32x16 acc[4][NB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    // halo slot s (< 720): pixel s / 4, channel quad s % 4
    auto halo_load = [&](int ks, f32x4 (&h)[3]) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int s = tid + 256 * u;
            const int p = s >> 2, q = s & 3;
            const int hy = p / kWinoHW, hx = p - hy * kWinoHW;
            const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (s < kWinoHH * kWinoHW * 4 && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)
                v = *reinterpret_cast<const f32x4 *>(src + ((size_t)gy * a.W + gx) * a.Cpi + ks * 16 + 4 * q);
            h[u] = v;
        }
    };
    f32x4 hnext[3];
    halo_load(0, hnext);
    const int par = lane >> 5, trow = lane & 31;
    // this wave's B fragments of one K step: xi = 4w + i, 32-column block j (k-contiguous, 2 x 16 B per lane)
    auto b_load = [&](int ks, f32x4 (&b)[4][NB][2]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const float *bp =
                    a.u + (((((size_t)(4 * wave + i)) * ksteps + ks) * a.Cpo + n0 + 32 * j + trow) * 2 + par) * 8;
                b[i][j][0] = *reinterpret_cast<const f32x4 *>(bp);
                b[i][j][1] = *reinterpret_cast<const f32x4 *>(bp + 4);
            }
    };
    f32x4 bcur[4][NB][2];
    b_load(0, bcur);
    for (int ks = 0; ks < ksteps; ++ks) {
        __syncthreads();  // the previous step's transform has read the halo
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int s = tid + 256 * u;
            if (s < kWinoHH * kWinoHW * 4)
                *reinterpret_cast<f32x4 *>(halo + (s >> 2) * kWinoHP + 4 * (s & 3)) = hnext[u];
        }
        if (ks + 1 < ksteps) halo_load(ks + 1, hnext);  // in flight during this step's transform and MFMAs
        __syncthreads();  // halo written; the previous step's MFMAs have read V
        // input transform: item = tile * 16 + c, two per thread
#pragma unroll
        for (int it = 0; it < (FVP_WINO_MODE == 2 ? 0 : 2); ++it) {
            const int item = tid + 256 * it;
            const int t = item >> 4, c = item & 15;
            const int ti = t >> 3, tj = t & 7;
            const float *hp = halo + ((2 * ti) * kWinoHW + 2 * tj) * kWinoHP + c;
            float d[4][4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int s = 0; s < 4; ++s) d[r][s] = hp[(r * kWinoHW + s) * kWinoHP];
            // B^T d: rows (d0 - d2, d1 + d2, d2 - d1, d1 - d3)
            float e[4][4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                e[0][s] = d[0][s] - d[2][s];
                e[1][s] = d[1][s] + d[2][s];
                e[2][s] = d[2][s] - d[1][s];
                e[3][s] = d[1][s] - d[3][s];
            }
            float *vp = vt + ((c & 1) * 32 + t) * kWinoVT + (c >> 1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v0 = e[r][0] - e[r][2], v1 = e[r][1] + e[r][2];
                const float v2 = e[r][2] - e[r][1], v3 = e[r][1] - e[r][3];
                vp[(r * 4 + 0) * 2 * 32 * kWinoVT] = v0;
                vp[(r * 4 + 1) * 2 * 32 * kWinoVT] = v1;
                vp[(r * 4 + 2) * 2 * 32 * kWinoVT] = v2;
                vp[(r * 4 + 3) * 2 * 32 * kWinoVT] = v3;
            }
        }
        __syncthreads();
#if FVP_WINO_MODE != 1
        // MFMAs: wave w, xi = 4w + i; lane: tile row trow (A) / column (B), c parity par
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int xi = 4 * wave + i;
            const float *ap = vt + ((xi * 2 + par) * 32 + trow) * kWinoVT;
            const f32x4 a0 = *reinterpret_cast<const f32x4 *>(ap);
            const f32x4 a1 = *reinterpret_cast<const f32x4 *>(ap + 4);
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const f32x4 b0 = bcur[i][j][0], b1 = bcur[i][j][1];
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[k], b0[k], acc[i][j], 0, 0, 0);
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[k], b1[k], acc[i][j], 0, 0, 0);
            }
        }
#endif
        if (ks + 1 < ksteps) b_load(ks + 1, bcur);  // lands during the next step's halo write and transform
    }
#if FVP_WINO_MODE == 3
    if (acc[0][0][0] == 1.2345e-30f) a.out[0] = acc[0][NB - 1][15];  // keep the MFMAs live, no output phase
    return;
#endif
    // output transform, one 32-column block at a time: accumulators -> xch[xi][tile][col].
    // A thread's four items share its column (item = tid + 256 it, column = tid % 32);
    // their scale / shift and residuals are loaded before the exchange, so no load
    // waits behind an output store (out may alias nothing, but the compiler cannot
    // know: loads after a store were each a dependent round trip).
    const int col = tid & 31;
    const float *__restrict__ rpre_p = a.res_pre;
    const float *__restrict__ rpost_p = a.res_post;
    auto out_off = [&](int t, int dy, int dx, int co, bool &ok) {
        const int oy = y0 + 2 * (t >> 3) + dy, ox = x0 + 2 * (t & 7) + dx;
        ok = oy < a.H && ox < a.W;
        return (((size_t)img * a.H + oy) * a.W + ox) * a.Cpo + co;
    };
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int co = n0 + 32 * j + col;
        const float sc = a.scale[co], sh = a.shift[co];
        // the layer's residual (res_pre, else res_post; with both, res_post is read at the store)
        const float *__restrict__ rfirst = rpre_p ? rpre_p : rpost_p;
        float rv[4][4];
#pragma unroll
        for (int it = 0; it < 4; ++it)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                bool ok;
                const size_t off = out_off((tid + 256 * it) >> 5, q >> 1, q & 1, co, ok);
                rv[it][q] = (rfirst && ok) ? rfirst[off] : 0.0f;
            }
        __syncthreads();  // K loop done / the previous block's transform has read xch
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int xi = 4 * wave + i;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int t = 8 * (r >> 2) + 4 * par + (r & 3);  // v_mfma_f32_32x32x2f32 row of register r
                xch[(xi * 32 + t) * 32 + trow] = acc[i][j][r];
            }
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int t = (tid + 256 * it) >> 5;
            float m[4][4];
#pragma unroll
            for (int xi = 0; xi < 16; ++xi) m[xi >> 2][xi & 3] = xch[(xi * 32 + t) * 32 + col];
            // A^T m: rows (m0 + m1 + m2, m1 - m2 - m3)
            float f[2][4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                f[0][s] = (m[0][s] + m[1][s]) + m[2][s];
                f[1][s] = (m[1][s] - m[2][s]) - m[3][s];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int dy = q >> 1, dx = q & 1;
                bool ok;
                const size_t off = out_off(t, dy, dx, co, ok);
                if (!ok) continue;
                float v = dx == 0 ? (f[dy][0] + f[dy][1]) + f[dy][2] : (f[dy][1] - f[dy][2]) - f[dy][3];
                v = v * sc + sh;
                if (rpre_p) v = v + rv[it][q];
                if (a.relu) v = fmaxf(v, 0.0f);
                if (rpost_p) v = v + (rpre_p ? rpost_p[off] : rv[it][q]);
                a.out[off] = v;
            }
        }
    }
}

// The same convolution with the 16 transform positions of a (tile, column) in
// ONE lane: v_mfma_f32_16x16x4f32, a wave owns 16 tiles x NB*16 columns and
// keeps all 16 xi accumulators (16 * NB * 4 registers), so the output
// transform runs in registers -- no LDS exchange, no barrier after the K loop,
// 46 KB of LDS per block.  Waves: (tile half th = w & 1) x (column half ch = w >> 1).
// V in LDS: [xi][c mod 4][tile ^ 2 (c mod 4)][c / 4] (the XOR keeps the
// transform's stores conflict-free, the MFMA reads stay 16 contiguous tiles);
// U: [16][Cpi/16][c mod 4][Cpo][c/4 (4)].
constexpr int kWinoRV = 16 * 4 * 32 * 4;                    // 8,192 floats
constexpr int kWinoRLds = kWinoHalo + kWinoRV;

template <int NB>
__global__ __launch_bounds__(256, 2) void conv_wino_r_kernel(WinoArgs a) {
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
    const int th = wave & 1, chf = wave >> 1;
    const int nw = cbk * 32 * NB + chf * 16 * NB;  // this wave's first column
    const float *__restrict__ src = a.in + (size_t)img * a.H * a.W * a.Cpi;
    const int ksteps = a.Cpi / 16;
    const int l16 = lane & 15, cm = lane >> 4;

    f32x4 acc[16][NB];
#pragma unroll
    for (int x = 0; x < 16; ++x)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[x][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto halo_load = [&](int ks, f32x4 (&h)[3]) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int s = tid + 256 * u;
            const int p = s >> 2, q = s & 3;
            const int hy = p / kWinoHW, hx = p - hy * kWinoHW;
            const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (s < kWinoHH * kWinoHW * 4 && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)
                v = *reinterpret_cast<const f32x4 *>(src + ((size_t)gy * a.W + gx) * a.Cpi + ks * 16 + 4 * q);
            h[u] = v;
        }
    };
    // B fragment of (xi, step ks, column block j): U[xi][ks][cm][co][0..3], co = nw + 16 j + l16
    auto b_at = [&](int xi, int ks, int j) {
        return *reinterpret_cast<const f32x4 *>(
            a.u + ((((size_t)xi * ksteps + ks) * 4 + cm) * a.Cpo + nw + 16 * j + l16) * 4);
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
        f32x4 bq[2][4][NB];  // B of 4 xi at a time, the next group loading while one is used
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int j = 0; j < NB; ++j) bq[0][x][j] = b_at(x, ks, j);
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
        // MFMAs: 16 xi x NB column blocks x 4 channel quads
        const int ta = (16 * th + l16) ^ (2 * cm);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (g < 3) {
#pragma unroll
                for (int x = 0; x < 4; ++x)
#pragma unroll
                    for (int j = 0; j < NB; ++j) bq[(g + 1) & 1][x][j] = b_at(4 * (g + 1) + x, ks, j);
            }
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const int xi = 4 * g + x;
                const f32x4 av = *reinterpret_cast<const f32x4 *>(vt + ((xi * 4 + cm) * 32 + ta) * 4);
#pragma unroll
                for (int j = 0; j < NB; ++j)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        acc[xi][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[k], bq[g & 1][x][j][k], acc[xi][j], 0, 0, 0);
            }
        }
    }
    // output transform in registers: lane holds tiles 16 th + 4 cm + r (r < 4), column nw + 16 j + l16
    const float *__restrict__ rpre_p = a.res_pre;
    const float *__restrict__ rpost_p = a.res_post;
    const float *__restrict__ rfirst = rpre_p ? rpre_p : rpost_p;
    auto out_off = [&](int t, int q, int co, bool &ok) {
        const int oy = y0 + 2 * (t >> 3) + (q >> 1), ox = x0 + 2 * (t & 7) + (q & 1);
        ok = oy < a.H && ox < a.W;
        return (((size_t)img * a.H + oy) * a.W + ox) * a.Cpo + co;
    };
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int co = nw + 16 * j + l16;
        const float sc = a.scale[co], sh = a.shift[co];
        float rv[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                bool ok;
                const size_t off = out_off(16 * th + 4 * cm + r, q, co, ok);
                rv[r][q] = (rfirst && ok) ? rfirst[off] : 0.0f;
            }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = 16 * th + 4 * cm + r;
            float f[2][4];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                f[0][s2] = (acc[s2][j][r] + acc[4 + s2][j][r]) + acc[8 + s2][j][r];
                f[1][s2] = (acc[4 + s2][j][r] - acc[8 + s2][j][r]) - acc[12 + s2][j][r];
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
#if FVP_WINO_R
    const size_t lds = (size_t)fvp::kWinoRLds * sizeof(float);
    if (nb == 2)
        hipLaunchKernelGGL(fvp::conv_wino_r_kernel<2>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL(fvp::conv_wino_r_kernel<1>, dim3((unsigned)blocks), dim3(256), lds, s, a);
#else
    const size_t lds = (size_t)fvp::kWinoLds * sizeof(float);
    if (nb == 2)
        hipLaunchKernelGGL(fvp::conv_wino_kernel<2>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL(fvp::conv_wino_kernel<1>, dim3((unsigned)blocks), dim3(256), lds, s, a);
#endif
    return (int)hipGetLastError();
}
