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
// Block = 256 * XS threads, a TR x TC grid of Winograd tiles (<= 32: an 8 x 16
// output tile by default, 5 x 5 tiles on 20 x 20 maps, chosen by wino_plan) of
// one image x NB*32 output channels.  Per 16-channel K step:
//   1. the (2TR+2) x (2TC+2) x 16 input halo -> LDS (float4 loads issued a step
//      ahead, zero outside the image)
//   2. input transform: thread (tile, channel) -> V[xi][c mod 4][tile][c / 4]
//   3. v_mfma_f32_16x16x4f32 (16 tiles x 16 columns x 4 channels): A = V (one
//      ds_read_b128 per lane and 4 channels), B = the transformed weights
//      straight from global memory (one 16-B load per lane, 4 xi in flight)
// All 16 xi accumulators of a (tile, column) sit in one lane, so after the K
// loop the output transform runs in registers and the epilogue of
// fvp_conv2d_nhwc_ex is applied: acc * scale + shift (+ res_pre), ReLU,
// (+ res_post), NHWC stores -- and optionally the 2 x 2 max pool that follows
// (Pool2DBlock, cnns_2d.py:67-79): a Winograd tile's four outputs are exactly
// one pool window, so the pooled map is written from the same registers.
#include "fvp_layout.h"


namespace fvp {

struct WinoArgs {
    const float *in;        // [N][H][W][Cpi]
    const float *u;         // [16][Cpi/16][4][Cpo][4]: U = G g G^T per (xi, 16-channel step, c mod 4, co, c/4 mod 4)
    const float *scale;     // [Cpo]
    const float *shift;     // [Cpo]
    const float *res_pre;   // [N][H][W][Cpo] or null
    const float *res_post;  // [N][H][W][Cpo] or null
    float *out;             // [N][H][W][Cpo]
    float *pool;            // [N][H/2][W/2][Cpo]: max_pool2d(out, 2, 2), or null
    int N, H, W, Cpi, Cpo, relu;
    int tr, tc;             // Winograd tiles per block: tr rows x tc columns (tr * tc <= 32)
    int tiles_y, tiles_x;   // blocks per image: ceil(H / 2tr), ceil(W / 2tc)
};

constexpr int kWinoHP = 20;                  // halo LDS floats per pixel (16 + pad, 16-B aligned)
constexpr int kWinoHaloPx = 180;             // halo pixels: (2tr + 2)(2tc + 2) <= 180 (10 x 18 for 4 x 8 tiles)
constexpr int kWinoHalo = kWinoHaloPx * kWinoHP;  // 3,600 floats
constexpr int kWinoV = 16 * 4 * 32 * 4;      // 8,192 floats: V[xi][c mod 4][32 tiles][c / 4]

// The MFMA tile is 16 tiles x 16 columns (v_mfma_f32_16x16x4f32).  A lane keeps
// the 16 / XS transform positions xi of its (tile, column) pairs in registers.
// XS = 1: all 16, so the output transform runs in registers with no exchange.
// XS = 2 (under-filled launches): 8 waves, wave set xs = w >> 2 owns xi 8 xs ..
// 8 xs + 7 (the rows r = 2 xs, 2 xs + 1 of m = A-side 4 x 4); after the K loop
// the two sets swap the halves of their accumulators through LDS so that set
// xs finishes accumulator rows 2 xs, 2 xs + 1 -- twice the waves per block and
// half the MFMA chain per wave.  Within a set: NB = 2 (64 columns per block):
// wave w owns the 16 columns 16 w .. and both 16-tile halves, so every wave
// loads different weights; NB = 1 (32 columns): wave w owns tile half w & 1 of
// column block w >> 1.
// V in LDS: [xi][c mod 4][tile ^ 2 (c mod 4)][c / 4] (the XOR keeps the
// transform's stores conflict-free, the MFMA reads stay 16 contiguous tiles);
// U: [16][Cpi/16][c mod 4][Cpo][c/4 (4)].
__host__ __device__ constexpr int wino_lds_floats(int NB, int XS) {
    return XS == 1 ? kWinoHalo + kWinoV
                   : (kWinoHalo + kWinoV > 8 * 16 * NB * 64 ? kWinoHalo + kWinoV : 8 * 16 * NB * 64);
}

template <int V>
struct WinoIC {
    static constexpr int value = V;
};

template <int NB, int XS>
__global__ __launch_bounds__(256 * XS, XS == 1 ? 2 : 1) void conv_wino_kernel(WinoArgs a) {
    constexpr int NT = 256 * XS, NX = 16 / XS;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *halo = lds, *vt = lds + kWinoHalo;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int xs = XS == 1 ? 0 : wave >> 2, w4 = wave & 3;
    int bid = blockIdx.x;
    const int nblk = a.Cpo / (32 * NB);
    const int cbk = bid % nblk;
    bid /= nblk;
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int img = bid / a.tiles_y;
    const int tr = a.tr, tc = a.tc, ntiles = tr * tc;
    const int hh = 2 * tr + 2, hw = 2 * tc + 2;
    // exact quotients by multiply-shift: t / tc for t < 32 and p / hw for p < 180 (tc <= 16, hw <= 34:
    // the error of 65536 / d + 1 times x < 2^16 / d stays under 1 / d)
    const int mtc = 65536 / tc + 1, mhw = 65536 / hw + 1;
    const int y0 = ty * 2 * tr, x0 = tx * 2 * tc;
    const int th0 = NB == 2 ? 0 : (w4 & 1);                                 // first tile half
    const int nw = cbk * 32 * NB + 16 * (NB == 2 ? w4 : (w4 >> 1));          // this wave's 16 columns
    const float *__restrict__ src = a.in + (size_t)img * a.H * a.W * a.Cpi;
    const int ksteps = a.Cpi / 16;
    const int l16 = lane & 15, cm = lane >> 4;

    f32x4 acc[NX][NB];  // [xi - NX xs][tile half]
#pragma unroll
    for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int h = 0; h < NB; ++h) acc[x][h] = f32x4{0.f, 0.f, 0.f, 0.f};

    constexpr int HU = (kWinoHaloPx * 4 + NT - 1) / NT;  // halo float4 slots per thread
    const int hslots = hh * hw * 4;
    auto halo_load = [&](int ks, f32x4 (&hl)[HU]) {
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            const int sl = tid + NT * u;
            const int p = sl >> 2, q = sl & 3;
            const int hy = (p * mhw) >> 16, hx = p - hy * hw;
            const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (sl < hslots && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)
                v = *reinterpret_cast<const f32x4 *>(src + ((size_t)gy * a.W + gx) * a.Cpi + ks * 16 + 4 * q);
            hl[u] = v;
        }
    };
    // B fragment of (xi, step ks): U[xi][ks][cm][co][0..3], co = nw + l16
    const float *__restrict__ ub = a.u + ((size_t)cm * a.Cpo + nw + l16) * 4;
    auto b_at = [&](int xi, int ks) {
        return *reinterpret_cast<const f32x4 *>(ub + ((size_t)xi * ksteps + ks) * 16 * a.Cpo);
    };
    // XS = 2 (NB = 1, few blocks, registers to spare): the whole step's B (8 fragments) is loaded one
    // step ahead; otherwise groups of 4 xi, the next group loading while one is used (a cross-step
    // prefetch here measured slower: the copy at the loop's back edge waits for the loads, and the
    // extra registers cost the large launches occupancy)
    constexpr bool kPF = NB == 1 && XS == 2;
    constexpr int NBQ = kPF ? NX : 4;
    f32x4 bcur[NBQ], bnext[NBQ], bq[3][4];  // (bq: groups of 4 xi, a ring of 3 -- two groups in flight)
    if constexpr (kPF) {
#pragma unroll
        for (int x = 0; x < NBQ; ++x) bcur[x] = b_at(NX * xs + x, 0);
    }
    f32x4 hnext[HU];
    halo_load(0, hnext);
    for (int ks = 0; ks < ksteps; ++ks) {
        __syncthreads();  // the previous step's transform has read the halo
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            const int sl = tid + NT * u;
            if (sl < hslots) *reinterpret_cast<f32x4 *>(halo + (sl >> 2) * kWinoHP + 4 * (sl & 3)) = hnext[u];
        }
        if (ks + 1 < ksteps) {
            halo_load(ks + 1, hnext);
            if constexpr (kPF) {
#pragma unroll
                for (int x = 0; x < NBQ; ++x) bnext[x] = b_at(NX * xs + x, ks + 1);
            }
        }
        if constexpr (!kPF) {  // groups 0 and 1 land during the input transform
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                bq[0][x] = b_at(NX * xs + x, ks);
                bq[1][x] = b_at(NX * xs + 4 + x, ks);
            }
        }
        __syncthreads();  // halo written; the previous step's MFMAs have read V
#pragma unroll
        for (int it = 0; it < 512 / NT; ++it) {  // input transform: item = tile * 16 + c
            const int item = tid + NT * it;
            const int t = item >> 4, c = item & 15;
            if (t < ntiles) {  // (tiles past tr * tc: their V rows stay unwritten and their outputs unstored)
                const int ti = (t * mtc) >> 16, tj = t - ti * tc;
                const float *hp = halo + ((2 * ti) * hw + 2 * tj) * kWinoHP + c;
                float d[4][4];
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2) d[r][s2] = hp[(r * hw + s2) * kWinoHP];
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
        }
        __syncthreads();
        // MFMAs: NX xi x NB tile halves x 4 channel quads
#pragma unroll
        for (int g = 0; g < NX / 4; ++g) {
            if constexpr (!kPF) {  // group g + 2 into the slot group g - 1 used (ResNet-50 512->512: -4 %)
                if (g + 2 < NX / 4) {
#pragma unroll
                    for (int x = 0; x < 4; ++x) bq[(g + 2) % 3][x] = b_at(NX * xs + 4 * (g + 2) + x, ks);
                }
            }
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const int xl = 4 * g + x, xi = NX * xs + xl;
                const f32x4 bv = kPF ? bcur[xl] : bq[g % 3][x];
#pragma unroll
                for (int h = 0; h < NB; ++h) {
                    const int ta = (16 * (th0 + h) + l16) ^ (2 * cm);
                    const f32x4 av = *reinterpret_cast<const f32x4 *>(vt + ((xi * 4 + cm) * 32 + ta) * 4);
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        acc[xl][h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[k], bv[k], acc[xl][h], 0, 0, 0);
                }
            }
        }
        if constexpr (kPF) {
#pragma unroll
            for (int x = 0; x < NBQ; ++x) bcur[x] = bnext[x];
        }
    }
    // m[xi][r]: accumulator row r (tile 16 (th0 + h) + 4 cm + r) of transform position xi.  XS = 2: the
    // sets swap halves so that set xs holds all 16 xi of rows r = 2 xs, 2 xs + 1.
    constexpr int NR = 4 / XS;  // accumulator rows finished per lane
    // slot: [set that receives][w4][h][xi 0..7][row 0..1][lane]
    auto slot = [&](int to, int h, int x, int rr) {
        return lds + ((((to * 4 + w4) * NB + h) * 8 + x) * 2 + rr) * 64 + lane;
    };
    if constexpr (XS == 2) {
        __syncthreads();  // every wave's MFMAs have read V
        auto send = [&](auto to_c) {
            constexpr int TO = decltype(to_c)::value;
#pragma unroll
            for (int h = 0; h < NB; ++h)
#pragma unroll
                for (int x = 0; x < 8; ++x)
#pragma unroll
                    for (int rr = 0; rr < 2; ++rr) *slot(TO, h, x, rr) = acc[x][h][2 * TO + rr];
        };
        if (xs == 0) send(WinoIC<1>{});
        else send(WinoIC<0>{});
        __syncthreads();
    }
    const float *__restrict__ rpre_p = a.res_pre;
    const float *__restrict__ rpost_p = a.res_post;
    const float *__restrict__ rfirst = rpre_p ? rpre_p : rpost_p;
    auto out_off = [&](int t, int q, int co, bool &ok) {
        const int ti = (t * mtc) >> 16, tj = t - ti * tc;
        const int oy = y0 + 2 * ti + (q >> 1), ox = x0 + 2 * tj + (q & 1);
        ok = t < ntiles && oy < a.H && ox < a.W;
        return (((size_t)img * a.H + oy) * a.W + ox) * a.Cpo + co;
    };
    const int co = nw + l16;
    const float sc = a.scale[co], sh = a.shift[co];
    auto finish = [&](auto xs_c) {
        constexpr int XSI = decltype(xs_c)::value;
        float m[16][NB][NR];
#pragma unroll
        for (int h = 0; h < NB; ++h)
#pragma unroll
            for (int rr = 0; rr < NR; ++rr)
#pragma unroll
                for (int x = 0; x < NX; ++x) {
                    m[NX * XSI + x][h][rr] = acc[x][h][NR * XSI + rr];
                    if constexpr (XS == 2) m[8 * (1 - XSI) + x][h][rr] = *slot(XSI, h, x, rr);
                }
#pragma unroll
        for (int h = 0; h < NB; ++h) {
            float rv[NR][4];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    bool ok;
                    const size_t off = out_off(16 * (th0 + h) + 4 * cm + NR * XSI + rr, q, co, ok);
                    rv[rr][q] = (rfirst && ok) ? rfirst[off] : 0.0f;
                }
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) {
                const int t = 16 * (th0 + h) + 4 * cm + NR * XSI + rr;
                float f[2][4];
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    f[0][s2] = (m[s2][h][rr] + m[4 + s2][h][rr]) + m[8 + s2][h][rr];
                    f[1][s2] = (m[4 + s2][h][rr] - m[8 + s2][h][rr]) - m[12 + s2][h][rr];
                }
                float pv[4];
                bool full = true;  // the tile's 2 x 2 outputs all inside the image: one max_pool2d(2, 2) window
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int dy = q >> 1, dx = q & 1;
                    bool ok;
                    const size_t off = out_off(t, q, co, ok);
                    full = full && ok;
                    float v = dx == 0 ? (f[dy][0] + f[dy][1]) + f[dy][2] : (f[dy][1] - f[dy][2]) - f[dy][3];
                    v = v * sc + sh;
                    if (rpre_p) v = v + rv[rr][q];
                    if (a.relu) v = fmaxf(v, 0.0f);
                    if (rpost_p) v = v + (rpre_p ? (ok ? rpost_p[off] : 0.0f) : rv[rr][q]);
                    pv[q] = v;
                    if (ok) a.out[off] = v;
                }
                if (a.pool && full) {  // F.max_pool2d's window order (fvp_maxpool_nhwc): NaN-propagating
                    const int ti = (t * mtc) >> 16, tj = t - ti * tc;
                    const int py = (y0 >> 1) + ti, pxo = (x0 >> 1) + tj;
                    a.pool[(((size_t)img * (a.H >> 1) + py) * (a.W >> 1) + pxo) * a.Cpo + co] =
                        nanmax(nanmax(nanmax(pv[0], pv[1]), pv[2]), pv[3]);
                }
            }
        }
    };
    if (xs == 0) finish(WinoIC<0>{});
    else if constexpr (XS == 2) finish(WinoIC<1>{});
}

// ---- ConvTranspose2d(4, 2, 1) by Winograd F(2x2, 2x2) per output parity ------
// (resnet.py:147-158, the PoseResNet deconvolution head.)  Output pixel
// (2y + ry, 2x + rx) = sum_{i,j in {0,1}} sum_ci W[ci][co][3-2i-ry][3-2j-rx]
// in[y - 1 + ry + i][x - 1 + rx + j]: for each parity class (ry, rx) a 2x2
// convolution over the input grid.  F(2x2, 2x2) takes a 3x3 input patch per
// 2x2 class-space tile: V = Bt d B with Bt = [[1,-1,0],[0,1,0],[0,-1,1]], U = G
// g Gt with G = [[1,0],[1,1],[0,1]], out = At M A with At = [[1,1,0],[0,1,1]]:
// 9 products per 4 outputs and input channel instead of 16 (1.78x fewer MFMA
// operations); every transform is exact sums and differences.  Same block
// shape as conv_wino_kernel (XS = 1): a TR x TC grid of tiles of one class of
// one image x 32 NB output channels, one block per (class, tile grid, column
// block); U in [class][9][Cpi/16][4][Cpo][4].
template <int NB>
__global__ __launch_bounds__(256, 2) void deconv_wino_kernel(WinoArgs a) {
    constexpr int NX = 9, NG = 3;  // transform positions; groups of <= 4 positions (4, 4, 1)
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *halo = lds, *vt = lds + kWinoHalo;
    const int tid = threadIdx.x, lane = tid & 63, w4 = tid >> 6;
    int bid = blockIdx.x;
    const int nblk = a.Cpo / (32 * NB);
    const int cbk = bid % nblk;
    bid /= nblk;
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    bid /= a.tiles_y;
    const int img = bid % a.N, cls = bid / a.N;
    const int ry = cls >> 1, rx = cls & 1;
    const int tr = a.tr, tc = a.tc, ntiles = tr * tc;
    const int hh = 2 * tr + 2, hw = 2 * tc + 2;
    const int mtc = 65536 / tc + 1, mhw = 65536 / hw + 1;  // exact multiply-shift quotients (conv_wino_kernel)
    const int y0 = ty * 2 * tr, x0 = tx * 2 * tc;          // class-space tile grid origin (input resolution)
    const int th0 = NB == 2 ? 0 : (w4 & 1);
    const int nw = cbk * 32 * NB + 16 * (NB == 2 ? w4 : (w4 >> 1));
    const float *__restrict__ src = a.in + (size_t)img * a.H * a.W * a.Cpi;
    const int ksteps = a.Cpi / 16;
    const int l16 = lane & 15, cm = lane >> 4;

    f32x4 acc[NX][NB];
#pragma unroll
    for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int h = 0; h < NB; ++h) acc[x][h] = f32x4{0.f, 0.f, 0.f, 0.f};

    constexpr int HU = (kWinoHaloPx * 4 + 255) / 256;
    const int hslots = hh * hw * 4;
    auto halo_load = [&](int ks, f32x4 (&hl)[HU]) {  // halo (r, c) <- input (y0 - 1 + ry + r, x0 - 1 + rx + c)
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            const int sl = tid + 256 * u;
            const int p = sl >> 2, q = sl & 3;
            const int hy = (p * mhw) >> 16, hx = p - hy * hw;
            const int gy = y0 - 1 + ry + hy, gx = x0 - 1 + rx + hx;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (sl < hslots && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)
                v = *reinterpret_cast<const f32x4 *>(src + ((size_t)gy * a.W + gx) * a.Cpi + ks * 16 + 4 * q);
            hl[u] = v;
        }
    };
    const float *__restrict__ ub = a.u + (size_t)cls * NX * ksteps * 16 * a.Cpo + ((size_t)cm * a.Cpo + nw + l16) * 4;
    auto b_at = [&](int xi, int ks) {
        return *reinterpret_cast<const f32x4 *>(ub + ((size_t)xi * ksteps + ks) * 16 * a.Cpo);
    };
    f32x4 bq[3][4];  // groups of 4 positions, two in flight
    f32x4 hnext[HU];
    halo_load(0, hnext);
    for (int ks = 0; ks < ksteps; ++ks) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            const int sl = tid + 256 * u;
            if (sl < hslots) *reinterpret_cast<f32x4 *>(halo + (sl >> 2) * kWinoHP + 4 * (sl & 3)) = hnext[u];
        }
        if (ks + 1 < ksteps) halo_load(ks + 1, hnext);
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            bq[0][x] = b_at(x, ks);
            bq[1][x] = b_at(4 + x, ks);
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < 2; ++it) {  // input transform: item = tile * 16 + c
            const int item = tid + 256 * it;
            const int t = item >> 4, c = item & 15;
            if (t < ntiles) {
                const int ti = (t * mtc) >> 16, tj = t - ti * tc;
                const float *hp = halo + ((2 * ti) * hw + 2 * tj) * kWinoHP + c;
                float d[3][3];
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int s2 = 0; s2 < 3; ++s2) d[r][s2] = hp[(r * hw + s2) * kWinoHP];
                float e[3][3];
#pragma unroll
                for (int s2 = 0; s2 < 3; ++s2) {
                    e[0][s2] = d[0][s2] - d[1][s2];
                    e[1][s2] = d[1][s2];
                    e[2][s2] = d[2][s2] - d[1][s2];
                }
                const int cmod = c & 3;
                float *vp = vt + (cmod * 32 + (t ^ (2 * cmod))) * 4 + (c >> 2);
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    vp[(r * 3 + 0) * 4 * 32 * 4] = e[r][0] - e[r][1];
                    vp[(r * 3 + 1) * 4 * 32 * 4] = e[r][1];
                    vp[(r * 3 + 2) * 4 * 32 * 4] = e[r][2] - e[r][1];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            if (g + 2 < NG) {
#pragma unroll
                for (int x = 0; x < 4; ++x)
                    if (4 * (g + 2) + x < NX) bq[(g + 2) % 3][x] = b_at(4 * (g + 2) + x, ks);
            }
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const int xi = 4 * g + x;
                if (xi >= NX) break;
                const f32x4 bv = bq[g % 3][x];
#pragma unroll
                for (int h = 0; h < NB; ++h) {
                    const int ta = (16 * (th0 + h) + l16) ^ (2 * cm);
                    const f32x4 av = *reinterpret_cast<const f32x4 *>(vt + ((xi * 4 + cm) * 32 + ta) * 4);
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        acc[xi][h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[k], bv[k], acc[xi][h], 0, 0, 0);
                }
            }
        }
    }
    // output transform and epilogue: lane holds tiles 16 (th0 + h) + 4 cm + r, column nw + l16
    const int Ho = 2 * a.H, Wo = 2 * a.W;
    const float *__restrict__ rpre_p = a.res_pre;
    const float *__restrict__ rpost_p = a.res_post;
    const int co = nw + l16;
    const float sc = a.scale[co], sh = a.shift[co];
#pragma unroll
    for (int h = 0; h < NB; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = 16 * (th0 + h) + 4 * cm + r;
            const int ti = (t * mtc) >> 16, tj = t - ti * tc;
            float f[2][3];
#pragma unroll
            for (int s2 = 0; s2 < 3; ++s2) {
                f[0][s2] = acc[s2][h][r] + acc[3 + s2][h][r];
                f[1][s2] = acc[3 + s2][h][r] + acc[6 + s2][h][r];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int dy = q >> 1, dx = q & 1;
                const int cy = y0 + 2 * ti + dy, cx = x0 + 2 * tj + dx;  // class-space position
                if (t >= ntiles || cy >= a.H || cx >= a.W) continue;
                const size_t off = (((size_t)img * Ho + 2 * cy + ry) * Wo + 2 * cx + rx) * a.Cpo + co;
                float v = f[dy][dx] + f[dy][dx + 1];
                v = v * sc + sh;
                if (rpre_p) v = v + rpre_p[off];
                if (a.relu) v = fmaxf(v, 0.0f);
                if (rpost_p) v = v + rpost_p[off];
                a.out[off] = v;
            }
        }
}

// Launch plan: the tile grid with the fewest 32-tile slots over the image (ties:
// fewer tiles past the image, then the wider grid), NB = 2 where Cpo % 64 == 0 unless that leaves
// fewer than 2 blocks per CU, XS = 2 where the launch still has at most one block per CU.
struct WinoPlan {
    int tr, tc, nb, xs;
    long long blocks;
};

static WinoPlan wino_plan(int N, int H, int W, int Cpo) {
    WinoPlan p{4, 8, 1, 1, 0};
    long long best = -1, best_cov = 0;
    const int ty = (H + 1) / 2, tx = (W + 1) / 2;  // Winograd tiles of the image
    for (int tr = 2; tr <= 16; ++tr)
        for (int tc = 2; tc <= 16; ++tc) {
            if (tr * tc > 32 || (2 * tr + 2) * (2 * tc + 2) > kWinoHaloPx) continue;
            const long long nblk = (long long)((ty + tr - 1) / tr) * ((tx + tc - 1) / tc);
            const long long slots = nblk * 32, covered = nblk * tr * tc;
            const bool better = best < 0 || slots < best ||
                                (slots == best && (covered < best_cov || (covered == best_cov && tc > p.tc)));
            if (better) {
                best = slots;
                best_cov = covered;
                p.tr = tr;
                p.tc = tc;
            }
        }
    const long long per_img = (long long)((ty + p.tr - 1) / p.tr) * ((tx + p.tc - 1) / p.tc);
    const long long b1 = (long long)N * per_img * (Cpo / 32);
    p.nb = (Cpo % 64 == 0 && b1 / 2 >= 512) ? 2 : 1;
    p.blocks = b1 / p.nb;
    p.xs = p.blocks <= 256 ? 2 : 1;  // (thresholds 512 / 1024 measured slower: CenterNet 80^2, 400 blocks, 14.8 -> 18.4 us)
    return p;
}

}  // namespace fvp

extern "C" int fvp_conv3x3_wino_plan(int N, int H, int W, int Cpo, int *plan) {
    if (!plan) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || Cpo <= 0 || Cpo % 32) return FVP_ERR_SHAPE;
    const fvp::WinoPlan p = fvp::wino_plan(N, H, W, Cpo);
    const long long covered = (long long)((((H + 1) / 2) + p.tr - 1) / p.tr) * p.tr * 2 *
                              ((((W + 1) / 2) + p.tc - 1) / p.tc) * p.tc * 2;
    plan[0] = p.tr;
    plan[1] = p.tc;
    plan[2] = p.nb;
    plan[3] = p.xs;
    plan[4] = (int)((p.blocks > 0x7fffffffLL) ? 0x7fffffff : p.blocks);
    // slot coverage: 1000 x (32-tile slots x 4 px) / (H x W)
    plan[5] = (int)(1000 * ((covered / (4LL * p.tr * p.tc)) * 32 * 4) / ((long long)H * W));
    return FVP_OK;
}

extern "C" int fvp_conv3x3_wino_nhwc(const float *in, int N, int H, int W, int Cpi, const float *u, int Cpo,
                                     const float *scale, const float *shift, const float *res_pre,
                                     const float *res_post, int relu, float *out, float *pool, void *stream) {
    if (!in || !u || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || Cpi <= 0 || Cpi % 16 || Cpo <= 0 || Cpo % 32) return FVP_ERR_SHAPE;
    const fvp::WinoPlan p = fvp::wino_plan(N, H, W, Cpo);
    if (p.blocks > 0x7fffffffLL) return FVP_ERR_SHAPE;
    fvp::WinoArgs a{in, u, scale, shift, res_pre, res_post, out, pool, N, H, W, Cpi, Cpo, relu, p.tr, p.tc,
                    (H + 2 * p.tr - 1) / (2 * p.tr), (W + 2 * p.tc - 1) / (2 * p.tc)};
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)p.blocks);
    auto go = [&](auto kernel, int nb, int xs) {
        hipLaunchKernelGGL(kernel, grid, dim3(256 * xs), (size_t)fvp::wino_lds_floats(nb, xs) * sizeof(float), s, a);
    };
    if (p.nb == 2)  // (NB = 2 implies >= 512 blocks, so XS = 1)
        go(fvp::conv_wino_kernel<2, 1>, 2, 1);
    else if (p.xs == 2)
        go(fvp::conv_wino_kernel<1, 2>, 1, 2);
    else
        go(fvp::conv_wino_kernel<1, 1>, 1, 1);
    return (int)hipGetLastError();
}

extern "C" int fvp_deconv4s2_wino_nhwc(const float *in, int N, int H, int W, int Cpi, const float *u, int Cpo,
                                       const float *scale, const float *shift, const float *res_pre,
                                       const float *res_post, int relu, float *out, void *stream) {
    if (!in || !u || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || Cpi <= 0 || Cpi % 16 || Cpo <= 0 || Cpo % 32) return FVP_ERR_SHAPE;
    const fvp::WinoPlan p = fvp::wino_plan(N, H, W, Cpo);  // the class-space tile grid (one class's outputs)
    const long long blocks = 4 * p.blocks;  // x 4 parity classes
    if (blocks > 0x7fffffffLL) return FVP_ERR_SHAPE;
    fvp::WinoArgs a{in, u, scale, shift, res_pre, res_post, out, nullptr, N, H, W, Cpi, Cpo, relu, p.tr, p.tc,
                    (H + 2 * p.tr - 1) / (2 * p.tr), (W + 2 * p.tc - 1) / (2 * p.tc)};
    hipStream_t s = (hipStream_t)stream;
    const size_t lds = (size_t)fvp::wino_lds_floats(1, 1) * sizeof(float);
    if (p.nb == 2)
        hipLaunchKernelGGL(fvp::deconv_wino_kernel<2>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL(fvp::deconv_wino_kernel<1>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    return (int)hipGetLastError();
}
