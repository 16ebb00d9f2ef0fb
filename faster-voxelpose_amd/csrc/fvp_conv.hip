// Dense 2-D convolutions on the fp32 matrix cores: the HDN / JLN CNNs
// (CenterNet cnns_2d.py:235-295, P2PNet :185-232,
// their Basic2DBlock / Res2DBlock / Upsample2DBlock / EncoderDecorder parts
// :12-183, WeightNet's convolution, weight_net.py:48-80) and the PoseResNet
// heatmap backbone (§8(f) rank 4: resnet.py:98-201 -- strided 7x7 / 3x3 / 1x1
// convolutions and the ConvTranspose2d(4, 2, 1) deconvolution head).
//
// Implicit GEMM, NHWC fp32 activations with channels padded to a multiple of
// 16 (or 4 / 8 for a network's RGB input; padding channels hold zeros),
// out[m][co] = sum_k A[m][k] W[k][co] with m = (image, y, x) and
// k = (ky*KW + kx)*Cpi + ci.  v_mfma_f32_32x32x2_f32 is an exact fp32 fma
// chain, so the only difference from torch's fp32 conv is the summation
// order.  Eval-mode BatchNorm is folded into a per-channel scale/shift (with
// the conv bias), and the epilogue fuses the residual add of Res2DBlock /
// Bottleneck (before the ReLU), the ReLU, the decoder's skip add (after the
// ReLU) and the output scatter of the transposed convolutions:
//   mode 1  ConvTranspose2d(k=2, s=2): a 1x1 conv producing 4*Cout channels
//   mode 2  ConvTranspose1d(k=2, s=2): the same with 2*Cout on rows of H == 1
//   mode 3  ConvTranspose2d(k=4, s=2, p=1): four 2x2 convolutions over the
//           input grid, one per output parity (ry, rx) -- output pixel
//           (2y+ry, 2x+rx) takes input rows y-1+ry.. and kernel taps
//           ky = 3 - 2*i - ry (i = 0, 1) -- so no MFMA work is spent on the
//           zeros a dilated-input formulation would multiply.
//
// Block = 256 threads (4 waves); the tile follows the output width so no MFMA
// column is wasted on padding: Cout <= 16 -> 256 px x 16 ch on 16x16x4 MFMAs,
// <= 32 -> 128 x 32, wider -> 128 x 64 (2 accumulators per wave) on 32x32x2.
// The K dimension is walked in chunks of 16 (one (ky,kx) tap, 16 input
// channels; with Cpi < 16 a chunk spans 16/Cpi taps) staged through LDS, the
// next chunk's global loads issued before the current chunk's MFMAs.
#include <type_traits>

#include "fvp_layout.h"  // fvp_device.h, buffer descriptors (uniform_rsrc, kOOB)

namespace fvp {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct ConvArgs {
    const float *in;        // [N][H][W][Cpi]
    const float *w;         // [G][Krows][Cpo_w], Krows = KH*KW*Cpi rounded up to 16 (zero rows), G parity groups
    const float *scale;     // [Cpo]  (per output channel)
    const float *shift;     // [Cpo]
    const float *res_pre;   // [N][Ho][Wo][Cpo] or null: added before the ReLU
    const float *res_post;  // [N][Ho][Wo][Cpo] or null: added after the ReLU
    float *out;             // [N][Ho][Wo][Cpo]
    int N, H, W, Cpi, KH, KW, Cpo, Cpo_w, relu, up2;  // up2 = mode (0 conv, 1-3 transposed, see above)
    int Hm, Wm;             // GEMM row grid: output pixels (mode 0) or input pixels (modes 1-3)
    int sy, sx, py, px;     // stride and top/left zero padding: input = row * s - p + tap
    int ks;                 // split-K blocks per parity group (gridDim.z = groups * ks)
    float *part;            // split-K: raw partial sums [gridDim.z][M][Ntot] (no epilogue), else null
    int in_bf16, out_bf16;  // bf16 kernel only: activations (in; out + residuals) stored as bf16
};

__host__ __device__ __forceinline__ int conv_groups(int up2) { return up2 == 3 ? 4 : 1; }
__host__ __device__ __forceinline__ int conv_cols(int up2, int Cpo) {  // GEMM columns per group
    return (up2 == 1 ? 4 : up2 == 2 ? 2 : 1) * Cpo;
}
__host__ __device__ __forceinline__ int conv_krows(int KH, int KW, int Cpi) { return (KH * KW * Cpi + 15) & ~15; }

// Tile configuration: BM pixels x BN channels per 256-thread block, MFMA
// MSxMS (32: v_mfma_f32_32x32x2_f32, 16: v_mfma_f32_16x16x4_f32), waves
// arranged WR x WC, each wave TM x TN MFMA tiles; K chunks of KC (one tap).
template <int BM_, int BN_, int MS_, int WR_, int KC_ = 16>
struct Tile {
    static constexpr int BM = BM_, BN = BN_, MS = MS_, WR = WR_, WC = 4 / WR_;
    static constexpr int WTM = BM / WR, WTN = BN / WC;  // wave tile
    static constexpr int TM = WTM / MS, TN = WTN / MS;
    static constexpr int KC = KC_, AP = KC + 1;
    static constexpr int KSTEP = MS == 32 ? 2 : 4;      // k per MFMA
    static constexpr int NACC = MS == 32 ? 16 : 4;      // accumulator registers per MFMA tile
    static_assert(TM >= 1 && TN >= 1 && WTM % MS == 0 && WTN % MS == 0, "tile");
};

// Per-thread A rows (pixels) are fixed for the whole K loop: their image and
// input origin (row * stride - pad) are decoded once, so a chunk only adds
// the tap offset.
struct PixRef {
    int y, x;         // input coordinates of tap (0, 0) (y = -1 << 20 when past M)
    const float *p;   // input row base of the pixel's image
};

__device__ __forceinline__ void pix_ref(const ConvArgs &a, int m, int M, int py, int px, PixRef &pr) {
    const int HWm = a.Hm * a.Wm;
    const int img = m / HWm, r = m - img * HWm;
    const int yy = r / a.Wm, xx = r - (r / a.Wm) * a.Wm;
    pr.y = m < M ? yy * a.sy - py : -(1 << 20);
    pr.x = xx * a.sx - px;
    pr.p = a.in + (size_t)(m < M ? img : 0) * a.H * a.W * a.Cpi;
}

template <class TL>
__device__ __forceinline__ void load_chunk(const ConvArgs &a, const float *__restrict__ w, int n0, int chunk,
                                           const PixRef *pr, float4 *av, float4 *bv) {
    constexpr int AE = TL::BM * TL::KC / 4;        // float4 of the A chunk
    constexpr int AV = AE >= 256 ? AE / 256 : 1;   // per thread
    constexpr int BV = TL::KC * TL::BN / 4 / 256;  // float4 per thread (B), may be 0
    const int t = threadIdx.x;
    constexpr int Q = TL::KC / 4;                  // float4 per pixel row of a chunk
    if (a.Cpi >= TL::KC) {  // one tap per chunk (Cpi % KC == 0)
        const int cpc = a.Cpi / TL::KC;  // chunks per tap
        const int tap = chunk / cpc, c = chunk - tap * cpc;
        const int ky = tap / a.KW, kx = tap - ky * a.KW;
#pragma unroll
        for (int u = 0; u < AV; ++u) {
            const int e = u * 256 + t;  // -> (pixel e/Q, 4 channels)
            const int y = pr[u].y + ky, x = pr[u].x + kx;
            av[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < AE && (unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W)
                av[u] = *reinterpret_cast<const float4 *>(pr[u].p + ((size_t)y * a.W + x) * a.Cpi + c * TL::KC +
                                                         (e % Q) * 4);
        }
    } else {  // Cpi < KC (4 / 8 / 12 at KC = 16): each float4 is 4 channels of its own tap; k past the taps reads 0
        const int ntaps = a.KH * a.KW;
#pragma unroll
        for (int u = 0; u < AV; ++u) {
            const int e = u * 256 + t;
            const int k = chunk * TL::KC + (e % Q) * 4;
            const int tap = k / a.Cpi, ci = k - tap * a.Cpi;
            const int ky = tap / a.KW, kx = tap - ky * a.KW;
            const int y = pr[u].y + ky, x = pr[u].x + kx;
            av[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < AE && tap < ntaps && (unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W)
                av[u] = *reinterpret_cast<const float4 *>(pr[u].p + ((size_t)y * a.W + x) * a.Cpi + ci);
        }
    }
    if constexpr (BV > 0) {
#pragma unroll
        for (int u = 0; u < BV; ++u) {
            const int e = u * 256 + t;  // -> (k row e/(BN/4), 4 columns)
            const size_t row = (size_t)chunk * TL::KC + e / (TL::BN / 4);
            bv[u] = *reinterpret_cast<const float4 *>(w + row * a.Cpo_w + n0 + (e % (TL::BN / 4)) * 4);
        }
    } else {  // BN*KC/4 < 256: the first KC*BN/4 threads load one float4
        if (t < TL::KC * TL::BN / 4) {
            const size_t row = (size_t)chunk * TL::KC + t / (TL::BN / 4);
            bv[0] = *reinterpret_cast<const float4 *>(w + row * a.Cpo_w + n0 + (t % (TL::BN / 4)) * 4);
        }
    }
}

// Output element of GEMM row m (a pixel of the row grid), column n, parity
// group g: mode 0 the pixel itself; modes 1-3 the scattered pixel of the
// upsampled output.  co receives the output channel.
__device__ __forceinline__ size_t conv_out_offset(const ConvArgs &a, int m, int n, int g, int &co) {
    if (!a.up2) {
        co = n;
        return (size_t)m * a.Cpo + n;
    }
    const int q = a.up2 == 3 ? g : n / a.Cpo;  // (dy, dx) of the transposed conv
    co = a.up2 == 3 ? n : n - q * a.Cpo;
    const int HWm = a.Hm * a.Wm;
    const int img = m / HWm, rr = m - img * HWm;
    const int yy = rr / a.Wm, xx = rr - yy * a.Wm;
    const int Ho = a.up2 == 2 ? a.Hm : 2 * a.Hm, Wo = 2 * a.Wm;
    const int y = a.up2 == 2 ? yy : 2 * yy + (q >> 1);
    const int x = 2 * xx + (a.up2 == 2 ? q : (q & 1));
    return (((size_t)img * Ho + y) * Wo + x) * a.Cpo + co;
}

// Fused epilogue: out = act(acc * scale + shift + res_pre) + res_post at the
// output offset of (row m, column n), bf16 or fp32 output (BFO && a.out_bf16).
// The block's BM x BN accumulator tile is staged through LDS (cs: >= BM *
// (BN + 4) floats, free after the K loop), then each thread writes
// (pixel, 8 output channels) units with 16-B vector loads and stores.  (A
// lane-per-channel epilogue straight from the MFMA registers issues 2-4 B per
// lane: the wide 1x1 "expand" convolutions and their residual reads ran at
// ~1.4 TB/s; bf16 ResNet-50 19.0 -> 14.6 ms, P2PNet 1.89 -> 1.78 ms.)
template <int BM, int BN, bool BFO, typename RowM, int NT = 256>
__device__ __forceinline__ void epilogue_write(const ConvArgs &a, const RowM &rowm, int n0, int g, const float *cs);

template <int BM, int BN, int TM, int TN, int NACC, int MS, bool BFO, typename AccT, typename RowM>
__device__ __forceinline__ void epilogue_staged(const ConvArgs &a, const AccT (&acc)[TM][TN], const RowM &rowm,
                                                int mw, int nwl, int n0, int lane, int g, float *cs) {
    constexpr int CP = BN + 4;  // row pitch (floats): 16-B aligned rows
    auto rowof = [&](int r) { return MS == 32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : (lane >> 4) * 4 + r; };
    __syncthreads();  // every wave is past its last LDS read of the K loop
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < NACC; ++r)
                cs[(mw + i * MS + rowof(r)) * CP + nwl + j * MS + (lane % MS)] = acc[i][j][r];
    __syncthreads();
    epilogue_write<BM, BN, BFO>(a, rowm, n0, g, cs);
}

// The write half: each thread takes (pixel, 8 output channels) units of the
// staged [BM][BN + 4] fp32 tile; a thread's units share one channel group
// (NT % (BN / 8) == 0), so its scale / shift are loaded once.  NT: threads per block.
template <int BM, int BN, bool BFO, typename RowM, int NT>
__device__ __forceinline__ void epilogue_write(const ConvArgs &a, const RowM &rowm, int n0, int g, const float *cs) {
    constexpr int CP = BN + 4;
    constexpr int G = BN / 8;  // 8-channel groups per row
    static_assert(NT % G == 0, "one channel group per thread");
    const bool bfo = BFO && a.out_bf16;
    const int Ctot = conv_cols(a.up2, a.Cpo);
    const int cg = threadIdx.x % G;
    const int n = n0 + cg * 8;
    if (n >= Ctot) return;  // Ctot is a multiple of 16: whole groups
    const int co = (a.up2 == 1 || a.up2 == 2) ? n % a.Cpo : n;
    const float4 s0 = *reinterpret_cast<const float4 *>(a.scale + co);
    const float4 s1 = *reinterpret_cast<const float4 *>(a.scale + co + 4);
    const float4 h0 = *reinterpret_cast<const float4 *>(a.shift + co);
    const float4 h1 = *reinterpret_cast<const float4 *>(a.shift + co + 4);
    // all of this thread's units' output offsets and residual loads are issued
    // before the first is used (a unit-by-unit loop exposed one global round
    // trip per unit: the wide 1x1 "expand" layers are output / residual bound)
    constexpr int U = (BM * G + NT - 1) / NT;  // units per thread (the last may be past the tile: BM * G < NT)
    size_t off[U];
    bool ok[U];
    uint4 rpre[U][2], rpost[U][2];  // 8 channels: bf16 in [0], fp32 in [0..1]
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int row = threadIdx.x / G + u * (NT / G);
        const int m = row < BM ? rowm(row) : -1;
        ok[u] = m >= 0;
        int co_;
        off[u] = conv_out_offset(a, ok[u] ? m : rowm(0), n, g, co_);  // 8 consecutive output channels from off
    }
    auto load8 = [&](const float *base, size_t o, uint4 (&r)[2]) {
        if (bfo) {
            r[0] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const __bf16 *>(base) + o);
        } else {
            r[0] = *reinterpret_cast<const uint4 *>(base + o);
            r[1] = *reinterpret_cast<const uint4 *>(base + o + 4);
        }
    };
    auto unpack8 = [&](const uint4 (&r)[2], float (&o)[8]) {
        if (bfo) {
            const unsigned w4[4] = {r[0].x, r[0].y, r[0].z, r[0].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                o[2 * k] = __builtin_bit_cast(float, w4[k] << 16);
                o[2 * k + 1] = __builtin_bit_cast(float, w4[k] & 0xffff0000u);
            }
        } else {
            const unsigned w8[8] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w};
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = __builtin_bit_cast(float, w8[k]);
        }
    };
    if (a.res_pre) {
#pragma unroll
        for (int u = 0; u < U; ++u) load8(a.res_pre, off[u], rpre[u]);
    }
    if (a.res_post) {
#pragma unroll
        for (int u = 0; u < U; ++u) load8(a.res_post, off[u], rpost[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int row = min(threadIdx.x / G + u * (NT / G), BM - 1);
        const float4 c0 = *reinterpret_cast<const float4 *>(cs + row * CP + cg * 8);
        const float4 c1 = *reinterpret_cast<const float4 *>(cs + row * CP + cg * 8 + 4);
        float v[8] = {c0.x * s0.x + h0.x, c0.y * s0.y + h0.y, c0.z * s0.z + h0.z, c0.w * s0.w + h0.w,
                      c1.x * s1.x + h1.x, c1.y * s1.y + h1.y, c1.z * s1.z + h1.z, c1.w * s1.w + h1.w};
        if (a.res_pre) {
            float r8[8];
            unpack8(rpre[u], r8);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = v[k] + r8[k];
        }
        if (a.relu) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.0f);
        }
        if (a.res_post) {
            float r8[8];
            unpack8(rpost[u], r8);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = v[k] + r8[k];
        }
        if (!ok[u]) continue;
        if (bfo) {
            unsigned w4[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                w4[k] = (unsigned)__builtin_bit_cast(unsigned short, (__bf16)v[2 * k]) |
                        ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)v[2 * k + 1]) << 16);
            *reinterpret_cast<uint4 *>(reinterpret_cast<__bf16 *>(a.out) + off[u]) =
                make_uint4(w4[0], w4[1], w4[2], w4[3]);
        } else {
            *reinterpret_cast<float4 *>(a.out + off[u]) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<float4 *>(a.out + off[u] + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
    }
}

// Output tile of this workgroup.  Workgroups are dealt round robin over the 8
// XCDs (each with its own L2): the dispatch index is regrouped so that every
// XCD gets a contiguous run of logical tiles, and the logical order walks the
// column tiles of one row tile together, so a row tile's activations come from
// HBM once and from that XCD's L2 for its other column tiles (a 2-D grid in
// hardware order re-read them from HBM once per column tile).
__device__ __forceinline__ void conv_tile(int &mt, int &nt) {
    const unsigned T = gridDim.x * gridDim.y, lin = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned q = T >> 3, r = T & 7, x = lin & 7, loc = lin >> 3;
    const unsigned id = x < r ? x * (q + 1) + loc : r * (q + 1) + (x - r) * q + loc;
    nt = (int)(id % gridDim.y);
    mt = (int)(id / gridDim.y);
}

template <class TL, int PF = 1>
__global__ __launch_bounds__(256, 4) void conv_mfma_kernel(ConvArgs a) {
    constexpr int BM = TL::BM, BN = TL::BN, KC = TL::KC, AP = TL::AP, MS = TL::MS;
    constexpr int AE = BM * KC / 4;
    constexpr int AV = AE >= 256 ? AE / 256 : 1;
    constexpr int BVN = KC * BN / 4 / 256 > 0 ? KC * BN / 4 / 256 : 1;
    constexpr int KLDS = 2 * BM * AP + 2 * KC * BN, CLDS = BM * (BN + 4);  // K loop / staged epilogue
    __shared__ __attribute__((aligned(16))) float smem[KLDS > CLDS ? KLDS : CLDS];
    float (*As)[BM * AP] = reinterpret_cast<float (*)[BM * AP]>(smem);
    float (*Bs)[KC * BN] = reinterpret_cast<float (*)[KC * BN]>(smem + 2 * BM * AP);
    const int M = a.N * a.Hm * a.Wm;
    int mt, nt;
    conv_tile(mt, nt);
    const int m0 = mt * BM, n0 = nt * BN;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wr = wave % TL::WR, wc = wave / TL::WR;
    const int g = blockIdx.z / a.ks, kz = blockIdx.z - g * a.ks;  // parity group, split-K slice
    const int nchunks = conv_krows(a.KH, a.KW, a.Cpi) / KC;
    // split-K: slice kz walks chunks [cb, ce) and leaves raw partial sums
    const int cb = (int)((long long)kz * nchunks / a.ks);
    const int ce = (int)((long long)(kz + 1) * nchunks / a.ks);
    const float *__restrict__ w = a.w + (size_t)g * nchunks * KC * a.Cpo_w;
    const int py = a.up2 == 3 ? 1 - (g >> 1) : a.py, px = a.up2 == 3 ? 1 - (g & 1) : a.px;
    using acc_t = typename std::conditional<MS == 32, f32x16, f32x4>::type;
    acc_t acc[TL::TM][TL::TN];
#pragma unroll
    for (int i = 0; i < TL::TM; ++i)
#pragma unroll
        for (int j = 0; j < TL::TN; ++j)
#pragma unroll
            for (int r = 0; r < TL::NACC; ++r) acc[i][j][r] = 0.f;

    PixRef pr[AV];
#pragma unroll
    for (int u = 0; u < AV; ++u) pix_ref(a, m0 + (u * 256 + t) / (KC / 4), M, py, px, pr[u]);
    using AReg = float4[AV];
    using BReg = float4[BVN];
    auto stage = [&](int buf, const AReg &av, const BReg &bv) {  // registers -> LDS buffer buf
#pragma unroll
        for (int u = 0; u < AV; ++u) {
            const int e = u * 256 + t;
            if (e >= AE) break;
            float *ap = &As[buf][(e / (KC / 4)) * AP + (e % (KC / 4)) * 4];
            ap[0] = av[u].x; ap[1] = av[u].y; ap[2] = av[u].z; ap[3] = av[u].w;
        }
        if constexpr (KC * BN / 4 >= 256) {
#pragma unroll
            for (int u = 0; u < BVN; ++u) {
                const int e = u * 256 + t;
                *reinterpret_cast<float4 *>(&Bs[buf][(e / (BN / 4)) * BN + (e % (BN / 4)) * 4]) = bv[u];
            }
        } else if (t < KC * BN / 4) {
            *reinterpret_cast<float4 *>(&Bs[buf][(t / (BN / 4)) * BN + (t % (BN / 4)) * 4]) = bv[0];
        }
    };
    auto mfma = [&](int buf) {
#pragma unroll
        for (int kk = 0; kk < KC / TL::KSTEP; ++kk) {
            float fa[TL::TM], fb[TL::TN];
#pragma unroll
            for (int i = 0; i < TL::TM; ++i) {
                const int row = wr * TL::WTM + i * MS + (lane % MS);
                fa[i] = As[buf][row * AP + kk * TL::KSTEP + lane / MS];
            }
#pragma unroll
            for (int j = 0; j < TL::TN; ++j) {
                const int col = wc * TL::WTN + j * MS + (lane % MS);
                fb[j] = Bs[buf][(kk * TL::KSTEP + lane / MS) * BN + col];
            }
#pragma unroll
            for (int i = 0; i < TL::TM; ++i)
#pragma unroll
                for (int j = 0; j < TL::TN; ++j) {
                    if constexpr (MS == 32)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
                    else
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
                }
        }
    };
    float4 av[AV], bv[BVN];
    load_chunk<TL>(a, w, n0, cb, pr, av, bv);
    stage(cb & 1, av, bv);
    if constexpr (PF == 1) {
        __syncthreads();
        // One barrier per chunk: chunk ch+1's global loads are issued first, the
        // MFMAs of chunk ch next, and the loaded registers go to the other buffer
        // after the last MFMA has issued (it was last read before the previous
        // barrier), so the LDS stores and the barrier overlap the MFMA tail.
        for (int ch = cb; ch < ce; ++ch) {
            const bool more = ch + 1 < ce;
            if (more) load_chunk<TL>(a, w, n0, ch + 1, pr, av, bv);
            mfma(ch & 1);
            if (more) stage((ch & 1) ^ 1, av, bv);
            __syncthreads();
        }
    } else {
        // Two chunks in flight: chunk ch+2 is loaded into the register set that
        // chunk ch came through while chunk ch+1's registers (loaded one
        // iteration earlier) go to LDS -- a global round trip per two chunks of
        // MFMA work instead of one (the short-K-walk small tiles).
        float4 av2[AV], bv2[BVN];
        if (cb + 1 < ce) load_chunk<TL>(a, w, n0, cb + 1, pr, av2, bv2);
        __syncthreads();
        auto step = [&](int ch, AReg &la, BReg &lb, const AReg &sa, const BReg &sb) {
            if (ch + 2 < ce) load_chunk<TL>(a, w, n0, ch + 2, pr, la, lb);
            mfma(ch & 1);
            if (ch + 1 < ce) stage((ch & 1) ^ 1, sa, sb);
            __syncthreads();
        };
        for (int ch = cb; ch < ce; ch += 2) {
            step(ch, av, bv, av2, bv2);
            if (ch + 1 < ce) step(ch + 1, av2, bv2, av, bv);
        }
    }

    if (a.part) {  // split-K: raw partial sums, combined in z order by conv_splitk_reduce
        const int Ntot = conv_cols(a.up2, a.Cpo);
        float *__restrict__ dst = a.part + (size_t)blockIdx.z * M * Ntot;
#pragma unroll
        for (int j = 0; j < TL::TN; ++j) {
            const int n = n0 + wc * TL::WTN + j * MS + (lane % MS);
#pragma unroll
            for (int i = 0; i < TL::TM; ++i)
#pragma unroll
                for (int r = 0; r < TL::NACC; ++r) {
                    const int row = MS == 32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : (lane >> 4) * 4 + r;
                    const int m = m0 + wr * TL::WTM + i * MS + row;
                    if (m < M && n < Ntot) dst[(size_t)m * Ntot + n] = acc[i][j][r];
                }
        }
        return;
    }
    // epilogue: lane -> column (output channel), registers -> rows (pixels)
    auto rowm = [&](int l) { return m0 + l < M ? m0 + l : -1; };
    epilogue_staged<BM, BN, TL::TM, TL::TN, TL::NACC, MS, false>(a, acc, rowm, wr * TL::WTM, wc * TL::WTN, n0, lane,
                                                                g, smem);
}

// Split-K combine: out = act(sum_z part[z] * scale + shift + res_pre) + res_post,
// the ks slices of each parity group summed in z order (deterministic), with
// the epilogue's output mapping.
__global__ __launch_bounds__(256) void conv_splitk_reduce(ConvArgs a, int M, int Ntot) {
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long per = (long long)M * Ntot;
    if (e >= per * conv_groups(a.up2)) return;
    const int g = (int)(e / per);
    const long long r = e - g * per;
    const int m = (int)(r / Ntot), n = (int)(r - (long long)m * Ntot);
    float v = 0.0f;
    for (int z = 0; z < a.ks; ++z) v += a.part[((size_t)(g * a.ks + z) * M + m) * Ntot + n];
    int co;
    const size_t off = conv_out_offset(a, m, n, g, co);
    v = v * a.scale[co] + a.shift[co];
    if (a.res_pre) v = v + a.res_pre[off];
    if (a.relu) v = fmaxf(v, 0.0f);
    if (a.res_post) v = v + a.res_post[off];
    a.out[off] = v;
}

// Halo-tiled variant for KxK (K > 1) stride-1 "same" convolutions on images
// at least 16 pixels wide.  A block owns a TH x 16 tile of output pixels of
// one image (TH = BM / 16); per 16-channel chunk the (TH+KH-1) x (16+KW-1)
// input halo is staged into LDS once and serves every (ky, kx) tap, where the
// per-tap implicit-im2col loads of conv_mfma_kernel re-read each input pixel
// up to KH*KW times (10-26 % of a layer's time, profiles/round1/conv_probe.txt).  The K
// loop walks channel chunks outer and taps inner; the per-tap weight tiles are
// double-buffered and prefetched one step ahead as in conv_mfma_kernel, the
// next chunk's halo is loaded into registers during the current chunk's taps.
template <class TL, int KMAX>
__global__ __launch_bounds__(256, 4) void conv_halo_kernel(ConvArgs a, int tiles_x, int tiles_y) {
    constexpr int BM = TL::BM, BN = TL::BN, KC = TL::KC, AP = TL::AP, MS = TL::MS;
    constexpr int TW = 16, TH = BM / TW;
    constexpr int HMAX = (TH + KMAX - 1) * (TW + KMAX - 1);  // halo pixels at the largest kernel
    constexpr int HV = (HMAX * (KC / 4) + 255) / 256;         // halo float4 per thread
    constexpr int BVN = KC * BN / 4 / 256 > 0 ? KC * BN / 4 / 256 : 1;
    static_assert(BM % TW == 0 && KC == 16, "halo tile");
    constexpr int HLDS = ((HMAX * AP + 3) & ~3) + 2 * KC * BN, CLDS = BM * (BN + 4);  // K loop / staged epilogue
    __shared__ __attribute__((aligned(16))) float smem[HLDS > CLDS ? HLDS : CLDS];
    float *Hs = smem;
    float (*Bs)[KC * BN] = reinterpret_cast<float (*)[KC * BN]>(smem + ((HMAX * AP + 3) & ~3));
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wr = wave % TL::WR, wc = wave / TL::WR;
    const int per_img = tiles_x * tiles_y;
    int mt, nt;
    conv_tile(mt, nt);
    const int img = mt / per_img, tr = mt - img * per_img;
    const int y0 = (tr / tiles_x) * TH, x0 = (tr - (tr / tiles_x) * tiles_x) * TW;
    const int n0 = nt * BN;
    const int HWd = TW + a.KW - 1, HP = (TH + a.KH - 1) * HWd;
    const int hy0 = y0 - (a.KH - 1) / 2, hx0 = x0 - (a.KW - 1) / 2;
    const float *__restrict__ inimg = a.in + (size_t)img * a.H * a.W * a.Cpi;
    const int ntaps = a.KH * a.KW, ncc = a.Cpi / KC, nsteps = ntaps * ncc;
    using acc_t = typename std::conditional<MS == 32, f32x16, f32x4>::type;
    acc_t acc[TL::TM][TL::TN];
#pragma unroll
    for (int i = 0; i < TL::TM; ++i)
#pragma unroll
        for (int j = 0; j < TL::TN; ++j)
#pragma unroll
            for (int r = 0; r < TL::NACC; ++r) acc[i][j][r] = 0.f;

    float4 hv[HV], bv[BVN];
    auto load_halo = [&](int cc) {  // element e -> (halo pixel e/4, 4 channels)
#pragma unroll
        for (int u = 0; u < HV; ++u) {
            const int e = u * 256 + t, hp = e >> 2;
            hv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (hp < HP) {
                const int hy = hp / HWd, hx = hp - hy * HWd;
                const int y = hy0 + hy, x = hx0 + hx;
                if ((unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W)
                    hv[u] = *reinterpret_cast<const float4 *>(inimg + ((size_t)y * a.W + x) * a.Cpi + cc * KC +
                                                             (e & 3) * 4);
            }
        }
    };
    auto store_halo = [&]() {
#pragma unroll
        for (int u = 0; u < HV; ++u) {
            const int e = u * 256 + t, hp = e >> 2;
            if (hp < HP) {
                float *d = &Hs[hp * AP + (e & 3) * 4];
                d[0] = hv[u].x; d[1] = hv[u].y; d[2] = hv[u].z; d[3] = hv[u].w;
            }
        }
    };
    auto load_b = [&](int step) {  // weight rows of (tap, chunk) -> bv
        const int cc = step / ntaps, tap = step - cc * ntaps;
        const size_t row0 = (size_t)tap * a.Cpi + cc * KC;
        if constexpr (KC * BN / 4 >= 256) {
#pragma unroll
            for (int u = 0; u < BVN; ++u) {
                const int e = u * 256 + t;
                bv[u] = *reinterpret_cast<const float4 *>(a.w + (row0 + e / (BN / 4)) * a.Cpo_w + n0 +
                                                         (e % (BN / 4)) * 4);
            }
        } else if (t < KC * BN / 4) {
            bv[0] = *reinterpret_cast<const float4 *>(a.w + (row0 + t / (BN / 4)) * a.Cpo_w + n0 + (t % (BN / 4)) * 4);
        }
    };
    auto store_b = [&](int buf) {
        if constexpr (KC * BN / 4 >= 256) {
#pragma unroll
            for (int u = 0; u < BVN; ++u) {
                const int e = u * 256 + t;
                *reinterpret_cast<float4 *>(&Bs[buf][(e / (BN / 4)) * BN + (e % (BN / 4)) * 4]) = bv[u];
            }
        } else if (t < KC * BN / 4) {
            *reinterpret_cast<float4 *>(&Bs[buf][(t / (BN / 4)) * BN + (t % (BN / 4)) * 4]) = bv[0];
        }
    };
    // halo pixel of each of this lane's A rows at tap (0, 0)
    int hrow[TL::TM];
#pragma unroll
    for (int i = 0; i < TL::TM; ++i) {
        const int l = wr * TL::WTM + i * MS + (lane % MS);
        hrow[i] = (l / TW) * HWd + (l % TW);
    }
    load_halo(0);
    load_b(0);
    store_halo();
    store_b(0);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        const int cc = s / ntaps, tap = s - cc * ntaps;
        const int buf = s & 1;
        const bool more = s + 1 < nsteps;
        const bool next_chunk = tap == ntaps - 1 && cc + 1 < ncc;
        if (more) load_b(s + 1);
        if (tap == 0 && cc + 1 < ncc) load_halo(cc + 1);  // lands during this chunk's taps
        const int ky = tap / a.KW, kx = tap - ky * a.KW;
        const int toff = ky * HWd + kx;
#pragma unroll
        for (int kk = 0; kk < KC / TL::KSTEP; ++kk) {
            float fa[TL::TM], fb[TL::TN];
#pragma unroll
            for (int i = 0; i < TL::TM; ++i) fa[i] = Hs[(hrow[i] + toff) * AP + kk * TL::KSTEP + lane / MS];
#pragma unroll
            for (int j = 0; j < TL::TN; ++j) {
                const int col = wc * TL::WTN + j * MS + (lane % MS);
                fb[j] = Bs[buf][(kk * TL::KSTEP + lane / MS) * BN + col];
            }
#pragma unroll
            for (int i = 0; i < TL::TM; ++i)
#pragma unroll
                for (int j = 0; j < TL::TN; ++j) {
                    if constexpr (MS == 32)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
                    else
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
                }
        }
        if (more) store_b(buf ^ 1);
        if (next_chunk) {  // every wave is past this chunk's halo reads
            __syncthreads();
            store_halo();
        }
        __syncthreads();
    }
    const int HWimg = a.H * a.W;
    auto rowm = [&](int l) {
        const int y = y0 + l / TW, x = x0 + l % TW;
        return (y < a.H && x < a.W) ? img * HWimg + y * a.W + x : -1;
    };
    epilogue_staged<BM, BN, TL::TM, TL::TN, TL::NACC, MS, false>(a, acc, rowm, wr * TL::WTM, wc * TL::WTN, n0, lane,
                                                                0, smem);
}

// Tiles by output width; the big ones where the launch has >= 2 blocks per CU,
// smaller ones (16x16x4 MFMAs) so small layers still fill the 256 CUs.
using TileN16 = Tile<256, 16, 16, 4>;   // Cout <= 16: 4 waves x (64 px x 16 ch)
using TileN16s = Tile<64, 16, 16, 4>;   //             4 waves x (16 px x 16 ch)
using TileN32 = Tile<128, 32, 32, 4>;   // Cout <= 32: 4 waves x (32 px x 32 ch)
using TileN32s = Tile<64, 32, 16, 4>;   //             4 waves x (16 px x 32 ch)
using TileN64 = Tile<128, 64, 32, 2>;   // wider: 2x2 waves x (64 px x 32 ch), 2 accumulators
using TileN64m = Tile<64, 64, 32, 2>;   //        2x2 waves x (32 px x 32 ch)
using TileN64s = Tile<32, 64, 16, 2>;   //        2x2 waves x (16 px x 32 ch)
using TileN32sK = Tile<64, 32, 16, 4, 32>;  // TileN32s with 32-deep K chunks
// (larger wave tiles -- 64x64 per wave -- were slower; 32-deep K chunks win only
// on the 64 x 32 tile of the small CenterNet launches, see conv_launch)

}  // namespace fvp

namespace fvp {

// ---- bf16 operands (opt-in precision) -------------------------------------------
// Same implicit GEMM on v_mfma_f32_32x32x16_bf16 (fp32 accumulate): the fp32
// activations are rounded to bf16 while staged into LDS, weights are packed
// bf16 [Cpo_w][K] (k contiguous).  K chunks of KC (16 or 32) channels of one
// tap; lane half h of an MFMA takes k = 8h..8h+7 of each 16-wide step.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int BM_, int BN_, int WR_, int KC_>
struct TileB {
    static constexpr int BM = BM_, BN = BN_, WR = WR_, WC = 4 / WR_, KC = KC_;
    static constexpr int WTM = BM / WR, WTN = BN / WC, TM = WTM / 32, TN = WTN / 32;
    static constexpr int P = KC + 8;  // LDS row pitch in bf16: 16-B aligned, conflict-free b128 reads
    static_assert(TM >= 1 && TN >= 1, "tile");
};

template <class TL, bool INBF>
__global__ __launch_bounds__(256, 4) void conv_bf16_kernel(ConvArgs a, const __bf16 *__restrict__ wb) {
    constexpr int BM = TL::BM, BN = TL::BN, KC = TL::KC, P = TL::P;
    constexpr int CPE = INBF ? 8 : 4;                               // channels per A element (16 B bf16 / float4)
    constexpr int AE = BM * KC / CPE, AV = AE >= 256 ? AE / 256 : 1;
    constexpr int BE = BN * KC / 8, BV = BE >= 256 ? BE / 256 : 1;  // B: 8 bf16 per element
    constexpr int KLDS = (2 * BM * P + 2 * BN * P) / 2, CLDS = BM * (BN + 4);  // floats: K loop / epilogue
    __shared__ __attribute__((aligned(16))) float smem[KLDS > CLDS ? KLDS : CLDS];
    __bf16 (*As)[BM * P] = reinterpret_cast<__bf16 (*)[BM * P]>(smem);
    __bf16 (*Bs)[BN * P] = reinterpret_cast<__bf16 (*)[BN * P]>(reinterpret_cast<__bf16 *>(smem) + 2 * BM * P);  // [column][k]
    const int M = a.N * a.Hm * a.Wm;
    int mt, nt;
    conv_tile(mt, nt);
    const int m0 = mt * BM, n0 = nt * BN;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wr = wave % TL::WR, wc = wave / TL::WR;
    const int g = blockIdx.z;  // parity group (mode 3), else 0
    // Cpi % KC == 0: a chunk is one tap x KC channels; an RGB input at a 4 / 8 /
    // 12-channel pitch (fp32) instead spans several taps per chunk, each
    // element its own tap, with the weight rows zero padded to 16 (KC = 16)
    const bool small = a.Cpi % KC != 0;
    const int cpc = small ? 1 : a.Cpi / KC;
    const int ntaps = a.KH * a.KW;
    const size_t Ktot = small ? (size_t)conv_krows(a.KH, a.KW, a.Cpi) : (size_t)ntaps * a.Cpi;  // weight row
    const int nchunks = (int)(Ktot / KC);
    const __bf16 *__restrict__ w = wb + (size_t)g * a.Cpo_w * Ktot;
    const int py = a.up2 == 3 ? 1 - (g >> 1) : a.py, px = a.up2 == 3 ? 1 - (g & 1) : a.px;
    // input image rows: fp32 or bf16 elements
    const size_t esz = INBF ? 2 : 4;
    f32x16 acc[TL::TM][TL::TN];
#pragma unroll
    for (int i = 0; i < TL::TM; ++i)
#pragma unroll
        for (int j = 0; j < TL::TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    int pyx[AV][2];
    const char *pbase[AV];
#pragma unroll
    for (int u = 0; u < AV; ++u) {
        PixRef pr;
        pix_ref(a, m0 + ((u * 256 + t) / (KC / CPE)), M, py, px, pr);
        pyx[u][0] = pr.y;
        pyx[u][1] = pr.x;
        // pix_ref's row base assumes fp32 elements: recompute for the element size
        const int m = m0 + ((u * 256 + t) / (KC / CPE));
        const int img = m < M ? m / (a.Hm * a.Wm) : 0;
        pbase[u] = reinterpret_cast<const char *>(a.in) + (size_t)img * a.H * a.W * a.Cpi * esz;
    }
    uint4 av[AV];  // INBF: 8 bf16; else the bits of a float4
    uint4 bv[BV];
    auto load = [&](int chunk) {
        const int tap = chunk / cpc, c = chunk - tap * cpc;
#pragma unroll
        for (int u = 0; u < AV; ++u) {
            const int e = u * 256 + t;  // -> (pixel e/(KC/CPE), CPE channels)
            int tp = tap, ci = c * KC + (e % (KC / CPE)) * CPE;
            if (!INBF && small) {  // this element's own tap (k past the taps reads 0)
                const int k = chunk * KC + (e % (KC / CPE)) * CPE;
                tp = k / a.Cpi;
                ci = k - tp * a.Cpi;
            }
            const int ky = tp / a.KW, kx = tp - (tp / a.KW) * a.KW;
            const int y = pyx[u][0] + ky, x = pyx[u][1] + kx;
            av[u] = make_uint4(0u, 0u, 0u, 0u);
            if (e < AE && tp < ntaps && (unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W)
                av[u] = *reinterpret_cast<const uint4 *>(pbase[u] + (((size_t)y * a.W + x) * a.Cpi + ci) * esz);
        }
#pragma unroll
        for (int u = 0; u < BV; ++u) {
            const int e = u * 256 + t;  // -> (column e/(KC/8), 8 k)
            if (e < BE)
                bv[u] = *reinterpret_cast<const uint4 *>(w + (size_t)(n0 + e / (KC / 8)) * Ktot + (size_t)chunk * KC +
                                                        (e % (KC / 8)) * 8);
        }
    };
    load(0);
    for (int ch = 0; ch < nchunks; ++ch) {
        const int buf = ch & 1;
#pragma unroll
        for (int u = 0; u < AV; ++u) {
            const int e = u * 256 + t;
            if (e < AE) {
                if constexpr (INBF) {
                    *reinterpret_cast<uint4 *>(&As[buf][(e / (KC / 8)) * P + (e % (KC / 8)) * 8]) = av[u];
                } else {
                    bf16x4 h;
                    h[0] = (__bf16)__builtin_bit_cast(float, av[u].x);
                    h[1] = (__bf16)__builtin_bit_cast(float, av[u].y);
                    h[2] = (__bf16)__builtin_bit_cast(float, av[u].z);
                    h[3] = (__bf16)__builtin_bit_cast(float, av[u].w);
                    *reinterpret_cast<bf16x4 *>(&As[buf][(e / (KC / 4)) * P + (e % (KC / 4)) * 4]) = h;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < BV; ++u) {
            const int e = u * 256 + t;
            if (e < BE) *reinterpret_cast<uint4 *>(&Bs[buf][(e / (KC / 8)) * P + (e % (KC / 8)) * 8]) = bv[u];
        }
        __syncthreads();
        if (ch + 1 < nchunks) load(ch + 1);  // in flight during the MFMAs
#pragma unroll
        for (int ks = 0; ks < KC / 16; ++ks) {
            bf16x8 fa[TL::TM], fb[TL::TN];
#pragma unroll
            for (int i = 0; i < TL::TM; ++i)
                fa[i] = *reinterpret_cast<const bf16x8 *>(
                    &As[buf][(wr * TL::WTM + i * 32 + (lane & 31)) * P + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
            for (int j = 0; j < TL::TN; ++j)
                fb[j] = *reinterpret_cast<const bf16x8 *>(
                    &Bs[buf][(wc * TL::WTN + j * 32 + (lane & 31)) * P + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
            for (int i = 0; i < TL::TM; ++i)
#pragma unroll
                for (int j = 0; j < TL::TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
    }

    auto rowm = [&](int l) { return m0 + l < M ? m0 + l : -1; };
    epilogue_staged<BM, BN, TL::TM, TL::TN, 16, 32, true>(a, acc, rowm, wr * TL::WTM, wc * TL::WTN, n0, lane, g,
                                                         smem);
}

// ---- bf16 activations, Cpi % 32 == 0: LDS-DMA staged implicit GEMM -------------
// The bf16 layers (bf16 NHWC in, weights bf16 [G][Cpo_w][K]).  A K step is
// one tap x BK channels = one 128-B (BK 64) or 64-B (BK 32) row per pixel /
// output column (below for BK 64; BK 32: 16 rows per wave load, swizzle
// s ^ ((r >> 2) & 3)).
// Both operands go global -> LDS by buffer_load_dwordx4 ... lds (no VGPR
// staging, no LDS write pass): one wave instruction moves 8 whole rows (1 KiB, lane l
// -> row l/8, 16-B slot l%8).  The LDS image is lane-linear, so the bank
// swizzle is applied on the SOURCE side: slot s of row r holds the row's
// 16-B chunk s ^ ((r >> 1) & 7), which makes the ds_read_b128 fragment reads
// of v_mfma_f32_32x32x16_bf16 (lane -> row lane&31, chunk 2*kk + lane/32)
// conflict-free.  Padding taps and rows past M read zeros (range check).  Two
// stages: step s+1 is in flight while step s feeds the MFMAs (counted vmcnt,
// raw s_barrier: a __syncthreads() would drain the prefetch).  Tile 128 x BN,
// waves 2 x NW/2 (64 x 32 each at BN 128 with 8 waves: 108 VGPRs, 4 waves per
// SIMD; 4 waves of 64 x 64 took 184 VGPRs and ran 2.6 % slower over ResNet-50).  Measured before it (register-staged
// conv_bf16_kernel, 3x3 64->64 at 40 x 128 x 240): 18 VALU + 17 SALU per
// MFMA, 41 % of wave time parked on waits, 33 % of LDS cycles bank conflicts.

#define FVP_WAIT_BARRIER(vm) asm volatile("s_waitcnt vmcnt(" #vm ")\n\ts_barrier" ::: "memory")

template <int BN, int BK, int NW, bool F32>
__global__ __launch_bounds__(NW * 64, 2) void conv_dma_kernel(ConvArgs a, const void *__restrict__ wb) {
    // waves WRN (rows) x WCN (columns): 2 x NW/2 of 64 x BN/(NW/2), or NW x 1 of 32 x 32 at BN 32
    constexpr int NT = NW * 64, WCN = BN == 32 ? 1 : NW / 2, WRN = NW / WCN;
    constexpr int BM = 128, WTM = BM / WRN, TM = WTM / 32, WTN = BN / WCN, TN = WTN / 32;
    constexpr int ES = F32 ? 4 : 2;                             // operand bytes
    constexpr int RB = BK * ES, SPR = RB / 16, RPI = 1024 / RB;  // row bytes, 16-B slots per row, rows per wave load
    constexpr int NAI = BM / (NW * RPI), NBI = BN / (NW * RPI), NPS = NAI + NBI;  // wave loads per K step
    constexpr int ABYTES = BM * RB, STAGE = ABYTES + BN * RB;
    constexpr int KLDS = 2 * STAGE, CLDS = BM * (BN + 4) * 4;
    static_assert((RB == 64 || RB == 128) && (BN == 32 || BN == 64 || BN == 128) && (NW == 4 || NW == 8) &&
                  TM >= 1 && TN >= 1 && NAI >= 1 && NBI >= 1, "tile");
    __shared__ __attribute__((aligned(16))) float smem[(KLDS > CLDS ? KLDS : CLDS) / 4];
    char *lds = reinterpret_cast<char *>(smem);
    // conflict-free ds_read_b128 fragment reads: 16-B slot s of row r holds chunk s ^ swz(r)
    auto swz = [](int r) { return RB == 128 ? (r >> 1) & 7 : (r >> 2) & 3; };
    const int M = a.N * a.Hm * a.Wm;
    int mt, nt;
    conv_tile(mt, nt);
    const int m0 = mt * BM, n0 = nt * BN;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wr = wave % WRN, wc = wave / WRN;
    const int g = blockIdx.z;  // parity group (mode 3), else 0
    const int py = a.up2 == 3 ? 1 - (g >> 1) : a.py, px = a.up2 == 3 ? 1 - (g & 1) : a.px;
    const int cpc = a.Cpi / BK, nks = a.KH * a.KW * cpc;
    const size_t Ktot = (size_t)a.KH * a.KW * a.Cpi;
    const int slot = lane % SPR;
    // Both operands through buffer descriptors (32-bit offsets; the host keeps
    // the activations under 2 GiB): a padding tap or a row past M reads at
    // kOOB, which the range check turns into zeros.  Per row, the input offset
    // of tap (0, 0) and a bit mask of the taps inside the image are decoded
    // once (quotients by a float reciprocal + one correction: M < 2^24).
    const u32x4 ra = uniform_rsrc4(a.in, (unsigned)((size_t)a.N * a.H * a.W * a.Cpi * ES));
    const u32x4 rb = uniform_rsrc4(reinterpret_cast<const char *>(wb) + (size_t)g * a.Cpo_w * Ktot * ES,
                                   (unsigned)((size_t)a.Cpo_w * Ktot * ES));
    const int HWm = a.Hm * a.Wm;
    const float inv_hw = 1.0f / (float)HWm, inv_w = 1.0f / (float)a.Wm;
    auto qdiv = [](int n, int d, float inv) {
        int q = (int)((float)n * inv);
        const int r = n - q * d;
        return q + (r >= d) - (r < 0);
    };
    unsigned rep = 0;  // bit ky*KW set for every tap row (uniform)
    for (int ky = 0; ky < a.KH; ++ky) rep |= 1u << (ky * a.KW);
    int voa[NAI];
    unsigned tmask[NAI];
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
        const int r = (wave * NAI + i) * RPI + lane / SPR;
        const int m = m0 + r, mm = m < M ? m : 0;
        const int img = qdiv(mm, HWm, inv_hw), rr = mm - img * HWm;
        const int oy = qdiv(rr, a.Wm, inv_w), ox = rr - oy * a.Wm;
        const int y0 = oy * a.sy - py, x0 = ox * a.sx - px;
        // taps inside the image: ky in [max(0, -y0), min(KH, H - y0)), likewise kx
        const int ylo = min(max(-y0, 0), a.KH), yhi = min(max(a.H - y0, 0), a.KH);
        const int xlo = min(max(-x0, 0), a.KW), xhi = min(max(a.W - x0, 0), a.KW);
        const unsigned xm = ((1u << xhi) - 1u) & ~((1u << xlo) - 1u);  // KW <= 32 bits
        // tap rows ylo..yhi-1 of the all-rows pattern rep = sum 2^(ky*KW): mask = xm * rep(rows)
        const unsigned rows = (unsigned)(((1ull << (yhi * a.KW)) - 1ull) & ~((1ull << (ylo * a.KW)) - 1ull));
        tmask[i] = m < M ? xm * (rep & rows) : 0u;
        voa[i] = ((img * a.H + y0) * a.W + x0) * a.Cpi * ES + (slot ^ swz(r)) * 16;  // < 0 only for unused taps
    }
    int vob[NBI];
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
        const int r = (wave * NBI + i) * RPI + lane / SPR;
        vob[i] = (n0 + r) * (int)Ktot * ES + (slot ^ swz(r)) * 16;
    }
    typedef __attribute__((address_space(3))) char *lds_cp;
    const unsigned lds0 = (unsigned)(size_t)(lds_cp)lds;  // the stage buffers' LDS byte address
    auto issue = [&](int ks, int tap, int d, int buf) {
        const unsigned sa = lds0 + buf * STAGE;
#pragma unroll
        for (int i = 0; i < NAI; ++i) {
            const unsigned vo = (tmask[i] >> tap) & 1u ? (unsigned)(voa[i] + d) : kOOB;
            lds_dma16(ra, __builtin_amdgcn_readfirstlane(sa + (wave * NAI + i) * 1024), vo);
        }
#pragma unroll
        for (int i = 0; i < NBI; ++i)
            lds_dma16(rb, __builtin_amdgcn_readfirstlane(sa + ABYTES + (wave * NBI + i) * 1024),
                      (unsigned)(vob[i] + ks * RB));
    };
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    int tap = 0, kx = 0, cc = 0, d = 0;  // tap, its column and channel chunk, byte delta of the next step
    auto advance = [&]() {
        d += RB;
        if (++cc == cpc) {
            cc = 0;
            ++tap;
            if (++kx == a.KW) {
                kx = 0;
                d += (a.W - a.KW) * a.Cpi * ES;  // next tap row
            }
        }
    };
    issue(0, 0, 0, 0);
    advance();
    for (int ks = 0; ks < nks; ++ks) {
        const int buf = ks & 1;
        if (ks + 1 < nks) {  // buf ^ 1 was last read in step ks - 1, before its closing barrier
            issue(ks + 1, tap, d, buf ^ 1);
            advance();
            if constexpr (NPS == 8) FVP_WAIT_BARRIER(8);  // step ks landed (this wave's), then everyone's
            else if constexpr (NPS == 6) FVP_WAIT_BARRIER(6);
            else if constexpr (NPS == 5) FVP_WAIT_BARRIER(5);
            else if constexpr (NPS == 4) FVP_WAIT_BARRIER(4);
            else if constexpr (NPS == 3) FVP_WAIT_BARRIER(3);
            else {
                static_assert(NPS == 2, "wave loads per step");
                FVP_WAIT_BARRIER(2);
            }
        } else {
            FVP_WAIT_BARRIER(0);
        }
        const char *sa = lds + buf * STAGE, *sb = sa + ABYTES;
#pragma unroll
        for (int kk = 0; kk < RB / 32; ++kk) {  // a lane half reads one 16-B chunk of each row
            const int c = kk * 2 + (lane >> 5);
            const char *pa[TM], *pb[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wr * WTM + i * 32 + (lane & 31);
                pa[i] = sa + row * RB + ((c ^ swz(row)) << 4);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = wc * WTN + j * 32 + (lane & 31);
                pb[j] = sb + col * RB + ((c ^ swz(col)) << 4);
            }
            if constexpr (F32) {
                // fp32: chunk c of lane half h holds k = 8 kk + 4 h + q, q < 4, so the
                // q-th v_mfma_f32_32x32x2f32 sums the k pair {8 kk + q, 8 kk + 4 + q}
                // (both operands agree on it): one ds_read_b128 per operand feeds 4
                // MFMAs.  Every product is summed in fp32 as before, in another order.
                float4 fa[TM], fb[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const float4 *>(pa[i]);
#pragma unroll
                for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const float4 *>(pb[j]);
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[j][q], fa[i][q], acc[i][j], 0, 0, 0);
            } else {
                bf16x8 fa[TM], fb[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const bf16x8 *>(pa[i]);
#pragma unroll
                for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const bf16x8 *>(pb[j]);
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)  // D = W x A^T: lane -> pixel, 4 consecutive registers -> 4 channels
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // buf is free for step ks + 2
    }
    // stage [pixel][channel] with one 16-B write per 4 accumulators (register
    // r of tile (i, j): pixel i*32 + lane%32, channel j*32 + 8*(r/4) + 4*(lane/32) + r%4)
    {
        constexpr int CP = BN + 4;
        float *cs = smem + (wr * WTM + (lane & 31)) * CP + wc * WTN + 4 * (lane >> 5);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *reinterpret_cast<float4 *>(cs + i * 32 * CP + j * 32 + q * 8) =
                        make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
    }
    __syncthreads();
    auto rowm = [&](int l) { return m0 + l < M ? m0 + l : -1; };
    epilogue_write<BM, BN, true, decltype(rowm), NT>(a, rowm, n0, g, smem);
}
#undef FVP_WAIT_BARRIER

// ---- the RGB stem on bf16 MFMA, straight from the NCHW fp32 images ----------
// conv1 of PoseResNet (resnet.py:105-107: 7x7, stride 2, pad 3, <= 4 input
// channels -> 64) + BN + ReLU, bf16 NHWC output.  A block owns an 8 x 32
// output tile: the (2*8+5) x (2*32+5) input halo of its C planes is read once
// (coalesced rows of each NCHW plane), rounded to bf16 into LDS as
// [row][x][4 channels] (8 B per pixel), and the weights [64][7][8][4] (kx
// padded to 8, channels to 4, zeros) are staged next to it.  K = 7 rows x 2
// steps of 16 = 224: a lane's 8 k values of a 32x32x16 step are two
// x-adjacent taps x 4 channels = 16 contiguous LDS bytes (the halo starts at
// an even x, so ds_read_b128 stays aligned).  Wave w owns output rows 2w, 2w+1
// (32 pixels each) x 64 channels; the accumulators come out Wᵀ-major (lane ->
// pixel, 4 consecutive registers -> 4 channels), get BN + ReLU in registers
// and go through LDS to 16-B row stores.  Persistent blocks (2 per CU) walk
// the tiles: the weights are staged once per block, and the next tile's halo
// is loaded into registers while the current one runs its MFMAs, epilogue and
// stores.  Replaces the NCHW -> NHWC pass and the register-staged
// small-channel path (0.23 + 0.68 ms per 40 images).
constexpr int kStemTH = 8, kStemTW = 32, kStemHR = 2 * kStemTH + 5, kStemHX = 2 * kStemTW + 6;
constexpr int kStemWP = 232;  // weight row pitch (bf16): 224 + 8, conflict-free ds_read_b128
constexpr int kStemOP = 72;   // output staging pitch (bf16)
constexpr int kStemHE = (kStemHR * kStemHX + 255) / 256;  // halo pixels per thread

__global__ __launch_bounds__(256, 2) void conv_stem7_bf16_kernel(const float *__restrict__ img, int C, int H, int W,
                                                                  int Ho, int Wo, int tiles_x, int tiles_y,
                                                                  int ntiles, const __bf16 *__restrict__ wpk,
                                                                  const float *__restrict__ scale,
                                                                  const float *__restrict__ shift,
                                                                  __bf16 *__restrict__ out) {
    constexpr int HALO_B = kStemHR * kStemHX * 8, W_B = 64 * kStemWP * 2;
    constexpr int OUT_B = kStemTH * kStemTW * kStemOP * 2;
    __shared__ __attribute__((aligned(16))) unsigned char smem[HALO_B + W_B + OUT_B];
    __bf16 *halo = reinterpret_cast<__bf16 *>(smem);
    __bf16 *wl = reinterpret_cast<__bf16 *>(smem + HALO_B);
    __bf16 *st = reinterpret_cast<__bf16 *>(smem + HALO_B + W_B);
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int px = lane & 31, h = lane >> 5;
    const int per_img = tiles_x * tiles_y;
    // weights [64][224] -> LDS rows of kStemWP, once per block
    for (int e = t; e < 64 * 28; e += 256) {
        const int co = e / 28, q = e - (e / 28) * 28;
        *reinterpret_cast<uint4 *>(wl + co * kStemWP + q * 8) = *reinterpret_cast<const uint4 *>(wpk + co * 224 + q * 8);
    }
    float hv[kStemHE][3];  // the next tile's halo pixels (up to 3 planes; a 4th would be a C = 4 input)
    float hv4[kStemHE];
    auto load_halo = [&](int tile) {
        const int n = tile / per_img, tr = tile - n * per_img;
        const int iy0 = 2 * ((tr / tiles_x) * kStemTH) - 3, ix0 = 2 * ((tr - (tr / tiles_x) * tiles_x) * kStemTW) - 3;
        const float *__restrict__ src = img + (size_t)n * C * H * W;
#pragma unroll
        for (int u = 0; u < kStemHE; ++u) {
            const int e = t + u * 256;
            const int r = e / kStemHX, c = e - (e / kStemHX) * kStemHX;
            const int y = iy0 + r, x = ix0 + c;
            const bool in = e < kStemHR * kStemHX && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
            const size_t o = (size_t)(in ? y : 0) * W + (in ? x : 0);
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) hv[u][ch] = (in && ch < C) ? src[(size_t)ch * H * W + o] : 0.0f;
            hv4[u] = (in && C > 3) ? src[(size_t)3 * H * W + o] : 0.0f;
        }
    };
    int tile = blockIdx.x;
    if (tile < ntiles) load_halo(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        // halo registers -> LDS (every wave finished the previous tile's MFMAs: barrier below)
#pragma unroll
        for (int u = 0; u < kStemHE; ++u) {
            const int e = t + u * 256;
            if (e < kStemHR * kStemHX) {
                bf16x4 hb;
                hb[0] = (__bf16)hv[u][0];
                hb[1] = (__bf16)hv[u][1];
                hb[2] = (__bf16)hv[u][2];
                hb[3] = (__bf16)hv4[u];
                *reinterpret_cast<bf16x4 *>(halo + e * 4) = hb;
            }
        }
        __syncthreads();
        const int n = tile / per_img, tr = tile - n * per_img;
        const int oy0 = (tr / tiles_x) * kStemTH, ox0 = (tr - (tr / tiles_x) * tiles_x) * kStemTW;
        if (tile + (int)gridDim.x < ntiles) load_halo(tile + gridDim.x);  // in flight during the MFMAs
        f32x16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
        for (int ky = 0; ky < 7; ++ky) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int kx = 4 * s + 2 * h;  // this lane's two taps: kx, kx + 1
                bf16x8 fa[2], fb[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int oyl = wave * 2 + i;
                    fa[i] = *reinterpret_cast<const bf16x8 *>(halo + ((2 * oyl + ky) * kStemHX + 2 * px + kx) * 4);
                }
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    fb[j] = *reinterpret_cast<const bf16x8 *>(wl + (j * 32 + px) * kStemWP + (ky * 8 + kx) * 4);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
            }
        }
        // BN + ReLU -> bf16 staging (its previous reads, the stores below, precede the barrier above)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int co = j * 32 + 8 * q + 4 * h;  // channels co..co+3 of pixel px
                const float4 sc = *reinterpret_cast<const float4 *>(scale + co);
                const float4 sh = *reinterpret_cast<const float4 *>(shift + co);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    bf16x4 o;
                    o[0] = (__bf16)fmaxf(acc[i][j][4 * q + 0] * sc.x + sh.x, 0.0f);
                    o[1] = (__bf16)fmaxf(acc[i][j][4 * q + 1] * sc.y + sh.y, 0.0f);
                    o[2] = (__bf16)fmaxf(acc[i][j][4 * q + 2] * sc.z + sh.z, 0.0f);
                    o[3] = (__bf16)fmaxf(acc[i][j][4 * q + 3] * sc.w + sh.w, 0.0f);
                    *reinterpret_cast<bf16x4 *>(st + ((wave * 2 + i) * kStemTW + px) * kStemOP + co) = o;
                }
            }
        __syncthreads();  // staging complete; every wave is past its halo reads
        // 8 x 32 pixels x 128 B: 16-B pieces, a tile row's 32 pixels contiguous in NHWC
        for (int e = t; e < kStemTH * kStemTW * 8; e += 256) {
            const int pix = e >> 3, q = e & 7;
            const int oy = oy0 + pix / kStemTW, ox = ox0 + (pix % kStemTW);
            if (oy < Ho && ox < Wo)
                *reinterpret_cast<uint4 *>(out + (((size_t)n * Ho + oy) * Wo + ox) * 64 + q * 8) =
                    *reinterpret_cast<const uint4 *>(st + pix * kStemOP + q * 8);
        }
    }
}

// ---- the same stem on the fp32 matrix cores (the default precision) --------
// 7x7 / s2 / p3, C <= 3 NCHW planes -> 64 channels + BN + ReLU, fp32 NHWC64
// out.  The generic path converts the images to a 4-channel NHWC pitch first
// and walks K = 49 taps x 4 channels, a quarter of it the zero channel (1.42 +
// 0.1 ms per 40 images).  Here K is the 147 real (tap, channel) pairs in the
// order kk = ky * 21 + kx * 3 + c, padded to 148 = 37 steps of
// v_mfma_f32_16x16x4f32 with the weights as the A operand: the halo keeps the
// three planes interleaved ([row][x][c], 207-float rows), so within a kernel
// row kk - 21 ky is the lane's offset from its pixel (6 j for output column j)
// and a step whose four kk straddle two rows only adds the row step (186
// floats) on the lanes past the seam.  Persistent blocks (2 per CU) walk 8 x 32
// output tiles: the [148][64] weights are staged once per block, and the next
// tile's halo is loaded into registers during the current tile's MFMAs.  Wave
// w owns output rows 2w, 2w + 1 x 32 columns (4 pixel tiles) x the 64 channels
// (4 channel tiles): per step 4 A + 4 B reads for 16 MFMAs.  D[co][pixel]:
// lane -> pixel, its 4 registers -> 4 consecutive channels, one 16-B store.
constexpr int kS32TH = 8, kS32TW = 32, kS32HR = 2 * kS32TH + 5, kS32HX = 2 * kS32TW + 5;  // 21 x 69 halo
constexpr int kS32RP = kS32HX * 3;                           // halo row pitch (floats)
constexpr int kS32Halo = kS32HR * kS32RP;                    // 4,347 floats
constexpr int kS32HU = (kS32Halo + 255) / 256;               // halo floats per thread
constexpr int kS32K = 148, kS32WP = 80;                      // weight rows [kk][co], conflict-free pitch
constexpr int kS32HaloLds = (kS32Halo + 3) / 4 * 4;

__global__ __launch_bounds__(256, 2) void conv_stem7_f32_kernel(const float *__restrict__ img, int C, int H, int W,
                                                                 int Ho, int Wo, int tiles_x, int tiles_y,
                                                                 int ntiles, const float *__restrict__ wpk,
                                                                 const float *__restrict__ scale,
                                                                 const float *__restrict__ shift,
                                                                 float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float lds[kS32HaloLds + kS32K * kS32WP];
    float *halo = lds, *wl = lds + kS32HaloLds;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int j = lane & 15, g = lane >> 4;
    const int per_img = tiles_x * tiles_y;
    for (int e = t; e < kS32K * kS32WP / 4; e += 256)
        reinterpret_cast<f32x4 *>(wl)[e] = reinterpret_cast<const f32x4 *>(wpk)[e];
    float hv[kS32HU];
    auto origin = [&](int tile, int &n, int &oy0, int &ox0) {
        n = tile / per_img;
        const int tr = tile - n * per_img, ty = tr / tiles_x;
        oy0 = ty * kS32TH;
        ox0 = (tr - ty * tiles_x) * kS32TW;
    };
    // halo float e <- plane c = e / (HR * HX), row r, column x (consecutive threads: consecutive x)
    auto load_halo = [&](int tile) {
        int n, oy0, ox0;
        origin(tile, n, oy0, ox0);
        const float *__restrict__ src = img + (size_t)n * C * H * W;
#pragma unroll
        for (int u = 0; u < kS32HU; ++u) {
            const int e = t + 256 * u;
            const int c = e / (kS32HR * kS32HX), rem = e - c * (kS32HR * kS32HX);
            const int r = rem / kS32HX, xx = rem - r * kS32HX;
            const int y = 2 * oy0 - 3 + r, x = 2 * ox0 - 3 + xx;
            const bool in = e < kS32Halo && c < C && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
            hv[u] = in ? src[((size_t)c * H + y) * W + x] : 0.0f;
        }
    };
    f32x4 sc[4], sh[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        sc[c] = *reinterpret_cast<const f32x4 *>(scale + 16 * c + 4 * g);
        sh[c] = *reinterpret_cast<const f32x4 *>(shift + 16 * c + 4 * g);
    }
    // the lane's extra row step on a seam step, by the seam's first lane group (1, 2, 3)
    const int seam1 = g >= 1 ? kS32RP - 21 : 0, seam2 = g >= 2 ? kS32RP - 21 : 0, seam3 = g >= 3 ? kS32RP - 21 : 0;
    const float *wlane = wl + g * kS32WP + j;
    const float *hlane = halo + 4 * wave * kS32RP + 6 * j + g;
    int tile = blockIdx.x;
    if (tile < ntiles) load_halo(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        __syncthreads();  // every wave is past the previous tile's halo reads (and the weights are stored)
#pragma unroll
        for (int u = 0; u < kS32HU; ++u) {
            const int e = t + 256 * u;
            if (e < kS32Halo) {
                const int c = e / (kS32HR * kS32HX), rem = e - c * (kS32HR * kS32HX);
                halo[rem * 3 + c] = hv[u];  // [row][x][c]: row * 207 + x * 3 + c = rem * 3 + c
            }
        }
        if (tile + (int)gridDim.x < ntiles) load_halo(tile + gridDim.x);  // in flight during the MFMAs
        __syncthreads();
        f32x4 acc[4][4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int p = 0; p < 4; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kS32K / 4; ++s) {
            const int kk0 = 4 * s, ky0 = kk0 / 21, seam = 21 * (ky0 + 1) - kk0;  // lanes g >= seam: next row
            const int step = seam == 1 ? seam1 : seam == 2 ? seam2 : seam == 3 ? seam3 : 0;
            const int boff = kk0 + ky0 * (kS32RP - 21);
            f32x4 a, b;
#pragma unroll
            for (int c = 0; c < 4; ++c) a[c] = wlane[kk0 * kS32WP + 16 * c];
#pragma unroll
            for (int p = 0; p < 4; ++p) {  // pixel tile p: output row 2w + (p >> 1), columns 16 (p & 1) ..
                const float v = hlane[(p >> 1) * 2 * kS32RP + (p & 1) * 96 + boff + step];
                b[p] = (s == kS32K / 4 - 1 && g == 3) ? 0.0f : v;  // kk = 147: the zero K row
            }
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int p = 0; p < 4; ++p) acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], b[p], acc[c][p], 0, 0, 0);
        }
        int n, oy0, ox0;
        origin(tile, n, oy0, ox0);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int oy = oy0 + 2 * wave + (p >> 1), ox = ox0 + 16 * (p & 1) + j;
            if (oy < Ho && ox < Wo) {
                float *o = out + (((size_t)n * Ho + oy) * Wo + ox) * 64 + 4 * g;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    f32x4 v;
#pragma unroll
                    for (int k = 0; k < 4; ++k) v[k] = fmaxf(acc[c][p][k] * sc[c][k] + sh[c][k], 0.0f);
                    *reinterpret_cast<f32x4 *>(o + 16 * c) = v;
                }
            }
        }
    }
}

// ---- the CNNs' 7x7 J -> 16 front conv on bf16 MFMA, from the NCHW maps -------
// Basic2DBlock(J, 16, 7) of P2PNet / CenterNet (cnns_2d.py:12-29, 185-232,
// 235-295): 7x7, stride 1, pad 3, C <= 16 input planes -> 16 channels + BN +
// ReLU, bf16 NHWC16 out.  On the generic path it was the slowest layer of the
// bf16 P2PNet (16 output columns on a 32-wide MFMA tile, a conversion pass
// before it).  A block owns an 8 x 32 output tile: the 14 x 38 input halo of
// the C planes goes to LDS once as bf16 [row][x][16 channels] (48-B pixel
// pitch: conflict-free fragment reads), the weights [16][50 taps][16] (tap 49
// and channels >= C zero) beside it.  v_mfma_f32_16x16x32_bf16 with the
// weights as the A operand: K step = 2 taps x 16 channels, a lane's 8 k values
// = 8 channels of one tap (16 contiguous bytes), and the output comes out with
// lane -> pixel, 4 registers -> 4 consecutive channels.
constexpr int kFrTH = 8, kFrTW = 32, kFrHR = kFrTH + 6, kFrHX = kFrTW + 6, kFrPB = 48;  // pixel pitch (B)
constexpr int kFrWP = 50 * 16 + 8;                                                      // weight row (bf16)

__global__ __launch_bounds__(256) void conv_front7_bf16_kernel(const float *__restrict__ x, int C, int H, int W,
                                                               int tiles_x, int tiles_y,
                                                               const __bf16 *__restrict__ wpk,
                                                               const float *__restrict__ scale,
                                                               const float *__restrict__ shift,
                                                               __bf16 *__restrict__ out) {
    constexpr int HALO_B = kFrHR * kFrHX * kFrPB, W_B = 16 * kFrWP * 2, OUT_B = kFrTH * kFrTW * 16 * 2;
    __shared__ __attribute__((aligned(16))) unsigned char smem[HALO_B + W_B + OUT_B];
    unsigned char *halo = smem;
    __bf16 *wl = reinterpret_cast<__bf16 *>(smem + HALO_B);
    __bf16 *st = reinterpret_cast<__bf16 *>(smem + HALO_B + W_B);
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int per_img = tiles_x * tiles_y;
    const int n = blockIdx.x / per_img, tr = blockIdx.x - n * per_img;
    const int oy0 = (tr / tiles_x) * kFrTH, ox0 = (tr - (tr / tiles_x) * tiles_x) * kFrTW;
    const float *__restrict__ src = x + (size_t)n * C * H * W;
    // halo (r, c) <- input (oy0 - 3 + r, ox0 - 3 + c), C planes -> 16 bf16 (zeros past C / outside)
    for (int e = t; e < kFrHR * kFrHX; e += 256) {
        const int r = e / kFrHX, c = e - (e / kFrHX) * kFrHX;
        const int y = oy0 - 3 + r, xx = ox0 - 3 + c;
        const bool in = (unsigned)y < (unsigned)H && (unsigned)xx < (unsigned)W;
        const size_t o = (size_t)(in ? y : 0) * W + (in ? xx : 0);
        bf16x8 h0, h1;
#pragma unroll
        for (int ch = 0; ch < 8; ++ch) {
            h0[ch] = (__bf16)((in && ch < C) ? src[(size_t)ch * H * W + o] : 0.0f);
            h1[ch] = (__bf16)((in && ch + 8 < C) ? src[(size_t)(ch + 8) * H * W + o] : 0.0f);
        }
        *reinterpret_cast<bf16x8 *>(halo + e * kFrPB) = h0;
        *reinterpret_cast<bf16x8 *>(halo + e * kFrPB + 16) = h1;
    }
    for (int e = t; e < 16 * 100; e += 256) {  // weights: 16 rows x 100 pieces of 8
        const int co = e / 100, q = e - (e / 100) * 100;
        *reinterpret_cast<uint4 *>(wl + co * kFrWP + q * 8) = *reinterpret_cast<const uint4 *>(wpk + co * 800 + q * 8);
    }
    __syncthreads();
    const int px = lane & 15, g = lane >> 4;  // pixel of a 16-pixel M tile; k group
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    // wave w: output rows 2w, 2w+1 x 32 columns = 4 tiles of 16 pixels (i: row i/2, columns 16*(i%2)..)
#pragma unroll 5
    for (int s = 0; s < 25; ++s) {
        const int tap = 2 * s + (g >> 1), half = g & 1;  // this lane's tap (49: zero weights) and channel half
        const int ky = tap / 7, kx = tap - (tap / 7) * 7;
        const bf16x8 fw = *reinterpret_cast<const bf16x8 *>(wl + px * kFrWP + tap * 16 + half * 8);
        const int tky = tap < 49 ? ky : 0, tkx = tap < 49 ? kx : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int oyl = wave * 2 + (i >> 1), oxl = (i & 1) * 16 + px;
            const bf16x8 fa = *reinterpret_cast<const bf16x8 *>(halo + ((oyl + tky) * kFrHX + oxl + tkx) * kFrPB +
                                                                  half * 16);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw, fa, acc[i], 0, 0, 0);
        }
    }
    // D[co][pixel]: lane -> pixel px of tile i, registers r -> channel 4g + r
    const float4 sc = *reinterpret_cast<const float4 *>(scale + 4 * g);
    const float4 sh = *reinterpret_cast<const float4 *>(shift + 4 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int pix = (wave * 2 + (i >> 1)) * kFrTW + (i & 1) * 16 + px;
        bf16x4 o;
        o[0] = (__bf16)fmaxf(acc[i][0] * sc.x + sh.x, 0.0f);
        o[1] = (__bf16)fmaxf(acc[i][1] * sc.y + sh.y, 0.0f);
        o[2] = (__bf16)fmaxf(acc[i][2] * sc.z + sh.z, 0.0f);
        o[3] = (__bf16)fmaxf(acc[i][3] * sc.w + sh.w, 0.0f);
        *reinterpret_cast<bf16x4 *>(st + pix * 16 + 4 * g) = o;
    }
    __syncthreads();
    for (int e = t; e < kFrTH * kFrTW * 2; e += 256) {  // 16-B halves of the 32-B pixels
        const int pix = e >> 1, hh = e & 1;
        const int oy = oy0 + pix / kFrTW, ox = ox0 + (pix % kFrTW);
        if (oy < H && ox < W)
            *reinterpret_cast<uint4 *>(out + (((size_t)n * H + oy) * W + ox) * 16 + hh * 8) =
                *reinterpret_cast<const uint4 *>(st + pix * 16 + hh * 8);
    }
}

// ---- the same front conv on the fp32 matrix cores, from the NCHW maps -------
// 7x7, stride 1, pad 3, C <= 16 planes -> 16 channels + BN + ReLU, fp32 NHWC16
// out.  The generic kernels walk K = 49 taps x 16 channels in 49 chunks with a
// global round trip each (CenterNet at 8 frames: 42 us for 1.3 GFLOP); here a
// persistent block stages all 49 taps' weights in LDS once ([tap][co][16 c],
// 16-B quads XOR-swizzled by co so the A reads are conflict-free) and walks
// 8 x 16 output tiles: the 14 x 22 x 16 input halo goes to LDS ([pixel][c],
// 80-B pitch; the next tile's halo is loaded into registers during this tile's
// MFMAs, straight from the C planes: no layout pass), then 49 taps x 4
// v_mfma_f32_16x16x4f32 per 16-pixel row with the weights as the A operand
// (D[co][pixel]: lane -> pixel, its 4 registers -> 4 consecutive channels, one
// 16-B store per lane).  Exact fp32 products; the sum runs tap by tap in
// channel quads (an order of its own, like every fp32 kernel here).
constexpr int kF32TH = 8, kF32TW = 16, kF32HR = kF32TH + 6, kF32HX = kF32TW + 6, kF32HP = 20;
constexpr int kF32Halo = kF32HR * kF32HX;                          // 308 halo pixels
constexpr int kF32HaloItems = kF32Halo * 4;                        // (pixel, channel quad)
constexpr int kF32HU = (kF32HaloItems + 255) / 256;                // halo items per thread
constexpr int kF32Lds = 49 * 16 * 16 + kF32Halo * kF32HP;          // floats: 12,544 + 6,160

__global__ __launch_bounds__(256, 2) void conv_front7_f32_kernel(const float *__restrict__ x, int C, int H, int W,
                                                                 int tiles_x, int tiles_y, int ntiles,
                                                                 const float *__restrict__ wpk,
                                                                 const float *__restrict__ scale,
                                                                 const float *__restrict__ shift,
                                                                 float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float f32lds[];
    float *wl = f32lds, *halo = f32lds + 49 * 16 * 16;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int px = lane & 15, g = lane >> 4;  // pixel of a 16-pixel row; channel quad
    const int per_img = tiles_x * tiles_y;
    const size_t plane = (size_t)H * W;
    // weights [tap][co][c] -> LDS quad (c / 4) ^ ((co >> 2) & 3)
    for (int e = t; e < 49 * 16 * 4; e += 256) {
        const int row = e >> 2, q = e & 3, co = row & 15;
        *reinterpret_cast<f32x4 *>(wl + row * 16 + 4 * (q ^ ((co >> 2) & 3))) =
            *reinterpret_cast<const f32x4 *>(wpk + row * 16 + 4 * q);
    }
    auto origin = [&](int tile, int &n, int &oy0, int &ox0) {
        n = tile / per_img;
        const int tr = tile - n * per_img, ty = tr / tiles_x;
        oy0 = ty * kF32TH;
        ox0 = (tr - ty * tiles_x) * kF32TW;
    };
    f32x4 hv[kF32HU];
    auto load_halo = [&](int tile) {
        int n, oy0, ox0;
        origin(tile, n, oy0, ox0);
        const float *__restrict__ src = x + (size_t)n * C * plane;
#pragma unroll
        for (int u = 0; u < kF32HU; ++u) {
            const int e = t + 256 * u;
            const int p = e >> 2, q = e & 3;
            const int r = p / kF32HX, c = p - r * kF32HX;
            const int y = oy0 - 3 + r, xx = ox0 - 3 + c;
            const bool in = e < kF32HaloItems && (unsigned)y < (unsigned)H && (unsigned)xx < (unsigned)W;
            const size_t o = (size_t)(in ? y : 0) * W + (in ? xx : 0);
            f32x4 v;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = (in && 4 * q + k < C) ? src[(size_t)(4 * q + k) * plane + o] : 0.0f;
            hv[u] = v;
        }
    };
    const f32x4 sc = *reinterpret_cast<const f32x4 *>(scale + 4 * g);
    const f32x4 sh = *reinterpret_cast<const f32x4 *>(shift + 4 * g);
    int tile = blockIdx.x;
    if (tile < ntiles) load_halo(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        __syncthreads();  // every wave is past the previous tile's halo reads (and the weights are stored)
#pragma unroll
        for (int u = 0; u < kF32HU; ++u) {
            const int e = t + 256 * u;
            if (e < kF32HaloItems) *reinterpret_cast<f32x4 *>(halo + (e >> 2) * kF32HP + 4 * (e & 3)) = hv[u];
        }
        if (tile + (int)gridDim.x < ntiles) load_halo(tile + gridDim.x);  // in flight during the MFMAs
        __syncthreads();
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        // wave w: output rows 2w, 2w + 1 (16 pixels each)
#pragma unroll 7
        for (int tap = 0; tap < 49; ++tap) {
            const int ky = tap / 7, kx = tap - ky * 7;
            const f32x4 fw = *reinterpret_cast<const f32x4 *>(wl + (tap * 16 + px) * 16 + 4 * (g ^ ((px >> 2) & 3)));
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const f32x4 fa =
                    *reinterpret_cast<const f32x4 *>(halo + ((2 * wave + i + ky) * kF32HX + px + kx) * kF32HP + 4 * g);
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(fw[k], fa[k], acc[i], 0, 0, 0);
            }
        }
        int n, oy0, ox0;
        origin(tile, n, oy0, ox0);
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // D[co][pixel]: this lane = pixel px of row 2w + i, channels 4g .. 4g + 3
            const int oy = oy0 + 2 * wave + i, ox = ox0 + px;
            if (oy < H && ox < W) {
                f32x4 o;
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = fmaxf(acc[i][k] * sc[k] + sh[k], 0.0f);
                *reinterpret_cast<f32x4 *>(out + (((size_t)n * H + oy) * W + ox) * 16 + 4 * g) = o;
            }
        }
    }
}

// KHxKW / stride-(KH,KW) max pool, KH, KW in {1, 2}, NHWC (F.max_pool2d(x, 2, 2),
// cnns_2d.py Pool2DBlock; F.max_pool1d(x, 2, 2) on H == 1 rows, cnns_1d.py Pool1DBlock)
template <int KH, int KW>
__global__ __launch_bounds__(256) void maxpool_kernel(const float *__restrict__ in, float *__restrict__ out, int N,
                                                      int H, int W, int C) {
    const int Ho = H / KH, Wo = W / KW;
    const long long total = (long long)N * Ho * Wo * (C / 4);
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int c4 = (int)(gid % (C / 4));
    long long r = gid / (C / 4);
    const int x = (int)(r % Wo);
    r /= Wo;
    const int y = (int)(r % Ho);
    const long long img = r / Ho;
    const float4 *p = reinterpret_cast<const float4 *>(in + (((size_t)img * H + KH * y) * W + KW * x) * C) + c4;
    const size_t rs = (size_t)W * C / 4;
    float4 m = p[0];
    auto mx = [&](const float4 b) {
        m.x = nanmax(m.x, b.x);
        m.y = nanmax(m.y, b.y);
        m.z = nanmax(m.z, b.z);
        m.w = nanmax(m.w, b.w);
    };
    if (KW == 2) mx(p[C / 4]);
    if (KH == 2) {
        mx(p[rs]);
        if (KW == 2) mx(p[rs + C / 4]);
    }
    reinterpret_cast<float4 *>(out)[gid] = m;
}

// The same on bf16 activations (C % 8 == 0): 8 channels (16 B) per thread,
// exact (the maximum is one of the inputs).
__device__ __forceinline__ void bf16x8_max(float (&m)[8], const uint4 b) {
    const unsigned w4[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        m[2 * k] = nanmax(m[2 * k], __builtin_bit_cast(float, w4[k] << 16));
        m[2 * k + 1] = nanmax(m[2 * k + 1], __builtin_bit_cast(float, w4[k] & 0xffff0000u));
    }
}

__device__ __forceinline__ uint4 bf16x8_pack(const float (&m)[8]) {  // exact: low halves are zero
    unsigned o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o[k] = (__builtin_bit_cast(unsigned, m[2 * k]) >> 16) | (__builtin_bit_cast(unsigned, m[2 * k + 1]) & 0xffff0000u);
    return make_uint4(o[0], o[1], o[2], o[3]);
}

template <int KH, int KW>
__global__ __launch_bounds__(256) void maxpool_bf16_kernel(const uint4 *__restrict__ in, uint4 *__restrict__ out, int N,
                                                           int H, int W, int C) {
    const int Ho = H / KH, Wo = W / KW, C8 = C / 8;
    const long long total = (long long)N * Ho * Wo * C8;
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int c8 = (int)(gid % C8);
    long long r = gid / C8;
    const int x = (int)(r % Wo);
    r /= Wo;
    const int y = (int)(r % Ho);
    const long long img = r / Ho;
    const uint4 *p = in + (((size_t)img * H + KH * y) * W + KW * x) * C8 + c8;
    const size_t rs = (size_t)W * C8;
    float m[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = -INFINITY;
    bf16x8_max(m, p[0]);
    if (KW == 2) bf16x8_max(m, p[C8]);
    if (KH == 2) {
        bf16x8_max(m, p[rs]);
        if (KW == 2) bf16x8_max(m, p[rs + C8]);
    }
    out[gid] = bf16x8_pack(m);
}

// MaxPool2d(K, S, P) of NHWC activations with implicit -inf padding
// (resnet.py:109: kernel 3, stride 2, padding 1), NaN-propagating like torch.
__global__ __launch_bounds__(256) void maxpool_pad_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                          int N, int H, int W, int C, int K, int S, int P, int Ho,
                                                          int Wo) {
    const long long total = (long long)N * Ho * Wo * (C / 4);
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int c4 = (int)(gid % (C / 4));
    long long r = gid / (C / 4);
    const int x = (int)(r % Wo);
    r /= Wo;
    const int y = (int)(r % Ho);
    const long long img = r / Ho;
    const float4 *base = reinterpret_cast<const float4 *>(in + (size_t)img * H * W * C) + c4;
    float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    for (int ky = 0; ky < K; ++ky) {
        const int iy = y * S - P + ky;
        if ((unsigned)iy >= (unsigned)H) continue;
        for (int kx = 0; kx < K; ++kx) {
            const int ix = x * S - P + kx;
            if ((unsigned)ix >= (unsigned)W) continue;
            const float4 b = base[((size_t)iy * W + ix) * (C / 4)];
            m.x = nanmax(m.x, b.x);
            m.y = nanmax(m.y, b.y);
            m.z = nanmax(m.z, b.z);
            m.w = nanmax(m.w, b.w);
        }
    }
    reinterpret_cast<float4 *>(out)[gid] = m;
}

// ResNet's MaxPool2d(3, 2, 1) (resnet.py:109) with 32-bit index math (the
// generic kernel's 64-bit divisions were its VALU bound: 0.34 ms per 40 images
// of 128 x 240 x 64, 4.6 TB/s).  blockIdx.y = output row (image-major, so the
// row and image are wave-uniform), thread = (column, 4 channels) of that row.
__global__ __launch_bounds__(256) void maxpool3s2_kernel(const float4 *__restrict__ in, float4 *__restrict__ out,
                                                         int H, int W, int C4, int Ho, int Wo) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= Wo * C4) return;
    const int c4 = i % C4, x = i / C4;
    const int y = (int)blockIdx.y % Ho, img = (int)blockIdx.y / Ho;
    const float4 *base = in + (size_t)img * H * W * C4 + c4;
    float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
        const int iy = 2 * y - 1 + ky;
        if ((unsigned)iy >= (unsigned)H) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int ix = 2 * x - 1 + kx;
            if ((unsigned)ix >= (unsigned)W) continue;
            const float4 b = base[(iy * W + ix) * C4];
            m.x = nanmax(m.x, b.x);
            m.y = nanmax(m.y, b.y);
            m.z = nanmax(m.z, b.z);
            m.w = nanmax(m.w, b.w);
        }
    }
    out[(size_t)blockIdx.y * Wo * C4 + i] = m;
}

// The same on bf16 activations (C % 8 == 0): 8 channels (16 B) per thread; the
// maximum of bf16 values is one of them, so the result is exact.
__global__ __launch_bounds__(256) void maxpool_pad_bf16_kernel(const uint4 *__restrict__ in, uint4 *__restrict__ out,
                                                               int N, int H, int W, int C, int K, int S, int P, int Ho,
                                                               int Wo) {
    const int C8 = C / 8;
    const long long total = (long long)N * Ho * Wo * C8;
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int c8 = (int)(gid % C8);
    long long r = gid / C8;
    const int x = (int)(r % Wo);
    r /= Wo;
    const int y = (int)(r % Ho);
    const long long img = r / Ho;
    const uint4 *base = in + (size_t)img * H * W * C8 + c8;
    float m[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = -INFINITY;
    for (int ky = 0; ky < K; ++ky) {
        const int iy = y * S - P + ky;
        if ((unsigned)iy >= (unsigned)H) continue;
        for (int kx = 0; kx < K; ++kx) {
            const int ix = x * S - P + kx;
            if ((unsigned)ix >= (unsigned)W) continue;
            bf16x8_max(m, base[((size_t)iy * W + ix) * C8]);
        }
    }
    out[gid] = bf16x8_pack(m);
}

// NCHW (C channels) -> NHWC with Cp >= C channels (zero padded), and back.
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                           int N, int C, int HW, int Cp) {
    const long long total = (long long)N * HW * Cp;
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int c = (int)(gid % Cp);
    const long long r = gid / Cp;
    const int p = (int)(r % HW);
    const long long img = r / HW;
    out[gid] = c < C ? in[((size_t)img * C + c) * HW + p] : 0.0f;
}

__global__ __launch_bounds__(256) void nhwc_to_nchw_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                           int N, int C, int HW, int Cp) {
    const long long total = (long long)N * C * HW;
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int p = (int)(gid % HW);
    const long long r = gid / HW;
    const int c = (int)(r % C);
    const long long img = r / C;
    out[gid] = in[((size_t)img * HW + p) * Cp + c];
}

// The same through LDS: a block moves 64 pixels x Cp channels of one image --
// 16-B loads of whole pixels, then per channel 64 consecutive pixels (odd LDS
// pitch: conflict-free column reads).  Cp % 4 == 0, C <= 128, 16-B aligned input.
// Only channels 0 .. C-1 of a pixel are read (a partial last quad by scalars):
// `in` may point at channel c0 of a wider pitch (fvp.cnn.to_nchw_from), where a
// whole-pitch read would run c0 floats past the allocation at the last pixel.
__global__ __launch_bounds__(256) void nhwc_to_nchw_tiled_kernel(const float *__restrict__ in,
                                                                 float *__restrict__ out, int C, int HW, int Cp,
                                                                 int tiles_per_img) {
    __shared__ float t[64 * 129];
    const int img = blockIdx.x / tiles_per_img, p0 = (blockIdx.x - img * tiles_per_img) * 64;
    const int np = HW - p0 < 64 ? HW - p0 : 64, pitch = 129, nq = (C + 3) >> 2;
    const float *__restrict__ src = in + ((size_t)img * HW + p0) * Cp;
    for (int e = threadIdx.x; e < 64 * nq; e += 256) {
        const int p = e / nq, q = e - p * nq;
        if (p < np) {
            const float *px = src + (size_t)p * Cp + 4 * q;
            if (4 * q + 4 <= C) {
                const f32x4 v = *reinterpret_cast<const f32x4 *>(px);
#pragma unroll
                for (int k = 0; k < 4; ++k) t[p * pitch + 4 * q + k] = v[k];
            } else {
                for (int k = 0; 4 * q + k < C; ++k) t[p * pitch + 4 * q + k] = px[k];
            }
        }
    }
    __syncthreads();
    float *__restrict__ dst = out + (size_t)img * C * HW + p0;
    for (int e = threadIdx.x; e < C * 64; e += 256) {
        const int c = e >> 6, p = e & 63;
        if (p < np) dst[(size_t)c * HW + p] = t[p * pitch + c];
    }
}

// 1x1 convolution of NHWC activations written straight to NCHW:
// out[n][co][p] = act(scale[co] * sum_ci in[n][p][ci] W[ci][co] + shift[co]).  P2PNet's
// output layer (cnns_2d.py:185-232, Conv2d(32, J, 1)) feeds soft-argmax and WeightNet in
// the reference's NCHW layout; the GEMM kernels write NHWC, and the layout pass after
// them re-read and re-wrote the whole map.  A thread owns one pixel: its CIN4 float4 of
// input in registers, the weights [co][ci] in LDS (float4 broadcast reads), Cout outputs
// stored plane by plane (consecutive threads, consecutive pixels: coalesced rows).
template <int CIN4>
__global__ __launch_bounds__(256) void conv1x1_nchw_kernel(const float *__restrict__ in, int HW, int Cpi,
                                                           const float *__restrict__ w, int ldw, int Cout,
                                                           const float *__restrict__ scale,
                                                           const float *__restrict__ shift, int relu, long long npix,
                                                           float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float wl[64 * 4 * CIN4];  // [co][ci]
    __shared__ float ss[2 * 64];
    const int tid = threadIdx.x;
    for (int e = tid; e < Cout * 4 * CIN4; e += 256) {
        const int co = e / (4 * CIN4), ci = e - co * (4 * CIN4);
        wl[e] = w[(size_t)ci * ldw + co];
    }
    for (int e = tid; e < Cout; e += 256) {
        ss[e] = scale[e];
        ss[64 + e] = shift[e];
    }
    __syncthreads();
    const long long pix = (long long)blockIdx.x * 256 + tid;
    if (pix >= npix) return;
    f32x4 xv[CIN4];
    const float *px = in + (size_t)pix * Cpi;
#pragma unroll
    for (int q = 0; q < CIN4; ++q) xv[q] = *reinterpret_cast<const f32x4 *>(px + 4 * q);
    const long long n = pix / HW, p = pix - n * HW;
    float *o = out + (size_t)n * Cout * HW + p;
    for (int co = 0; co < Cout; ++co) {
        const f32x4 *wr = reinterpret_cast<const f32x4 *>(wl + co * 4 * CIN4);
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < CIN4; ++q) {
            const f32x4 wv = wr[q];
#pragma unroll
            for (int k = 0; k < 4; ++k) acc = __builtin_fmaf(xv[q][k], wv[k], acc);
        }
        float v = acc * ss[co] + ss[64 + co];
        if (relu) v = fmaxf(v, 0.0f);
        o[(size_t)co * HW] = v;
    }
}

// P2PNet's tail in one launch (cnns_2d.py:178-180, 209): y = ReLU(BN(ConvTranspose2d(k 2, s 2)(x)))
// + skip, then the 1x1 output conv z = Wh y + b written NCHW.  The two-kernel path writes y
// (126 MB per 240 planes of 64^2 x 32) and reads it back for the head; here y lives in LDS only.
// Item = 32 input pixels of one row (-> 2 output rows x 64 pixels); 256 threads; each block walks
// items blockIdx.x, + gridDim.x, ... with the next item's loads in flight during this one's GEMMs
// (one item per block, loads then GEMMs, ran the launch at 92 us = the memory time plus the
// matrix-core time: blocks started together stay in step, profiles/round6/up2_head/):
//   0. x [32 px][Cpi] and the item's skip [2 rows][64 px][32] -> LDS (16-B loads, branch-free so
//      all are in flight at once), channels permuted to [s][kq][c4] (c = 16 s + 4 c4 + kq) so
//      that one ds_read_b128 gives a lane the 4 channels of 4 successive v_mfma_f32_16x16x4f32
//   1. GEMM [32 px] x [Cpi] x [4 classes x 32 co] on the matrix cores: wave w owns pixel tile
//      w & 1 and column tiles 4 (w >> 1) .. + 3; the weights' B fragments (wd: [Cpi/16][4 kq]
//      [128 n][4 c4], n = (2 ry + rx) 32 + co) loaded once per block for the first 4 K steps
//   2. epilogue: * scale + shift, ReLU, + the staged skip -> y, in place in LDS
//   3. head GEMM [128 out px] x [32] x [16] (wh: [2][4 kq][16 j][4 c4]), * hscale + hshift
//   4. z through LDS to rows of 64 contiguous floats per plane
constexpr int kUpY = 36;    // y LDS pitch (conflict-free b128 reads)
constexpr int kUpZ = 132;   // z LDS pitch
__host__ __device__ constexpr int up2_x_pitch(int Cpi) { return Cpi + 4; }
__host__ __device__ constexpr int up2_lds_floats(int Cpi) { return 32 * up2_x_pitch(Cpi) + 128 * kUpY + 16 * kUpZ; }
__global__ __launch_bounds__(256) void up2_head_nchw_kernel(const float *__restrict__ in, int N, int H, int W,
                                                            int Cpi, const float *__restrict__ wd,
                                                            const float *__restrict__ scale,
                                                            const float *__restrict__ shift,
                                                            const float *__restrict__ skip, int Cps, int Cs,
                                                            const float *__restrict__ wh,
                                                            const float *__restrict__ hscale,
                                                            const float *__restrict__ hshift, int J,
                                                            float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int XP = up2_x_pitch(Cpi);
    float *const xl = lds, *const yl = lds + 32 * XP, *const zl = yl + 128 * kUpY;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, cm = lane >> 4;
    const int segs = W >> 5, items = N * H * segs;
    const int Ho = 2 * H, Wo = 2 * W;
    const int nq = Cpi >> 2, nx = 32 * nq;  // nx <= 1024
    const int mt = wave & 1, nt0 = (wave >> 1) * 4;
    const int ks = Cpi >> 4;
    // the block's constants: the first KB K steps' weight fragments (in registers: 80.5 us against
    // 86-87.5 for loading them per item at 3 blocks per CU), BN and head scales
    constexpr int KB = 4;
    f32x4 bw[4][4];
#pragma unroll
    for (int s = 0; s < KB; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
            bw[s][i] = *reinterpret_cast<const f32x4 *>(
                wd + (((size_t)min(s, ks - 1) * 4 + cm) * 128 + 16 * (nt0 + i) + l16) * 4);
    f32x4 hw2[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) hw2[s] = *reinterpret_cast<const f32x4 *>(wh + ((s * 4 + cm) * 16 + l16) * 4);
    float sc[4], sh[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int co = (16 * (nt0 + i) + l16) & 31;
        sc[i] = scale[co];
        sh[i] = shift[co];
    }
    const float hs = hscale[min(l16, J - 1)], hb = hshift[min(l16, J - 1)];

    // an item's loads go out one item ahead of its GEMMs (two ahead, in a second register set,
    // measured no faster: 82.5 vs 80.1 us)
    auto load = [&](int item, f32x4 (&xv)[4], f32x4 (&sv)[4]) {
        // every address clamped into the tensors, values selected at the LDS writes
        const int xs = item % segs, yy = (item / segs) % H, n = item / (segs * H);
        const float *__restrict__ src = in + (((size_t)n * H + yy) * W + xs * 32) * Cpi;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = min(tid + 256 * u, nx - 1);
            const int px = e / nq, q = e - px * nq;
            xv[u] = *reinterpret_cast<const f32x4 *>(src + (size_t)px * Cpi + 4 * q);
            const int e2 = tid + 256 * u, qo = e2 >> 3, p4 = min(e2 & 7, (Cs - 1) >> 2);  // (a quad that exists)
            const int oy = 2 * yy + (qo >> 6), ox = 64 * xs + (qo & 63);
            sv[u] = *reinterpret_cast<const f32x4 *>(skip + (((size_t)n * Ho + oy) * Wo + ox) * Cps + 4 * p4);
        }
    };
    auto body = [&](int item, f32x4 (&xv)[4], f32x4 (&sv)[4]) {
        // 0. this item's loads -> LDS, then the next item's loads go out
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = tid + 256 * u;
            if (e < nx) {
                const int px = e / nq, q = e - px * nq;  // channels 4q + kq = (s = q >> 2, c4 = q & 3, kq)
                float *d = xl + px * XP + (q >> 2) * 16 + (q & 3);
#pragma unroll
                for (int kq = 0; kq < 4; ++kq) d[kq * 4] = xv[u][kq];
            }
            const int qo = e >> 3, p4 = e & 7;
            float *d = yl + qo * kUpY + (p4 >> 2) * 16 + (p4 & 3);
#pragma unroll
            for (int kq = 0; kq < 4; ++kq) d[kq * 4] = 4 * p4 + kq < Cs ? sv[u][kq] : 0.0f;
        }
        __syncthreads();  // (B1) x and skip staged; the last item's stores have read z
        const int xs = item % segs, yy = (item / segs) % H, n = item / (segs * H);
        if (item + (int)gridDim.x < items) load(item + gridDim.x, xv, sv);
        // 1. the deconvolution GEMM
        f32x4 acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        auto step = [&](int s, const f32x4 (&bv)[4]) {
            const f32x4 av = *reinterpret_cast<const f32x4 *>(xl + (16 * mt + l16) * XP + s * 16 + cm * 4);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[k], bv[i][k], acc[i], 0, 0, 0);
        };
#pragma unroll
        for (int s = 0; s < KB; ++s)
            if (s < ks) step(s, bw[s]);
        for (int s = KB; s < ks; ++s) {
            f32x4 bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                bv[i] = *reinterpret_cast<const f32x4 *>(wd + (((size_t)s * 4 + cm) * 128 + 16 * (nt0 + i) + l16) * 4);
            step(s, bv);
        }
        // 2. BN, ReLU, + skip -> y[q][co] in place, q = 64 ry + 2 px + rx
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int nn = 16 * (nt0 + i) + l16, cls = nn >> 5, co = nn & 31;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int px = 16 * mt + 4 * cm + r;
                float *yp = yl + (64 * (cls >> 1) + 2 * px + (cls & 1)) * kUpY + (co >> 4) * 16 + (co & 3) * 4 +
                            ((co >> 2) & 3);
                *yp = fmaxf(acc[i][r] * sc[i] + sh[i], 0.0f) + *yp;
            }
        }
        __syncthreads();  // (B2) y complete; x read
        // 3. the head: wave w owns output-pixel tiles 2w, 2w + 1
        f32x4 z[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f32x4 av =
                    *reinterpret_cast<const f32x4 *>(yl + (16 * (2 * wave + h) + l16) * kUpY + s * 16 + cm * 4);
#pragma unroll
                for (int k = 0; k < 4; ++k) z[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[k], hw2[s][k], z[h], 0, 0, 0);
            }
        if (l16 < J) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int r = 0; r < 4; ++r) zl[l16 * kUpZ + 16 * (2 * wave + h) + 4 * cm + r] = z[h][r] * hs + hb;
        }
        __syncthreads();  // (B3) z complete; y read
        // 4. NCHW rows: plane j, output rows 2yy, 2yy + 1, columns 64 xs .. 64 xs + 63
        for (int e = tid; e < J * 128; e += 256) {
            const int j = e >> 7, q = e & 127;
            out[(((size_t)n * J + j) * Ho + 2 * yy + (q >> 6)) * Wo + 64 * xs + (q & 63)] = zl[j * kUpZ + q];
        }
    };
    f32x4 xv[4], sv[4];
    if ((int)blockIdx.x < items) load(blockIdx.x, xv, sv);
    for (int item = blockIdx.x; item < items; item += gridDim.x) body(item, xv, sv);
}

}  // namespace fvp

namespace fvp {
// Launch plan of one convolution: the halo-tiled kernel's tile (0: not used)
// or the per-tap kernel's tile and its split-K factor.
struct ConvPlan {
    int halo;   // 1/3/5 = TileN16/N32/N64 (2/4/6/7 small tiles when forced), 0 = per-tap kernel
    int tile;   // per-tap tile id 1..7 (kTileBM / kTileBN)
    int ks;     // split-K factor of the per-tap kernel (1 = none)
};

static const int kTileBM[8] = {0, 256, 64, 128, 64, 128, 64, 32};
static const int kTileBN[8] = {0, 16, 16, 32, 32, 64, 64, 64};

// Geometry of one launch, validated: the GEMM row grid (Hm x Wm) and the
// output image (Ho x Wo).
struct ConvGeom {
    int mode, sy, sx, py, px, Hm, Wm, Ho, Wo;
};

static int conv_geom(int H, int W, int Cpi, int KH, int KW, int mode, int sy, int sx, int py, int px, ConvGeom &g) {
    if (H <= 0 || W <= 0 || KH <= 0 || KW <= 0 || Cpi <= 0 || Cpi % 4 || (Cpi > 16 && Cpi % 16)) return FVP_ERR_SHAPE;
    g = ConvGeom{mode, sy, sx, py, px, H, W, H, W};
    if (mode == 0) {
        if (sy < 1 || sx < 1 || sy > 4 || sx > 4 || py < 0 || px < 0 || py >= KH || px >= KW) return FVP_ERR_SHAPE;
        g.Hm = g.Ho = (H + 2 * py - KH) / sy + 1;
        g.Wm = g.Wo = (W + 2 * px - KW) / sx + 1;
        if (H + 2 * py < KH || W + 2 * px < KW) return FVP_ERR_SHAPE;
        return FVP_OK;
    }
    g.sy = g.sx = 1;
    g.py = g.px = 0;
    if (mode == 1 || mode == 2) {
        if (KH != 1 || KW != 1) return FVP_ERR_SHAPE;
        g.Ho = mode == 1 ? 2 * H : H;
        g.Wo = 2 * W;
        return FVP_OK;
    }
    if (mode == 3) {  // ConvTranspose2d(4, 2, 1): 2x2 taps per output parity
        if (KH != 2 || KW != 2) return FVP_ERR_SHAPE;
        g.Ho = 2 * H;
        g.Wo = 2 * W;
        return FVP_OK;
    }
    return FVP_ERR_SHAPE;
}

static ConvPlan conv_plan(int N, int Cpi, int KH, int KW, int Ntot, const ConvGeom &g, int algo) {
    ConvPlan p{0, 0, 1};
    const int G = conv_groups(g.mode);
    const long long M = (long long)N * g.Hm * g.Wm;
    const long long enough = 512;  // >= 2 blocks per CU
    // Halo tiles are 16 pixels wide: only where a row wastes <= 1/8 of them
    // (CenterNet's 20- and 40-wide maps stay per-tap), and only with the large
    // tiles (>= 8 rows: halo overhead <= 1.4x of the tile) at >= 2 blocks per
    // CU -- measured (profiles/round1/conv_probe.txt): 7x7 front 205 -> 147 us, 3x3
    // layers at 64/32 px 4-6 % faster; 4-row tiles and sub-2-per-CU launches
    // were 2-10 % slower than per-tap.  Stride-1 "same" convolutions only.
    const int W = g.Wm, H = g.Hm;
    const int tx = (W + 15) / 16;
    const bool same = g.mode == 0 && g.sy == 1 && g.sx == 1 && 2 * g.py == KH - 1 && 2 * g.px == KW - 1;
    const bool halo = (algo == FVP_CONV_AUTO || algo == FVP_CONV_HALO) && same && Cpi % 16 == 0 &&
                      (KH > 1 || KW > 1) && KH <= 7 && KW <= 7 && W >= 16 && (tx * 16 - W) * 8 <= W;
    auto hblocks = [&](int id) {
        const int rows = kTileBM[id] / 16;
        return (long long)N * tx * ((H + rows - 1) / rows) * ((Ntot + kTileBN[id] - 1) / kTileBN[id]);
    };
    if (halo) {
        const bool any = algo == FVP_CONV_HALO;  // every eligible layer, small tiles too
        const int big = Ntot <= 16 ? 1 : Ntot <= 32 ? 3 : 5;
        if (hblocks(big) >= enough) p.halo = big;
        else if (any) p.halo = big == 5 ? (hblocks(6) >= enough ? 6 : 7) : big + 1;
        if (p.halo) return p;
    }
    auto blocks = [&](int id) {
        return G * ((M + kTileBM[id] - 1) / kTileBM[id]) * (long long)((Ntot + kTileBN[id] - 1) / kTileBN[id]);
    };
    if (Ntot <= 16) p.tile = blocks(1) >= enough ? 1 : 2;
    else if (Ntot <= 32) p.tile = blocks(3) >= enough ? 3 : 4;
    else p.tile = blocks(5) >= enough ? 5 : blocks(6) >= enough ? 6 : 7;
    // Split-K for launches under one block per CU with a long K walk (CenterNet's
    // 20x20 / 40x40 levels at small batch, the deep ResNet stages): each K-chunk
    // step waits on a global round trip, so fewer, longer block chains leave the
    // CUs idle (CenterNet on 8 frames 0.61 -> 0.55 ms; C2CNet's 1-D rows were
    // slower split).
    const int nchunks = conv_krows(KH, KW, Cpi) / 16;
    const long long nb = blocks(p.tile);
    if (algo != FVP_CONV_PER_TAP_NOSPLIT && g.Hm > 1 && nb < 256 && nchunks >= 8) {  // 2-D maps only
        int ks = (int)((512 + nb - 1) / nb);
        ks = ks < nchunks / 4 ? ks : nchunks / 4;
        p.ks = ks < 8 ? ks : 8;
        if (p.ks < 2) p.ks = 1;
    }
    return p;
}

static size_t conv_ws_bytes(int N, int Cpi, int KH, int KW, int Cpo, const ConvGeom &g, int algo) {
    const int Ntot = conv_cols(g.mode, Cpo);
    const ConvPlan p = conv_plan(N, Cpi, KH, KW, Ntot, g, algo);
    return p.ks > 1 ? (size_t)conv_groups(g.mode) * p.ks * N * g.Hm * g.Wm * Ntot * sizeof(float) : 0;
}

// bf16 flags: FVP_CONV_BF16 (operands), FVP_CONV_BF16_IN / _OUT (activations stored as bf16;
// the output's residuals likewise) -- the last two only with bf16 operands.
static int conv_launch(const float *in, int N, int H, int W, int Cpi, const void *wpack, int KH, int KW, int Cpo,
                       int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                       const float *res_post, int relu, const ConvGeom &g, float *out, int bf16, int algo, void *ws,
                       size_t ws_bytes, void *stream) {
    if (bf16 & ~(FVP_CONV_BF16 | FVP_CONV_BF16_IN | FVP_CONV_BF16_OUT | FVP_CONV_F32_KC)) return FVP_ERR_SHAPE;
    if ((bf16 & (FVP_CONV_BF16_IN | FVP_CONV_BF16_OUT)) && !(bf16 & FVP_CONV_BF16)) return FVP_ERR_SHAPE;
    if ((bf16 & FVP_CONV_F32_KC) && (bf16 & FVP_CONV_BF16)) return FVP_ERR_SHAPE;
    if (!in || !wpack || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || Cpo <= 0 || Cpo % 16) return FVP_ERR_SHAPE;
    if (algo < FVP_CONV_AUTO || algo > FVP_CONV_PER_TAP_NOSPLIT) return FVP_ERR_SHAPE;
    const int Ntot = conv_cols(g.mode, Cpo);
    if (Cpo_w < Ntot || Cpo_w % 128) return FVP_ERR_SHAPE;
    const long long M = (long long)N * g.Hm * g.Wm;
    if ((long long)N * g.Ho * g.Wo * Cpo > 0x7fffffffLL * 4 || (long long)N * H * W * Cpi > 0x7fffffffLL * 4)
        return FVP_ERR_SHAPE;
    const int G = conv_groups(g.mode);
    fvp::ConvArgs a{in, reinterpret_cast<const float *>(wpack), scale, shift, res_pre, res_post, out, N, H, W, Cpi,
                    KH, KW, Cpo, Cpo_w, relu, g.mode, g.Hm, g.Wm, g.sy, g.sx, g.py, g.px, 1, nullptr,
                    (bf16 & FVP_CONV_BF16_IN) ? 1 : 0, (bf16 & FVP_CONV_BF16_OUT) ? 1 : 0};
    hipStream_t st = (hipStream_t)stream;
    // LDS-DMA kernel: one K step = one tap x a 128-B (or 64-B) row of channels
    const int es = (bf16 & FVP_CONV_BF16) ? 2 : 4;
    const long long Kd = (long long)KH * KW * Cpi;
    const bool fits = (long long)N * H * W * Cpi * es < (1LL << 31) && (long long)Cpo_w * Kd * es < (1LL << 31) &&
                      KH * KW <= 32 && M < (1 << 24);  // 32-bit buffer offsets, tap masks, row decode
    auto dma = [&](auto f32) {
        constexpr bool F = decltype(f32)::value;
        constexpr int E = F ? 4 : 2;
        // 32-column tiles (4 waves of 32 x 32) for the <= 32-channel layers, 128-B rows only.
        // fp32 takes 64-column tiles where bf16 takes 128: 4 waves and 48 KB of LDS per
        // block, 3 blocks per CU instead of 2 of 8 waves -- PoseResNet-50 fp32 layers
        // 31.02 -> 30.53 ms (3x3/s2 512->512 at 32 x 60: 0.85 -> 0.73 ms, the 1x1
        // expand layers 3-7 %; profiles/round6/dma_bn64/)
        const int BN = Ntot > 64 ? (F ? 64 : 128) : (Ntot > 32 || Cpi * E % 128) ? 64 : 32;
        const dim3 gr((unsigned)((M + 127) / 128), (unsigned)((Ntot + BN - 1) / BN), (unsigned)G);
        if (BN == 32) {
            hipLaunchKernelGGL((fvp::conv_dma_kernel<32, 128 / E, 4, F>), gr, dim3(256), 0, st, a, wpack);
        } else if (Cpi * E % 128 == 0) {  // 128-B rows
            if (BN == 128) hipLaunchKernelGGL((fvp::conv_dma_kernel<128, 128 / E, 8, F>), gr, dim3(512), 0, st, a, wpack);
            else hipLaunchKernelGGL((fvp::conv_dma_kernel<64, 128 / E, 4, F>), gr, dim3(256), 0, st, a, wpack);
        } else {  // 64-B rows (32 bf16 / 16 fp32 channels)
            if (BN == 128) hipLaunchKernelGGL((fvp::conv_dma_kernel<128, 64 / E, 8, F>), gr, dim3(512), 0, st, a, wpack);
            else hipLaunchKernelGGL((fvp::conv_dma_kernel<64, 64 / E, 4, F>), gr, dim3(256), 0, st, a, wpack);
        }
        return (int)hipGetLastError();
    };
    if (bf16 & FVP_CONV_F32_KC) {  // fp32 operands, weights [G][Cpo_w][Krows]: the DMA kernel or nothing
        if (Cpi % 16 || !fits) return FVP_ERR_SHAPE;
        return dma(std::true_type{});
    }
    if (bf16) {  // chunks of one tap x 16 / 32 channels (or several taps of a 4/8/12-channel input), no split
        if (Cpi % 16 && (bf16 & FVP_CONV_BF16_IN)) return FVP_ERR_SHAPE;
        const __bf16 *wb = reinterpret_cast<const __bf16 *>(wpack);
        // LDS-DMA kernel (measured against the register-staged one on ResNet-50
        // at 40 x 960 x 512: 3x3 64->64 0.21 -> 0.15 ms, deconv 256->256 at 64x120
        // 1.21 -> 0.76 ms, 1x1 256->1024 at 32x60 0.15 -> 0.11 ms; the 64->256
        // expand layers at 128x240 tie at 0.31 ms, output bound)
        if (a.in_bf16 && Cpi % 32 == 0 && algo != FVP_CONV_PER_TAP_NOSPLIT && fits) return dma(std::false_type{});
#define FVP_CONVB(BM, BN, WR, KC)                                                                               \
    do {                                                                                                          \
        const dim3 gr((unsigned)((M + BM - 1) / BM), (unsigned)((Ntot + BN - 1) / BN), (unsigned)G);             \
        if (a.in_bf16)                                                                                            \
            hipLaunchKernelGGL((fvp::conv_bf16_kernel<fvp::TileB<BM, BN, WR, KC>, true>), gr, dim3(256), 0, st, a, \
                               wb);                                                                               \
        else                                                                                                      \
            hipLaunchKernelGGL((fvp::conv_bf16_kernel<fvp::TileB<BM, BN, WR, KC>, false>), gr, dim3(256), 0, st,  \
                               a, wb);                                                                            \
    } while (0)
        const bool k32 = Cpi % 32 == 0;
        const long long b128 = G * ((M + 127) / 128) * ((Ntot + 63) / 64);
        if (Ntot <= 32) {
            if (k32) FVP_CONVB(128, 32, 4, 32); else FVP_CONVB(128, 32, 4, 16);
        } else if (b128 >= 512) {
            if (k32) FVP_CONVB(128, 64, 2, 32); else FVP_CONVB(128, 64, 2, 16);
        } else {
            if (k32) FVP_CONVB(64, 64, 2, 32); else FVP_CONVB(64, 64, 2, 16);
        }
#undef FVP_CONVB
        return (int)hipGetLastError();
    }
    ConvPlan p = conv_plan(N, Cpi, KH, KW, Ntot, g, algo);
    if (p.ks > 1 && (!ws || ws_bytes < (size_t)G * p.ks * M * Ntot * sizeof(float))) p.ks = 1;  // no scratch: no split
    if (p.ks > 1) {
        a.part = reinterpret_cast<float *>(ws);
        a.ks = p.ks;
    }
    if (p.halo) {
        const int tx = (W + 15) / 16;
#define FVP_HALO(TL)                                                                                              \
    do {                                                                                                          \
        const int ty = (H + fvp::TL::BM / 16 - 1) / (fvp::TL::BM / 16);                                           \
        const dim3 gr((unsigned)((long long)N * tx * ty), (unsigned)((Ntot + fvp::TL::BN - 1) / fvp::TL::BN));    \
        if (KH <= 3 && KW <= 3)                                                                                   \
            hipLaunchKernelGGL((fvp::conv_halo_kernel<fvp::TL, 3>), gr, dim3(256), 0, st, a, tx, ty);             \
        else                                                                                                      \
            hipLaunchKernelGGL((fvp::conv_halo_kernel<fvp::TL, 7>), gr, dim3(256), 0, st, a, tx, ty);             \
    } while (0)
        switch (p.halo) {
            case 1: FVP_HALO(TileN16); break;
            case 2: FVP_HALO(TileN16s); break;
            case 3: FVP_HALO(TileN32); break;
            case 4: FVP_HALO(TileN32s); break;
            case 5: FVP_HALO(TileN64); break;
            case 6: FVP_HALO(TileN64m); break;
            default: FVP_HALO(TileN64s); break;
        }
#undef FVP_HALO
        return (int)hipGetLastError();
    }
#define FVP_CONV(TL)                                                                                              \
    hipLaunchKernelGGL((fvp::conv_mfma_kernel<fvp::TL>),                                                          \
                       dim3((unsigned)((M + fvp::TL::BM - 1) / fvp::TL::BM),                                      \
                            (unsigned)((Ntot + fvp::TL::BN - 1) / fvp::TL::BN), (unsigned)(G * p.ks)),            \
                       dim3(256), 0, st, a)
#define FVP_CONV2(TL)                                                                                             \
    hipLaunchKernelGGL((fvp::conv_mfma_kernel<fvp::TL, 2>),                                                       \
                       dim3((unsigned)((M + fvp::TL::BM - 1) / fvp::TL::BM),                                      \
                            (unsigned)((Ntot + fvp::TL::BN - 1) / fvp::TL::BN), (unsigned)(G * p.ks)),            \
                       dim3(256), 0, st, a)
    // Measured per layer on CenterNet at 8 frames (rocprofv3 kernel traces,
    // profiles/round3/centernet_trace): 32-deep K chunks on the 64 x 32 tile
    // (3x3 32->32 at 80x80: 24-26 -> 21-24 us) and two chunks in flight on the
    // 64 x 16 tile (7x7 16->16 front: 46 -> 42.5 us); the same changes on the
    // 32 x 64 tile, a padded B pitch and an LDS-free wave-per-tile kernel were
    // neutral or slower.
    if (p.tile == 4 && Cpi % 32 == 0) {  // (a 32-deep chunk = 32 channels of one tap)
        FVP_CONV(TileN32sK);
    } else if (p.tile == 2) {
        FVP_CONV2(TileN16s);
    } else switch (p.tile) {  // (tile 2 took the branch above)
        case 1: FVP_CONV(TileN16); break;
        case 3: FVP_CONV(TileN32); break;
        case 4: FVP_CONV(TileN32s); break;
        case 5: FVP_CONV(TileN64); break;
        case 6: FVP_CONV(TileN64m); break;
        default: FVP_CONV(TileN64s); break;
    }
#undef FVP_CONV
#undef FVP_CONV2
    if (p.ks > 1) {
        const long long tot = G * M * Ntot;
        hipLaunchKernelGGL(fvp::conv_splitk_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, a, (int)M,
                           Ntot);
    }
    return (int)hipGetLastError();
}

// The stride-1 "same" convolutions and 2x transposed convolutions of the
// HDN / JLN CNNs (odd kernels, padding (K-1)/2).
static int legacy_geom(int H, int W, int Cpi, int KH, int KW, int upsample2, ConvGeom &g) {
    if (Cpi % 16 || (KH & 1) == 0 || (KW & 1) == 0 || upsample2 < 0 || upsample2 > 2) return FVP_ERR_SHAPE;
    return conv_geom(H, W, Cpi, KH, KW, upsample2, 1, 1, (KH - 1) / 2, (KW - 1) / 2, g);
}
}  // namespace fvp

extern "C" int fvp_conv2d_nhwc(const float *in, int N, int H, int W, int Cpi, const float *wpack, int KH, int KW,
                               int Cpo, int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                               const float *res_post, int relu, int upsample2, float *out, void *stream) {
    return fvp_conv2d_nhwc_ws(in, N, H, W, Cpi, wpack, KH, KW, Cpo, Cpo_w, scale, shift, res_pre, res_post, relu,
                              upsample2, out, FVP_CONV_AUTO, nullptr, 0, stream);
}

extern "C" size_t fvp_conv2d_workspace_bytes(int N, int H, int W, int Cpi, int KH, int KW, int Cpo, int upsample2,
                                             int algo) {
    fvp::ConvGeom g;
    if (N <= 0 || Cpo <= 0 || Cpo % 16 || algo < FVP_CONV_AUTO || algo > FVP_CONV_PER_TAP_NOSPLIT) return 0;
    if (fvp::legacy_geom(H, W, Cpi, KH, KW, upsample2, g) != FVP_OK) return 0;
    return fvp::conv_ws_bytes(N, Cpi, KH, KW, Cpo, g, algo);
}

extern "C" int fvp_conv2d_nhwc_ws(const float *in, int N, int H, int W, int Cpi, const float *wpack, int KH, int KW,
                                  int Cpo, int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                                  const float *res_post, int relu, int upsample2, float *out, int algo,
                                  void *workspace, size_t workspace_bytes, void *stream) {
    if (!in || !wpack || !scale || !shift || !out) return FVP_ERR_NULL;
    fvp::ConvGeom g;
    const int st = fvp::legacy_geom(H, W, Cpi, KH, KW, upsample2, g);
    if (st != FVP_OK) return st;
    return fvp::conv_launch(in, N, H, W, Cpi, wpack, KH, KW, Cpo, Cpo_w, scale, shift, res_pre, res_post, relu, g,
                            out, 0, algo, workspace, workspace_bytes, stream);
}

extern "C" int fvp_conv2d_nhwc_bf16(const float *in, int N, int H, int W, int Cpi, const void *wpack_bf16, int KH,
                                    int KW, int Cpo, int Cpo_w, const float *scale, const float *shift,
                                    const float *res_pre, const float *res_post, int relu, int upsample2, float *out,
                                    void *stream) {
    if (!in || !wpack_bf16 || !scale || !shift || !out) return FVP_ERR_NULL;
    fvp::ConvGeom g;
    const int st = fvp::legacy_geom(H, W, Cpi, KH, KW, upsample2, g);
    if (st != FVP_OK) return st;
    return fvp::conv_launch(in, N, H, W, Cpi, wpack_bf16, KH, KW, Cpo, Cpo_w, scale, shift, res_pre, res_post, relu,
                            g, out, FVP_CONV_BF16, FVP_CONV_AUTO, nullptr, 0, stream);
}

extern "C" int fvp_conv2d_geom(int H, int W, int Cpi, int KH, int KW, int mode, int sy, int sx, int py, int px,
                               int *out_hw) {
    fvp::ConvGeom g;
    const int st = fvp::conv_geom(H, W, Cpi, KH, KW, mode, sy, sx, py, px, g);
    if (st == FVP_OK && out_hw) {
        out_hw[0] = g.Ho;
        out_hw[1] = g.Wo;
    }
    return st;
}

extern "C" size_t fvp_conv2d_ex_workspace_bytes(int N, int H, int W, int Cpi, int KH, int KW, int Cpo, int mode,
                                                int sy, int sx, int py, int px, int algo) {
    fvp::ConvGeom g;
    if (N <= 0 || Cpo <= 0 || Cpo % 16 || algo < FVP_CONV_AUTO || algo > FVP_CONV_PER_TAP_NOSPLIT) return 0;
    if (fvp::conv_geom(H, W, Cpi, KH, KW, mode, sy, sx, py, px, g) != FVP_OK) return 0;
    return fvp::conv_ws_bytes(N, Cpi, KH, KW, Cpo, g, algo);
}

extern "C" int fvp_conv2d_nhwc_ex(const float *in, int N, int H, int W, int Cpi, const void *wpack, int KH, int KW,
                                  int Cpo, int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                                  const float *res_post, int relu, int mode, int sy, int sx, int py, int px,
                                  int bf16, int algo, float *out, void *workspace, size_t workspace_bytes,
                                  void *stream) {
    if (!in || !wpack || !scale || !shift || !out) return FVP_ERR_NULL;
    fvp::ConvGeom g;
    const int st = fvp::conv_geom(H, W, Cpi, KH, KW, mode, sy, sx, py, px, g);
    if (st != FVP_OK) return st;
    return fvp::conv_launch(in, N, H, W, Cpi, wpack, KH, KW, Cpo, Cpo_w, scale, shift, res_pre, res_post, relu, g,
                            out, bf16, algo, workspace, workspace_bytes, stream);
}

extern "C" int fvp_maxpool_pad_nhwc(const float *in, int N, int H, int W, int C, int K, int S, int P, float *out,
                                    void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 || K < 1 || S < 1 || P < 0 || 2 * P > K) return FVP_ERR_SHAPE;
    if (H + 2 * P < K || W + 2 * P < K) return FVP_ERR_SHAPE;
    const int Ho = (H + 2 * P - K) / S + 1, Wo = (W + 2 * P - K) / S + 1;
    const long long total = (long long)N * Ho * Wo * (C / 4);
    if (K == 3 && S == 2 && P == 1 && (long long)N * Ho <= 65535 && (long long)H * W * (C / 4) < 0x7fffffffLL) {
        const int row = Wo * (C / 4);
        hipLaunchKernelGGL(fvp::maxpool3s2_kernel, dim3((unsigned)((row + 255) / 256), (unsigned)(N * Ho)), dim3(256),
                           0, (hipStream_t)stream, reinterpret_cast<const float4 *>(in),
                           reinterpret_cast<float4 *>(out), H, W, C / 4, Ho, Wo);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(fvp::maxpool_pad_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, in, out, N, H, W, C, K, S, P, Ho, Wo);
    return (int)hipGetLastError();
}

extern "C" int fvp_maxpool_pad_nhwc_bf16(const void *in, int N, int H, int W, int C, int K, int S, int P, void *out,
                                         void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || K < 1 || S < 1 || P < 0 || 2 * P > K) return FVP_ERR_SHAPE;
    if (H + 2 * P < K || W + 2 * P < K) return FVP_ERR_SHAPE;
    const int Ho = (H + 2 * P - K) / S + 1, Wo = (W + 2 * P - K) / S + 1;
    const long long total = (long long)N * Ho * Wo * (C / 8);
    hipLaunchKernelGGL(fvp::maxpool_pad_bf16_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, reinterpret_cast<const uint4 *>(in), reinterpret_cast<uint4 *>(out), N, H,
                       W, C, K, S, P, Ho, Wo);
    return (int)hipGetLastError();
}

extern "C" int fvp_maxpool_nhwc_bf16(const void *in, int N, int H, int W, int C, int KH, int KW, void *out,
                                     void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (KH < 1 || KH > 2 || KW < 1 || KW > 2) return FVP_ERR_SHAPE;
    if (N <= 0 || H < KH || W < KW || C <= 0 || C % 8) return FVP_ERR_SHAPE;
    const long long total = (long long)N * (H / KH) * (W / KW) * (C / 8);
    const dim3 g((unsigned)((total + 255) / 256)), b(256);
    hipStream_t st = (hipStream_t)stream;
    const uint4 *i4 = reinterpret_cast<const uint4 *>(in);
    uint4 *o4 = reinterpret_cast<uint4 *>(out);
    if (KH == 2 && KW == 2) hipLaunchKernelGGL((fvp::maxpool_bf16_kernel<2, 2>), g, b, 0, st, i4, o4, N, H, W, C);
    else if (KH == 1 && KW == 2) hipLaunchKernelGGL((fvp::maxpool_bf16_kernel<1, 2>), g, b, 0, st, i4, o4, N, H, W, C);
    else if (KH == 2) hipLaunchKernelGGL((fvp::maxpool_bf16_kernel<2, 1>), g, b, 0, st, i4, o4, N, H, W, C);
    else hipLaunchKernelGGL((fvp::maxpool_bf16_kernel<1, 1>), g, b, 0, st, i4, o4, N, H, W, C);
    return (int)hipGetLastError();
}

extern "C" int fvp_maxpool_nhwc(const float *in, int N, int H, int W, int C, int KH, int KW, float *out,
                                void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (KH < 1 || KH > 2 || KW < 1 || KW > 2) return FVP_ERR_SHAPE;
    if (N <= 0 || H < KH || W < KW || C <= 0 || C % 4) return FVP_ERR_SHAPE;
    const long long total = (long long)N * (H / KH) * (W / KW) * (C / 4);
    const dim3 g((unsigned)((total + 255) / 256)), b(256);
    hipStream_t st = (hipStream_t)stream;
    if (KH == 2 && KW == 2) hipLaunchKernelGGL((fvp::maxpool_kernel<2, 2>), g, b, 0, st, in, out, N, H, W, C);
    else if (KH == 1 && KW == 2) hipLaunchKernelGGL((fvp::maxpool_kernel<1, 2>), g, b, 0, st, in, out, N, H, W, C);
    else if (KH == 2) hipLaunchKernelGGL((fvp::maxpool_kernel<2, 1>), g, b, 0, st, in, out, N, H, W, C);
    else hipLaunchKernelGGL((fvp::maxpool_kernel<1, 1>), g, b, 0, st, in, out, N, H, W, C);
    return (int)hipGetLastError();
}

extern "C" int fvp_maxpool2_nhwc(const float *in, int N, int H, int W, int C, float *out, void *stream) {
    return fvp_maxpool_nhwc(in, N, H, W, C, 2, 2, out, stream);
}

extern "C" int fvp_nchw_to_nhwc(const float *in, int N, int C, int H, int W, int Cp, float *out, void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (N <= 0 || C <= 0 || Cp < C || H <= 0 || W <= 0) return FVP_ERR_SHAPE;
    hipStream_t s = (hipStream_t)stream;
    // pitches of 4..32 channels (heatmaps: 16 * ceil(J / 16)): the voxelize layout
    // pass, one float4 per thread, a wave writing a contiguous 1 KiB run
    switch (Cp) {
        case 4: fvp::launch_layout<1, float>(in, N, 1, C, C, H, W, out, s); return (int)hipGetLastError();
        case 8: fvp::launch_layout<2, float>(in, N, 1, C, C, H, W, out, s); return (int)hipGetLastError();
        case 16: fvp::launch_layout<4, float>(in, N, 1, C, C, H, W, out, s); return (int)hipGetLastError();
        case 32: fvp::launch_layout<8, float>(in, N, 1, C, C, H, W, out, s); return (int)hipGetLastError();
        default: break;
    }
    const long long total = (long long)N * H * W * Cp;
    hipLaunchKernelGGL(fvp::nchw_to_nhwc_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, in, out, N, C,
                       H * W, Cp);
    return (int)hipGetLastError();
}

extern "C" int fvp_conv_stem7_bf16(const float *img, int N, int C, int H, int W, const void *wpack, const float *scale,
                                   const float *shift, void *out, void *stream) {
    if (!img || !wpack || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || C < 1 || C > 4 || H < 1 || W < 1) return FVP_ERR_SHAPE;
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;  // (H + 2*3 - 7) / 2 + 1
    const int tx = (Wo + fvp::kStemTW - 1) / fvp::kStemTW, ty = (Ho + fvp::kStemTH - 1) / fvp::kStemTH;
    if ((long long)N * tx * ty > 0x7fffffffLL) return FVP_ERR_SHAPE;
    const int ntiles = N * tx * ty;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int blocks = ntiles < 2 * cus ? ntiles : 2 * cus;  // persistent: 2 blocks per CU walk the tiles
    hipLaunchKernelGGL(fvp::conv_stem7_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, img, C,
                       H, W, Ho, Wo, tx, ty, ntiles, reinterpret_cast<const __bf16 *>(wpack), scale, shift,
                       reinterpret_cast<__bf16 *>(out));
    return (int)hipGetLastError();
}

extern "C" int fvp_conv_stem7_f32(const float *img, int N, int C, int H, int W, const float *wpack, const float *scale,
                                  const float *shift, float *out, void *stream) {
    if (!img || !wpack || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || C < 1 || C > 3 || H < 1 || W < 1) return FVP_ERR_SHAPE;
    if (((uintptr_t)wpack | (uintptr_t)scale | (uintptr_t)shift | (uintptr_t)out) & 15) return FVP_ERR_SHAPE;
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;  // (H + 2*3 - 7) / 2 + 1
    const int tx = (Wo + fvp::kS32TW - 1) / fvp::kS32TW, ty = (Ho + fvp::kS32TH - 1) / fvp::kS32TH;
    if ((long long)N * tx * ty > 0x7fffffffLL) return FVP_ERR_SHAPE;
    const int ntiles = N * tx * ty;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int blocks = ntiles < 2 * cus ? ntiles : 2 * cus;  // persistent: 2 blocks per CU walk the tiles
    hipLaunchKernelGGL(fvp::conv_stem7_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, img, C,
                       H, W, Ho, Wo, tx, ty, ntiles, wpack, scale, shift, out);
    return (int)hipGetLastError();
}

extern "C" int fvp_conv_front7_bf16(const float *x, int N, int C, int H, int W, const void *wpack,
                                    const float *scale, const float *shift, void *out, void *stream) {
    if (!x || !wpack || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || C < 1 || C > 16 || H < 1 || W < 1) return FVP_ERR_SHAPE;
    const int tx = (W + fvp::kFrTW - 1) / fvp::kFrTW, ty = (H + fvp::kFrTH - 1) / fvp::kFrTH;
    if ((long long)N * tx * ty > 0x7fffffffLL) return FVP_ERR_SHAPE;
    hipLaunchKernelGGL(fvp::conv_front7_bf16_kernel, dim3((unsigned)(N * tx * ty)), dim3(256), 0, (hipStream_t)stream,
                       x, C, H, W, tx, ty, reinterpret_cast<const __bf16 *>(wpack), scale, shift,
                       reinterpret_cast<__bf16 *>(out));
    return (int)hipGetLastError();
}

extern "C" int fvp_conv_front7_f32(const float *x, int N, int C, int H, int W, const float *wpack, const float *scale,
                                   const float *shift, float *out, void *stream) {
    if (!x || !wpack || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || C < 1 || C > 16 || H < 1 || W < 1) return FVP_ERR_SHAPE;
    const int tx = (W + fvp::kF32TW - 1) / fvp::kF32TW, ty = (H + fvp::kF32TH - 1) / fvp::kF32TH;
    if ((long long)N * tx * ty > 0x7fffffffLL) return FVP_ERR_SHAPE;
    const int ntiles = N * tx * ty;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int blocks = ntiles < 2 * cus ? ntiles : 2 * cus;  // persistent: 2 blocks per CU walk the tiles
    hipLaunchKernelGGL(fvp::conv_front7_f32_kernel, dim3((unsigned)blocks), dim3(256),
                       (size_t)fvp::kF32Lds * sizeof(float), (hipStream_t)stream, x, C, H, W, tx, ty, ntiles, wpack,
                       scale, shift, out);
    return (int)hipGetLastError();
}

extern "C" int fvp_nhwc_to_nchw(const float *in, int N, int C, int H, int W, int Cp, float *out, void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (N <= 0 || C <= 0 || Cp < C || H <= 0 || W <= 0) return FVP_ERR_SHAPE;
    const long long total = (long long)N * C * H * W;
    const int HW = H * W, tiles = (HW + 63) / 64;
    if (Cp % 4 == 0 && C <= 128 && (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (long long)N * tiles <= 0x7fffffffLL) {
        hipLaunchKernelGGL(fvp::nhwc_to_nchw_tiled_kernel, dim3((unsigned)(N * tiles)), dim3(256), 0,
                           (hipStream_t)stream, in, out, C, HW, Cp, tiles);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(fvp::nhwc_to_nchw_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, in, out, N, C, HW, Cp);
    return (int)hipGetLastError();
}

extern "C" int fvp_conv1x1_nchw(const float *in, int N, int H, int W, int Cpi, int Cin, const float *w, int ldw,
                                int Cout, const float *scale, const float *shift, int relu, float *out,
                                void *stream) {
    if (!in || !w || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cpi < Cin || Cpi % 4 || Cout <= 0 || Cout > 64 || ldw < Cout)
        return FVP_ERR_SHAPE;
    // float4s read per pixel: 4, 8 or 16 (<= the pitch); w holds that many rows, zero past Cin
    const int cin4 = (Cin + 3) / 4, t4 = cin4 <= 4 ? 4 : cin4 <= 8 ? 8 : 16;
    if (cin4 > 16 || 4 * t4 > Cpi || (reinterpret_cast<uintptr_t>(in) & 15)) return FVP_ERR_SHAPE;
    const long long npix = (long long)N * H * W;
    const dim3 g((unsigned)((npix + 255) / 256)), b(256);
    hipStream_t st = (hipStream_t)stream;
    auto go = [&](auto c) {
        hipLaunchKernelGGL(fvp::conv1x1_nchw_kernel<decltype(c)::value>, g, b, 0, st, in, H * W, Cpi, w, ldw, Cout,
                           scale, shift, relu, npix, out);
    };
    if (t4 == 4) go(std::integral_constant<int, 4>{});
    else if (t4 == 8) go(std::integral_constant<int, 8>{});
    else go(std::integral_constant<int, 16>{});
    return (int)hipGetLastError();
}

extern "C" int fvp_up2_head_nchw(const float *in, int N, int H, int W, int Cpi, const float *wd, const float *scale,
                                 const float *shift, const float *skip, int Cps, int Cs, const float *wh,
                                 const float *hscale, const float *hshift, int J, float *out, void *stream) {
    if (!in || !wd || !scale || !shift || !skip || !wh || !hscale || !hshift || !out) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || W % 32 || Cpi <= 0 || Cpi % 16 || Cpi > 128 || Cs <= 0 || Cs > 32 ||
        Cps < Cs || Cps % 4 || J <= 0 || J > 16 || (reinterpret_cast<uintptr_t>(in) & 15) ||
        (reinterpret_cast<uintptr_t>(skip) & 15))
        return FVP_ERR_SHAPE;
    const long long items = (long long)N * H * (W / 32);
    if (items > 0x7fffffffLL || (long long)N * J * 4 * H * W > (1LL << 40)) return FVP_ERR_SHAPE;
    // the blocks walk the items in turn: as many as are resident at once (VGPRs, LDS)
    const size_t lds = (size_t)fvp::up2_lds_floats(Cpi) * sizeof(float);
    int dev = 0, cus = 256, per_cu = 2;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fvp::up2_head_nchw_kernel, 256, lds) != hipSuccess ||
        per_cu <= 0)
        per_cu = 2;
    const long long slots = (long long)cus * per_cu;
    const long long blocks = items < slots ? items : slots;
    hipLaunchKernelGGL(fvp::up2_head_nchw_kernel, dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, in, N, H,
                       W, Cpi, wd, scale, shift, skip, Cps, Cs, wh, hscale, hshift, J, out);
    return (int)hipGetLastError();
}
