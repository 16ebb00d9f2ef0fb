// Dense 2-D convolutions of the HDN / JLN CNNs on the fp32 matrix cores
// (CenterNet cnns_2d.py:235-295, P2PNet :185-232,
// their Basic2DBlock / Res2DBlock / Upsample2DBlock / EncoderDecorder parts
// :12-183, and WeightNet's convolution, weight_net.py:48-80).
//
// Implicit GEMM, NHWC fp32 activations with channels padded to a multiple of
// 16 (padding channels hold zeros), out[m][co] = sum_k A[m][k] W[k][co] with
// m = (image, y, x) and k = ((ky*KW + kx)*Cp_in + ci).  v_mfma_f32_32x32x2_f32
// is an exact fp32 fma chain, so the only difference from torch's fp32 conv
// is the summation order.  Eval-mode BatchNorm is folded into a per-channel
// scale/shift (with the conv bias), and the epilogue fuses the residual add
// of Res2DBlock (before the ReLU), the ReLU, the decoder's skip add (after
// the ReLU) and, for ConvTranspose2d(k=2, s=2), the 2x upsampling scatter
// (the transposed conv is a 1x1 conv producing 4*Cout channels).
//
// Block = 256 threads (4 waves, 2x2), tile 64 pixels x 64 output channels,
// one 32x32 MFMA accumulator per wave; the K dimension is walked in chunks of
// 16 (one (ky,kx) tap, 16 input channels) staged through LDS, the next
// chunk's global loads issued before the current chunk's 8 MFMAs.
#include "fvp_device.h"

namespace fvp {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBM = 64, kBN = 64, kKC = 16, kAP = kKC + 1;  // A tile pitch 17: conflict-free column reads

struct ConvArgs {
    const float *in;        // [N][H][W][Cpi]
    const float *w;         // [KH*KW*Cpi][Cpo_w]  (Cpo_w = roundup(Cout_total, 64))
    const float *scale;     // [Cpo]  (per output channel)
    const float *shift;     // [Cpo]
    const float *res_pre;   // [N][Ho][Wo][Cpo] or null: added before the ReLU
    const float *res_post;  // [N][Ho][Wo][Cpo] or null: added after the ReLU
    float *out;             // [N][Ho][Wo][Cpo]
    int N, H, W, Cpi, KH, KW, Cpo, Cpo_w, relu, up2;
};

__device__ __forceinline__ void load_chunk(const ConvArgs &a, int m0, int n0, int chunk, int M, float4 &av,
                                           float4 &bv) {
    const int t = threadIdx.x;
    const int cpc = a.Cpi / kKC;  // chunks per tap
    const int tap = chunk / cpc, c = chunk - tap * cpc;
    const int ky = tap / a.KW, kx = tap - ky * a.KW;
    // A: thread -> (pixel t/4, 4 channels)
    {
        const int m = m0 + (t >> 2);
        av = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < M) {
            const int HW = a.H * a.W;
            const int img = m / HW, r = m - img * HW;
            const int y = r / a.W + ky - (a.KH - 1) / 2, x = r % a.W + kx - (a.KW - 1) / 2;
            if ((unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W)
                av = *reinterpret_cast<const float4 *>(a.in + (((size_t)img * a.H + y) * a.W + x) * a.Cpi + c * kKC +
                                                      (t & 3) * 4);
        }
    }
    // B: thread -> (k row t/16, 4 output columns)
    {
        const size_t row = (size_t)tap * a.Cpi + c * kKC + (t >> 4);
        bv = *reinterpret_cast<const float4 *>(a.w + row * a.Cpo_w + n0 + (t & 15) * 4);
    }
}

__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
    __shared__ float As[2][kBM * kAP];
    __shared__ __attribute__((aligned(16))) float Bs[2][kKC * kBN];
    const int M = a.N * a.H * a.W;
    const int m0 = blockIdx.x * kBM, n0 = blockIdx.y * kBN;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int nchunks = a.KH * a.KW * (a.Cpi / kKC);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;

    float4 av, bv;
    load_chunk(a, m0, n0, 0, M, av, bv);
    for (int ch = 0; ch < nchunks; ++ch) {
        const int buf = ch & 1;
        {
            float *ap = &As[buf][(t >> 2) * kAP + (t & 3) * 4];
            ap[0] = av.x; ap[1] = av.y; ap[2] = av.z; ap[3] = av.w;
            *reinterpret_cast<float4 *>(&Bs[buf][(t >> 4) * kBN + (t & 15) * 4]) = bv;
        }
        __syncthreads();
        if (ch + 1 < nchunks) load_chunk(a, m0, n0, ch + 1, M, av, bv);  // in flight during the MFMAs
        const float *Aw = &As[buf][(wm * 32 + (lane & 31)) * kAP + (lane >> 5)];
        const float *Bw = &Bs[buf][(lane >> 5) * kBN + wn * 32 + (lane & 31)];
#pragma unroll
        for (int kk = 0; kk < kKC / 2; ++kk)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Aw[2 * kk], Bw[2 * kk * kBN], acc, 0, 0, 0);
        // the next iteration writes the other buffer; the one after rewrites this
        // one only after its own barrier, which every wave reaches after these reads
    }

    // epilogue: lane -> column (output channel), registers -> 16 rows (pixels)
    const int n = n0 + wn * 32 + (lane & 31);
    const int Ctot = a.up2 ? 4 * a.Cpo : a.Cpo;
    if (n >= Ctot) return;
    const int co = a.up2 ? n % a.Cpo : n;
    const int q = a.up2 ? n / a.Cpo : 0;  // (dy, dx) of the transposed conv
    const float sc = a.scale[co], sh = a.shift[co];
    const int Ho = a.up2 ? 2 * a.H : a.H, Wo = a.up2 ? 2 * a.W : a.W;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= M) continue;
        size_t o;
        if (a.up2) {
            const int HW = a.H * a.W;
            const int img = m / HW, rr = m - img * HW;
            const int y = 2 * (rr / a.W) + (q >> 1), x = 2 * (rr % a.W) + (q & 1);
            o = (((size_t)img * Ho + y) * Wo + x) * a.Cpo + co;
        } else {
            o = (size_t)m * a.Cpo + co;
        }
        float v = acc[r] * sc + sh;
        if (a.res_pre) v = v + a.res_pre[o];
        if (a.relu) v = fmaxf(v, 0.0f);
        if (a.res_post) v = v + a.res_post[o];
        a.out[o] = v;
    }
}

// 2x2 / stride-2 max pool, NHWC (F.max_pool2d(x, 2, 2), cnns_2d.py Pool2DBlock)
__global__ __launch_bounds__(256) void maxpool2_kernel(const float *__restrict__ in, float *__restrict__ out, int N,
                                                       int H, int W, int C) {
    const int Ho = H / 2, Wo = W / 2;
    const long long total = (long long)N * Ho * Wo * (C / 4);
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int c4 = (int)(gid % (C / 4));
    long long r = gid / (C / 4);
    const int x = (int)(r % Wo);
    r /= Wo;
    const int y = (int)(r % Ho);
    const long long img = r / Ho;
    const float4 *p = reinterpret_cast<const float4 *>(in + (((size_t)img * H + 2 * y) * W + 2 * x) * C) + c4;
    const size_t rs = (size_t)W * C / 4;
    const float4 a = p[0], b = p[C / 4], c = p[rs], d = p[rs + C / 4];
    float4 m;
    m.x = nanmax(nanmax(a.x, b.x), nanmax(c.x, d.x));
    m.y = nanmax(nanmax(a.y, b.y), nanmax(c.y, d.y));
    m.z = nanmax(nanmax(a.z, b.z), nanmax(c.z, d.z));
    m.w = nanmax(nanmax(a.w, b.w), nanmax(c.w, d.w));
    reinterpret_cast<float4 *>(out)[gid] = m;
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

}  // namespace fvp

extern "C" int fvp_conv2d_nhwc(const float *in, int N, int H, int W, int Cpi, const float *wpack, int KH, int KW,
                               int Cpo, int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                               const float *res_post, int relu, int upsample2, float *out, void *stream) {
    if (!in || !wpack || !scale || !shift || !out) return FVP_ERR_NULL;
    if (N <= 0 || H <= 0 || W <= 0 || Cpi <= 0 || Cpi % 16 || Cpo <= 0 || Cpo % 16 || KH <= 0 || KW <= 0 ||
        (KH & 1) == 0 || (KW & 1) == 0)
        return FVP_ERR_SHAPE;
    const int Ntot = upsample2 ? 4 * Cpo : Cpo;
    if (Cpo_w < Ntot || Cpo_w % 64) return FVP_ERR_SHAPE;
    const long long M = (long long)N * H * W;
    if (M * (upsample2 ? 4 : 1) * Cpo > 0x7fffffffLL * 4) return FVP_ERR_SHAPE;
    fvp::ConvArgs a{in, wpack, scale, shift, res_pre, res_post, out, N, H, W, Cpi, KH, KW, Cpo, Cpo_w, relu, upsample2};
    const dim3 grid((unsigned)((M + fvp::kBM - 1) / fvp::kBM), (unsigned)((Ntot + fvp::kBN - 1) / fvp::kBN));
    hipLaunchKernelGGL(fvp::conv_mfma_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

extern "C" int fvp_maxpool2_nhwc(const float *in, int N, int H, int W, int C, float *out, void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (N <= 0 || H < 2 || W < 2 || C <= 0 || C % 4) return FVP_ERR_SHAPE;
    const long long total = (long long)N * (H / 2) * (W / 2) * (C / 4);
    hipLaunchKernelGGL(fvp::maxpool2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       in, out, N, H, W, C);
    return (int)hipGetLastError();
}

extern "C" int fvp_nchw_to_nhwc(const float *in, int N, int C, int H, int W, int Cp, float *out, void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (N <= 0 || C <= 0 || Cp < C || H <= 0 || W <= 0) return FVP_ERR_SHAPE;
    const long long total = (long long)N * H * W * Cp;
    hipLaunchKernelGGL(fvp::nchw_to_nhwc_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, in, out, N, C, H * W, Cp);
    return (int)hipGetLastError();
}

extern "C" int fvp_nhwc_to_nchw(const float *in, int N, int C, int H, int W, int Cp, float *out, void *stream) {
    if (!in || !out) return FVP_ERR_NULL;
    if (N <= 0 || C <= 0 || Cp < C || H <= 0 || W <= 0) return FVP_ERR_SHAPE;
    const long long total = (long long)N * C * H * W;
    hipLaunchKernelGGL(fvp::nhwc_to_nchw_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, in, out, N, C, H * W, Cp);
    return (int)hipGetLastError();
}
