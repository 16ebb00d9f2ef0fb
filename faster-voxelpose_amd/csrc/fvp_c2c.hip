// A whole 1-D network of the HDN in ONE launch: C2CNet (cnns_1d.py:182-241:
// Basic1DBlock / Res1DBlock / Pool1DBlock / Upsample1DBlock in the
// EncoderDecorder, eval BatchNorm folded) on the z-columns of the proposals
// (human_detection_net.py:199-205), SURVEY.md §8(f) rank 1.
//
// Per layer the generic engine (fvp_conv.hip) launches one implicit-GEMM
// kernel over rows of height 1: ~22 launches of 2-15 us for 0.4 GFLOP at C3
// B = 8 (80 columns of 15 x 20), each a latency-bound chain -- 0.21 ms even
// replayed from a hipGraph.  Here one block owns one column for the whole
// network: the activations ([C][L] per buffer, every buffer of the net) never
// leave LDS, and each layer's weights stream through LDS in chunks of input
// channels, the next chunk's 16-B loads in flight while the current one is
// multiplied (the only global traffic: the weights, from L2, once per block).
// The layer list is a program built on the host (fvp/cnn.py C2CProgram):
//   conv   out[co][l] = act(scale[co] * sum_{ci,t} W[ci][t][co] in[ci][l+t-p] + shift[co]
//                              (+ res_pre[co][l])) (+ res_post[co][l]),  p = (k-1)/2
//   convt  ConvTranspose1d(k = 2, s = 2): out[co][2l+d] = ... W[ci][d][co] in[ci][l] ...
//   pool   max_pool1d(2, 2), NaN-propagating in F.max_pool1d's window order
// Exact fp32 products and sums (fma-free: -ffp-contract=off), summed over
// (ci, t) in order -- an order of its own, like every fp32 kernel here.
#include "fvp_layout.h"

namespace fvp {

// one op of the program: 12 ints
struct C2COp {
    int kind;   // 0 conv, 1 convt (k 2, s 2), 2 pool (2, 2)
    int cin, cout, k, L;  // L = input length
    int src, dst, res_pre, res_post;  // activation buffer ids (-1: none)
    int relu;
    int w_off;  // params offset (floats, % 4 == 0): W [cin][k][cout], then scale [cout], shift [cout]
    int cic;    // input channels per staged weight chunk (% 4 == 0, cic * k * cout <= the chunk size)
};
static_assert(sizeof(C2COp) == 12 * sizeof(int), "C2COp layout");

constexpr int kC2CThreads = 1024;
// Weight chunk buffers (two): wchunk floats each, a multiple of kC2CStageFloats up to
// kC2CMaxStage of them -- 12,288 (48 KB) unless the activations need the room (C5's
// Z = 64 columns: 8,192).  The split-K partial sums take kC2CThreads * LG floats.
constexpr int kC2CStageFloats = 4 * kC2CThreads;  // one float4 load per thread
constexpr int kC2CMaxStage = 3;

// Activation rows in LDS are padded: [C][3 zeros, L values, 3 zeros] (pitch L + 6),
// so a tap outside the row reads a zero and the products need no guards.
constexpr int kC2CPad = 3;

// Thread layout of one conv: items (co, position group g) = cout x groups, each
// with KS threads splitting the input channels (4-channel steps interleaved),
// thread t = ks * items + item, so consecutive lanes hold consecutive co.
__device__ __forceinline__ int c2c_splits(int items, int cin) {
    int ks = 1;
    while (ks < 4 && items * ks * 2 <= kC2CThreads && cin >= 4 * ks * 2) ks *= 2;
    return ks;
}

// The products of one weight chunk for this thread's item: K, the convt flag
// and LG compile-time, so the unrolled (ci, t, j) body is straight FMAs on
// registers: 4 (2 for K >= 5) input channels per step, their (LG + K - 1)
// inputs and K weights loaded together.
template <int K, bool CT, int LG>
__device__ __forceinline__ void c2c_products(const C2COp &op, const float *__restrict__ in,
                                             const float *__restrict__ wl, int ci0, int nci, int co, int g, int ks,
                                             int KS, float (&acc)[LG]) {
    constexpr int PAD = CT ? 0 : (K - 1) / 2;
    constexpr int NX = CT ? LG / 2 : LG + K - 1;  // inputs per item and channel
    constexpr int U = K >= 5 ? 2 : 4;              // channels per step (registers: 128 at 1,024 threads)
    const int Lp = op.L + 2 * kC2CPad, cout = op.cout;
    const int x0 = kC2CPad + (CT ? g * (LG / 2) : g * LG - PAD);
    for (int ci = U * ks; ci < nci; ci += U * KS) {
        float xv[U][NX], wv[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float *xr = in + (ci0 + ci + u) * Lp + x0;
#pragma unroll
            for (int q = 0; q < NX; ++q) xv[u][q] = xr[q];
#pragma unroll
            for (int t = 0; t < K; ++t) wv[u][t] = wl[((ci + u) * K + t) * cout + co];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int t = 0; t < K; ++t)
#pragma unroll
                for (int jj = 0; jj < LG; ++jj) {
                    if (CT) {  // output 2l + d takes tap d of input l
                        if ((jj & 1) == t) acc[jj] = acc[jj] + wv[u][t] * xv[u][jj >> 1];
                    } else {
                        acc[jj] = acc[jj] + wv[u][t] * xv[u][jj + t];
                    }
                }
    }
}

template <int LG>
__device__ __forceinline__ void c2c_conv(const C2COp &op, const float *__restrict__ in, const float *__restrict__ wl,
                                         int ci0, int nci, int co, int g, int ks, int KS, float (&acc)[LG]) {
    if (op.kind == 1) c2c_products<2, true, LG>(op, in, wl, ci0, nci, co, g, ks, KS, acc);
    else if (op.k == 1) c2c_products<1, false, LG>(op, in, wl, ci0, nci, co, g, ks, KS, acc);
    else if (op.k == 3) c2c_products<3, false, LG>(op, in, wl, ci0, nci, co, g, ks, KS, acc);
    else if (op.k == 5) c2c_products<5, false, LG>(op, in, wl, ci0, nci, co, g, ks, KS, acc);
    else c2c_products<7, false, LG>(op, in, wl, ci0, nci, co, g, ks, KS, acc);
}

// one block per column; dynamic LDS: [2][wchunk] weights, the split partial sums
// [kC2CThreads * LG], then nbuf activation buffers of slot floats
template <int LG>
__global__ __launch_bounds__(kC2CThreads) void c2c_net_kernel(const float *__restrict__ x, int cin0, int L0,
                                                              const C2COp *__restrict__ prog, int nops,
                                                              const float *__restrict__ params, int slot, int nbuf,
                                                              int wchunk, int out_buf, int cout_final, int Lfinal,
                                                              float *__restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) float c2clds[];
    float *wbuf0 = c2clds, *wbuf1 = c2clds + wchunk, *red = c2clds + 2 * wchunk;
    float *act = red + kC2CThreads * LG;
    const int nstage = wchunk / kC2CStageFloats;
    const int tid = threadIdx.x, col = blockIdx.x;
    const int cin4 = (cin0 + 3) & ~3, Lp0 = L0 + 2 * kC2CPad;  // channels past cin0: zero rows
    for (int e = tid; e < cin4 * Lp0; e += kC2CThreads) {
        const int c = e / Lp0, q = e - c * Lp0 - kC2CPad;
        act[e] = (c < cin0 && q >= 0 && q < L0) ? x[((size_t)col * cin0 + c) * L0 + q] : 0.0f;
    }
    (void)nbuf;
    f32x4 st[kC2CMaxStage];
    auto chunk_floats = [&](const C2COp &q, int c) {
        return (c + 1 < (q.cin + q.cic - 1) / q.cic ? q.cic : q.cin - c * q.cic) * q.k * q.cout;
    };
    for (int o = 0; o < nops; ++o) {
        const C2COp op = prog[o];
        __syncthreads();  // the previous op's outputs are written
        const float *in = act + op.src * slot;
        float *out = act + op.dst * slot;
        if (op.kind == 2) {  // max_pool1d(2, 2): window (2l, 2l + 1), pads included
            const int Lo = op.L >> 1, Lpi = op.L + 2 * kC2CPad, Lpo = Lo + 2 * kC2CPad;
            for (int e = tid; e < op.cin * Lpo; e += kC2CThreads) {
                const int c = e / Lpo, l = e - c * Lpo - kC2CPad;
                const float *r = in + c * Lpi + kC2CPad;
                out[e] = (l >= 0 && l < Lo) ? nanmax(r[2 * l], r[2 * l + 1]) : 0.0f;
            }
            continue;
        }
        const int Lout = op.kind == 1 ? 2 * op.L : op.L;
        const int ngroups = (Lout + LG - 1) / LG, items = op.cout * ngroups;
        const int KS = c2c_splits(items, op.cic);
        const int ks = tid / items, item = tid - ks * items;
        const bool active = ks < KS;
        const int co = item % op.cout, g = item / op.cout;
        const float *__restrict__ W = params + op.w_off;
        const int nchunks = (op.cin + op.cic - 1) / op.cic;
        float acc[LG];
#pragma unroll
        for (int j = 0; j < LG; ++j) acc[j] = 0.0f;
        auto load_chunk = [&](int c) {
            const int n4 = chunk_floats(op, c) >> 2;
            const f32x4 *src = reinterpret_cast<const f32x4 *>(W + (size_t)c * op.cic * op.k * op.cout);
#pragma unroll
            for (int u = 0; u < kC2CMaxStage; ++u) {
                const int e = tid + kC2CThreads * u;
                if (u < nstage && e < n4) st[u] = src[e];
            }
        };
        auto store_chunk = [&](int c, float *dstw) {
            const int n4 = chunk_floats(op, c) >> 2;
#pragma unroll
            for (int u = 0; u < kC2CMaxStage; ++u) {
                const int e = tid + kC2CThreads * u;
                if (u < nstage && e < n4) reinterpret_cast<f32x4 *>(dstw)[e] = st[u];
            }
        };
        // (a prefetch of the next op's first chunk during this op measured slower: 142 -> 160 us)
        load_chunk(0);
        store_chunk(0, wbuf0);
        for (int c = 0; c < nchunks; ++c) {
            if (c + 1 < nchunks) load_chunk(c + 1);  // in flight during this chunk's products
            __syncthreads();                         // chunk c is in LDS (and the previous op's outputs)
            const int ci0 = c * op.cic, nci = op.cin - ci0 < op.cic ? op.cin - ci0 : op.cic;
            if (active) c2c_conv<LG>(op, in, (c & 1) ? wbuf1 : wbuf0, ci0, nci, co, g, ks, KS, acc);
            if (c + 1 < nchunks) store_chunk(c + 1, ((c + 1) & 1) ? wbuf1 : wbuf0);  // (buffer c - 1 is consumed)
        }
        if (KS > 1) {  // the splits' partial sums meet in LDS, added in split order
            if (active)
#pragma unroll
                for (int j = 0; j < LG; ++j) red[(ks * items + item) * LG + j] = acc[j];
            __syncthreads();
            if (ks == 0)
#pragma unroll
                for (int j = 0; j < LG; ++j) {
                    float v = red[item * LG + j];
                    for (int q = 1; q < KS; ++q) v = v + red[(q * items + item) * LG + j];
                    acc[j] = v;
                }
        }
        if (ks == 0) {
            const float *sc = W + op.cin * op.k * op.cout, *sh = sc + op.cout;
            const float *rpre = op.res_pre >= 0 ? act + op.res_pre * slot : nullptr;
            const float *rpost = op.res_post >= 0 ? act + op.res_post * slot : nullptr;
            const float sv = sc[co], bv = sh[co];
            const int row = co * (Lout + 2 * kC2CPad) + kC2CPad;
#pragma unroll
            for (int j = 0; j < LG; ++j) {
                const int lo = g * LG + j;
                if (lo >= Lout) continue;
                float v = acc[j] * sv + bv;
                if (rpre) v = v + rpre[row + lo];
                if (op.relu) v = fmaxf(v, 0.0f);
                if (rpost) v = v + rpost[row + lo];
                out[row + lo] = v;
            }
            if (g == 0)  // the row's zero pads (a buffer is reused at other lengths)
                for (int q = 1; q <= kC2CPad; ++q) out[row - q] = 0.0f;
            if (g == ngroups - 1)
                for (int q = 0; q < kC2CPad; ++q) out[row + Lout + q] = 0.0f;
        }
    }
    __syncthreads();
    const float *res = act + out_buf * slot;
    for (int e = tid; e < cout_final * Lfinal; e += kC2CThreads) {
        const int c = e / Lfinal, l = e - c * Lfinal;
        y[(size_t)col * cout_final * Lfinal + e] = res[c * (Lfinal + 2 * kC2CPad) + kC2CPad + l];
    }
}

}  // namespace fvp

extern "C" size_t fvp_conv1d_net_lds_bytes(int slot, int nbuf, int wchunk, int lg) {
    return (size_t)(2 * (size_t)wchunk + (size_t)fvp::kC2CThreads * lg + (size_t)slot * nbuf) * sizeof(float);
}

extern "C" int fvp_conv1d_net(const float *x, int ncols, int cin0, int L0, const int *prog, int nops,
                              const float *params, int slot, int nbuf, int wchunk, int out_buf, int cout_final,
                              int Lfinal, int lg, float *y, void *stream) {
    if (!x || !prog || !params || !y) return FVP_ERR_NULL;
    if (ncols <= 0 || cin0 <= 0 || L0 <= 0 || nops <= 0 || slot <= 0 || nbuf <= 0 || out_buf < 0 || out_buf >= nbuf ||
        cout_final <= 0 || Lfinal <= 0 || ((cin0 + 3) & ~3) * (L0 + 6) > slot || cout_final * (Lfinal + 6) > slot ||
        wchunk <= 0 || wchunk % fvp::kC2CStageFloats || wchunk > fvp::kC2CMaxStage * fvp::kC2CStageFloats)
        return FVP_ERR_SHAPE;
    if (lg != 4 && lg != 8) return FVP_ERR_SHAPE;
    const size_t lds = fvp_conv1d_net_lds_bytes(slot, nbuf, wchunk, lg);
    if (lds > 160 * 1024) return FVP_ERR_SHAPE;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g((unsigned)ncols), b(fvp::kC2CThreads);
    auto P = reinterpret_cast<const fvp::C2COp *>(prog);
    if (lg == 4)
        hipLaunchKernelGGL(fvp::c2c_net_kernel<4>, g, b, lds, s, x, cin0, L0, P, nops, params, slot, nbuf, wchunk,
                           out_buf, cout_final, Lfinal, y);
    else
        hipLaunchKernelGGL(fvp::c2c_net_kernel<8>, g, b, lds, s, x, cin0, L0, P, nops, params, slot, nbuf, wchunk,
                           out_buf, cout_final, Lfinal, y);
    return (int)hipGetLastError();
}
