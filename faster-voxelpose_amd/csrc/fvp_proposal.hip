// Proposal selection on the 2-D detection map and the per-proposal gathers
// (A9, A10 of SURVEY.md §8(a)).
//
// The 3x3/stride-1/pad-1 max-pool keep mask (proposal.py:34-52) zeroes every
// element that is not its neighbourhood's maximum, then the top-K of the
// masked map is taken (proposal.py:73) in a total order -- value descending
// (NaN first, as torch.topk), then flat index ascending -- so the result is
// deterministic.  Indices decode as get_index2D does, dividing by
// shape[1] == X (proposal.py:27-29,75).
//
// nms_topk_small_kernel (K <= 16): one 1024-thread block per frame; each
// thread keeps a sorted register list of its elements' candidates, each wave
// extracts its top-K by K wave arg-max rounds (a 64-bit order key reduced
// over DPP), and one wave merges the per-wave lists the same way.
// nms_topk_kernel (K > 16): one 256-thread block per frame, the masked map in
// LDS, K block-wide arg-max rounds over a taken bitmap.
#include "fvp_device.h"

namespace fvp {

struct Cand {
    float v;
    int i;
};

// a precedes b: larger value first, then smaller index.  NaN sorts first, as
// torch.topk treats NaN as the largest value.
__device__ __forceinline__ bool before(const Cand &a, const Cand &b) {
    const bool an = a.v != a.v, bn = b.v != b.v;
    if (an != bn) return an;
    if (!an && a.v != b.v) return a.v > b.v;
    return a.i < b.i;
}

// The `before` order as one unsigned 64-bit key (larger = earlier): NaN
// highest, then float order (+-0 equal), then smaller index.  A wave arg-max
// is then a branch-free 64-bit max butterfly.
__device__ __forceinline__ unsigned long long cand_key(const Cand &c) {
    const unsigned u = c.v == 0.0f ? 0u : __builtin_bit_cast(unsigned, c.v);
    const unsigned ord = (c.v != c.v) ? 0xffffffffu : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
    return ((unsigned long long)ord << 32) | (unsigned)~(unsigned)c.i;
}

// one DPP step of the max reduction: lanes the control does not write keep
// their key (the move returns 0, the identity of the unsigned max)
template <int CTRL, int ROW_MASK, int BANK_MASK>
__device__ __forceinline__ unsigned long long dpp_max(unsigned long long k) {
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(k >> 32), CTRL, ROW_MASK, BANK_MASK, false);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)k, CTRL, ROW_MASK, BANK_MASK, false);
    const unsigned long long o = ((unsigned long long)hi << 32) | lo;
    return o > k ? o : k;
}

__device__ __forceinline__ Cand wave_best(Cand c) {
    // the wave64 DPP reduction (row_shr 1/2/3, 4 and 8 within rows of 16, then
    // row_bcast 15 / 31): lane 63 ends with the maximum key, read back as a scalar
    const unsigned long long own = cand_key(c);
    unsigned long long k = own;
    k = dpp_max<0x111, 0xf, 0xf>(k);
    k = dpp_max<0x112, 0xf, 0xf>(k);
    k = dpp_max<0x113, 0xf, 0xf>(k);
    k = dpp_max<0x114, 0xf, 0xe>(k);
    k = dpp_max<0x118, 0xf, 0xc>(k);
    k = dpp_max<0x142, 0xa, 0xf>(k);
    k = dpp_max<0x143, 0xc, 0xf>(k);
    const unsigned khi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(k >> 32), 63);
    const unsigned klo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)k, 63);
    k = ((unsigned long long)khi << 32) | klo;
    // the candidate itself comes from the lane holding the winning key (keys
    // are unique per element), so -0.0 and NaN payloads pass through unchanged
    // as in torch.topk
    const unsigned long long who = __builtin_amdgcn_ballot_w64(own == k);
    const int lane = who ? (int)__builtin_ctzll(who) : 0;
    Cand b;
    b.v = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, c.v), lane));
    b.i = __builtin_amdgcn_readlane(c.i, lane);
    return b;
}

constexpr int kNmsThreads = 256;

__global__ __launch_bounds__(kNmsThreads) void nms_topk_kernel(const float *__restrict__ prob, long long stride, int X,
                                                               int Y, int K,
                                                               float *__restrict__ vals, int64_t *__restrict__ flat,
                                                               int64_t *__restrict__ xy) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int M = X * Y;
    float *nmsv = reinterpret_cast<float *>(smem);                           // [M]
    unsigned *taken = reinterpret_cast<unsigned *>(smem + (size_t)M * 4);    // [ceil(M/32)]
    __shared__ Cand red[kNmsThreads / kWave];
    __shared__ Cand winner;
    const int b = blockIdx.x;
    const float *__restrict__ p = prob + (size_t)b * stride;
    const int tid = threadIdx.x;

    for (int e = tid; e < M; e += kNmsThreads) {
        const int ex = e / Y, ey = e - (e / Y) * Y;
        const float c = p[e];
        float m = -INFINITY;
        bool nan = false;
        for (int dx = -1; dx <= 1; ++dx) {
            const int xx = ex + dx;
            if (xx < 0 || xx >= X) continue;
            for (int dy = -1; dy <= 1; ++dy) {
                const int yy = ey + dy;
                if (yy < 0 || yy >= Y) continue;
                const float q = p[xx * Y + yy];
                nan |= (q != q);
                m = fmaxf(m, q);
            }
        }
        // max_pool2d propagates NaN; (c == NaN) is false -> keep = 0 -> 0*c.
        const float keep = (!nan && c == m) ? 1.0f : 0.0f;
        nmsv[e] = keep * c;
    }
    for (int w = tid; w < (M + 31) / 32; w += kNmsThreads) taken[w] = 0u;
    __syncthreads();

    for (int k = 0; k < K; ++k) {
        Cand best{-INFINITY, 0x7fffffff};
        bool have = false;
        for (int e = tid; e < M; e += kNmsThreads) {
            if (taken[e >> 5] & (1u << (e & 31))) continue;
            const Cand c{nmsv[e], e};
            if (!have || before(c, best)) {
                best = c;
                have = true;
            }
        }
        if (!have) best = Cand{-INFINITY, 0x7fffffff};
        best = wave_best(best);
        if ((tid & 63) == 0) red[tid >> 6] = best;
        __syncthreads();
        if (tid == 0) {
            Cand w = red[0];
            for (int i = 1; i < kNmsThreads / kWave; ++i)
                if (before(red[i], w)) w = red[i];
            winner = w;
            if (w.i < M) taken[w.i >> 5] |= (1u << (w.i & 31));
            vals[(size_t)b * K + k] = w.v;
            flat[(size_t)b * K + k] = w.i;
            if (xy) {
                xy[((size_t)b * K + k) * 2 + 0] = (int64_t)(w.i / X);
                xy[((size_t)b * K + k) * 2 + 1] = (int64_t)(w.i % X);
            }
        }
        __syncthreads();
    }
}

// Fast path for K <= 16: one NT-thread block per frame.  The map is staged
// in LDS with unrolled (8 loads in flight per thread) coalesced reads, each
// thread evaluates the 3x3 peak mask branch-free for its elements and keeps a
// sorted top-KMAX in registers (KMAX >= min(K, elements per thread)); each
// wave then extracts its top-K with K shuffle arg-max rounds and one wave
// merges the per-wave lists the same way (no block-wide rounds, no rescans).
template <int KMAX, int NT>
__global__ __launch_bounds__(NT) void nms_topk_small_kernel(const float *__restrict__ prob, long long stride, int X,
                                                            int Y, int K, float *__restrict__ vals,
                                                            int64_t *__restrict__ flat, int64_t *__restrict__ xy) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *map = reinterpret_cast<float *>(smem);  // [X*Y]
    __shared__ Cand wtop[NT / kWave][16];  // each wave's top-K (K <= 16)
    const int M = X * Y;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const float *__restrict__ p = prob + (size_t)b * stride;
    constexpr int U = 8;
    for (int e0 = tid; e0 < M; e0 += NT * U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = (e0 + u * NT < M) ? p[e0 + u * NT] : 0.0f;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (e0 + u * NT < M) map[e0 + u * NT] = v[u];
    }
    __syncthreads();

    Cand top[KMAX];
#pragma unroll
    for (int t = 0; t < KMAX; ++t) top[t] = Cand{-INFINITY, 0x7fffffff};
    int have = 0;
    for (int e = tid; e < M; e += NT) {
        const int ex = e / Y, ey = e - (e / Y) * Y;
        const float c = map[e];
        float m = -INFINITY;
        bool nan = false;
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy) {
                const int xx = ex + dx, yy = ey + dy;
                const bool ok = (unsigned)xx < (unsigned)X && (unsigned)yy < (unsigned)Y;
                const float q = map[ok ? xx * Y + yy : e];  // max_pool2d's -inf padding: out-of-map taps ignored
                nan |= ok && (q != q);
                m = ok ? fmaxf(m, q) : m;
            }
        }
        // max_pool2d propagates NaN; (c == NaN) is false -> keep = 0 -> 0*c.
        Cand cand{((!nan && c == m) ? 1.0f : 0.0f) * c, e};
        // sorted insertion (descending by `before`), fully unrolled: registers only
#pragma unroll
        for (int t = 0; t < KMAX; ++t) {
            if (t >= have || before(cand, top[t])) {
                const Cand tmp = top[t];
                top[t] = cand;
                cand = tmp;
            }
        }
        have = have < KMAX ? have + 1 : KMAX;
    }
    // merge, level 1: each wave's top-K by K rounds of wave arg-max over its
    // lanes' heads (shuffles only, no barriers); the winning lane pops its head
    const int lane = tid & 63, wave = tid >> 6;
    const Cand none{-INFINITY, 0x7fffffff};
    for (int k = 0; k < K; ++k) {
        const Cand head = have > 0 ? top[0] : none;
        const Cand best = wave_best(head);
        if (lane == 0) wtop[wave][k] = best;
        if (have > 0 && head.i == best.i) {  // indices are unique: exactly one lane pops
#pragma unroll
            for (int t = 0; t < KMAX - 1; ++t) top[t] = top[t + 1];
            top[KMAX - 1] = none;
            --have;
        }
    }
    __syncthreads();
    // level 2: wave 0 merges the NT/64 sorted lists the same way
    if (wave != 0) return;
    constexpr int PL = ((NT / kWave) * 16 + kWave - 1) / kWave;  // candidates per lane
    Cand l2[PL];
#pragma unroll
    for (int t = 0; t < PL; ++t) l2[t] = none;
    int h2 = 0;
    for (int c = lane; c < (NT / kWave) * K; c += kWave) {
        Cand cand = wtop[c / K][c - (c / K) * K];
#pragma unroll
        for (int t = 0; t < PL; ++t) {
            if (t >= h2 || before(cand, l2[t])) {
                const Cand tmp = l2[t];
                l2[t] = cand;
                cand = tmp;
            }
        }
        h2 = h2 < PL ? h2 + 1 : PL;
    }
    for (int k = 0; k < K; ++k) {
        const Cand head = h2 > 0 ? l2[0] : none;
        const Cand w = wave_best(head);
        if (lane == 0) {
            vals[(size_t)b * K + k] = w.v;
            flat[(size_t)b * K + k] = w.i;
            if (xy) {
                xy[((size_t)b * K + k) * 2 + 0] = (int64_t)(w.i / X);
                xy[((size_t)b * K + k) * 2 + 1] = (int64_t)(w.i % X);
            }
        }
        if (h2 > 0 && head.i == w.i) {
#pragma unroll
            for (int t = 0; t < PL - 1; ++t) l2[t] = l2[t + 1];
            l2[PL - 1] = none;
            --h2;
        }
    }
}

// columns[b,k,j,z] = cube[b,j,flat[b,k],z]; one thread per output element,
// z fastest so reads and writes are contiguous runs of Z floats.
__global__ __launch_bounds__(256) void gather_columns_kernel(const float *__restrict__ cube,
                                                             const int64_t *__restrict__ flat,
                                                             float *__restrict__ out, int J, int XY, int Z, int K,
                                                             long long total) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= total) return;
    const int z = (int)(gid % Z);
    long long r = gid / Z;
    const int j = (int)(r % J);
    r /= J;
    const int k = (int)(r % K);
    const long long b = r / K;
    const int64_t f = flat[b * K + k];
    out[gid] = cube[((b * J + j) * XY + f) * Z + z];
}

__global__ __launch_bounds__(256) void gather_bbox_kernel(const float *__restrict__ size,
                                                          const int64_t *__restrict__ flat, float *__restrict__ out,
                                                          int XY, int K, long long total) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= total) return;
    const int c = (int)(gid & 1);
    const long long bk = gid >> 1;
    const long long b = bk / K;
    out[gid] = size[(b * 2 + c) * XY + flat[bk]];
}

}  // namespace fvp

extern "C" int fvp_nms_topk(const float *prob, int B, int X, int Y, long long frame_stride, int K, float *vals,
                            int64_t *flat, int64_t *xy, void *stream) {
    if (!prob || !vals || !flat) return FVP_ERR_NULL;
    if (B <= 0 || X <= 0 || Y <= 0 || K <= 0 || K > X * Y) return FVP_ERR_SHAPE;
    const size_t M = (size_t)X * Y;
    const size_t lds = M * 4 + ((M + 31) / 32) * 4;
    if (lds > 150 * 1024) return FVP_ERR_SHAPE;
    if (frame_stride == 0) frame_stride = (long long)M;
    if (frame_stride < (long long)M) return FVP_ERR_SHAPE;
    if (K <= 16) {
        // per-thread list: every element a thread owns when that is <= 8 (then the
        // list holds them all; 80x80 maps: 7), else the top 16
        if ((M + 1023) / 1024 <= 8)
            hipLaunchKernelGGL((fvp::nms_topk_small_kernel<8, 1024>), dim3(B), dim3(1024), M * 4,
                               (hipStream_t)stream, prob, frame_stride, X, Y, K, vals, flat, xy);
        else
            hipLaunchKernelGGL((fvp::nms_topk_small_kernel<16, 1024>), dim3(B), dim3(1024), M * 4,
                               (hipStream_t)stream, prob, frame_stride, X, Y, K, vals, flat, xy);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(fvp::nms_topk_kernel, dim3(B), dim3(fvp::kNmsThreads), lds, (hipStream_t)stream, prob,
                       frame_stride, X, Y, K, vals, flat, xy);
    return (int)hipGetLastError();
}

extern "C" int fvp_gather_columns(const float *cube, int B, int J, int X, int Y, int Z, const int64_t *flat, int K,
                                  float *columns, void *stream) {
    if (!cube || !flat || !columns) return FVP_ERR_NULL;
    if (B <= 0 || J <= 0 || X <= 0 || Y <= 0 || Z <= 0 || K <= 0) return FVP_ERR_SHAPE;
    const long long total = (long long)B * K * J * Z;
    hipLaunchKernelGGL(fvp::gather_columns_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, cube, flat, columns, J, X * Y, Z, K, total);
    return (int)hipGetLastError();
}

extern "C" int fvp_gather_bbox(const float *size, int B, int X, int Y, const int64_t *flat, int K, float *out,
                               void *stream) {
    if (!size || !flat || !out) return FVP_ERR_NULL;
    if (B <= 0 || X <= 0 || Y <= 0 || K <= 0) return FVP_ERR_SHAPE;
    const long long total = (long long)B * K * 2;
    hipLaunchKernelGGL(fvp::gather_bbox_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, size, flat, out, X * Y, K, total);
    return (int)hipGetLastError();
}
