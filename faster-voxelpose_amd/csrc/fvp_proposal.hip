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
// nms_select_kernel (K <= 16, X*Y <= 32640): one 1024-thread block per frame,
// the elements' 64-bit order keys in registers; a threshold from the wave
// maxima bounds the candidates, which are compacted and ranked (below).
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

// wave maximum of a 64-bit key, uniform in every lane
__device__ __forceinline__ unsigned long long wave_max_key(unsigned long long k) {
    k = dpp_max<0x111, 0xf, 0xf>(k);
    k = dpp_max<0x112, 0xf, 0xf>(k);
    k = dpp_max<0x113, 0xf, 0xf>(k);
    k = dpp_max<0x114, 0xf, 0xe>(k);
    k = dpp_max<0x118, 0xf, 0xc>(k);
    k = dpp_max<0x142, 0xa, 0xf>(k);
    k = dpp_max<0x143, 0xc, 0xf>(k);
    const unsigned khi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(k >> 32), 63);
    const unsigned klo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)k, 63);
    return ((unsigned long long)khi << 32) | klo;
}

constexpr int kSelThreads = 1024;
constexpr int kSelWaves = kSelThreads / kWave;  // 16 >= K
constexpr int kSelCap = 4096;                   // candidate list capacity
constexpr int kSelMaxE = 32;                    // elements per thread: maps up to 32768 (C5's 160 x 160)

// Element e of the masked map (max_pool2d 3x3/s1/p1 keep mask, proposal.py:34-52,
// 66-70): the value itself where it is its neighbourhood's maximum, else
// 0 * value (max_pool2d propagates NaN; NaN == m is false -> 0 * NaN).
// e / Y for 0 <= e < 2^16 without an integer division: a float estimate
// (off by at most one) and one correction step.
__device__ __forceinline__ int div_small(int e, int Y, float rY) {
    int q = (int)((float)e * rY);
    const int r = e - q * Y;
    q += (r >= Y) - (r < 0);
    return q;
}

__device__ __forceinline__ float masked_value(const float *map, int e, int X, int Y, float rY) {
    const int ex = div_small(e, Y, rY), ey = e - ex * Y;
    const float c = map[e];
    float m = -INFINITY;
    bool nan = false;
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx)
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy) {
            const int xx = ex + dx, yy = ey + dy;
            const bool ok = (unsigned)xx < (unsigned)X && (unsigned)yy < (unsigned)Y;
            const float q = map[ok ? xx * Y + yy : e];  // -inf padding: outside taps ignored
            nan |= ok && (q != q);
            m = ok ? fmaxf(m, q) : m;
        }
    return ((!nan && c == m) ? 1.0f : 0.0f) * c;
}

// Optionally fused with the column gather of the winners (cols != null:
// cols[b,k,j,:] = cube[b,j,flat[b,k],:], human_detection_net.py:199-200), so a
// frame's proposals and their z-columns come from one launch.
struct ColGather {
    const float *cube;  // [B][J][X*Y][Z]
    float *cols;        // [B][K][J][Z]
    int J, Z;
};

__device__ __forceinline__ void write_winner(int b, int K, int slot, int idx, float v, int X, float *__restrict__ vals,
                                             int64_t *__restrict__ flat, int64_t *__restrict__ xy, int *widx) {
    const size_t o = (size_t)b * K + slot;
    vals[o] = v;
    flat[o] = idx;
    widx[slot] = idx;
    if (xy) {
        xy[o * 2 + 0] = (int64_t)(idx / X);
        xy[o * 2 + 1] = (int64_t)(idx % X);
    }
}

// Top-K (K <= 16) of one frame's masked map by threshold selection, one
// 1024-thread block per frame, each thread owning E elements (e = tid + i*1024)
// as 64-bit order keys in registers (cand_key: NaN first, value descending,
// index ascending; every key of a real element is > 0; the masked values are
// recomputed from the staged map for the few candidates):
//   1. t = the K-th largest of the 64 16-lane row maxima.  Those K maxima are
//      distinct elements >= t, so at least K elements are >= t, and the top-K are
//      among the elements >= t.
//   2. the elements >= t are compacted into an LDS list by wave ballots (a map
//      typically has tens; an all-equal plateau at most 16*(K-1)+1 below the threshold row),
//   3. every listed candidate counts the listed keys above its own: that rank
//      is its output slot when < K.
// A list longer than kSelCap (only for adversarial value layouts) falls back
// to K block-wide extraction rounds of the largest key below the previous
// winner (no taken bitmap: keys are unique).
//
// STRIP (Y <= 1024, es = ceil(X / (1024 / Y)) <= E <= 16): the masked map is
// computed by column strips -- thread (xb, y) owns (xb*es .. xb*es + es - 1, y),
// so the 3x3 window maxima come from the row maxima of es + 2 rows: 3 LDS reads
// per element instead of 9, no index division (C3 / C2 frames: 4.6 -> ~2 us of
// a 1-CU launch) -- and written over the map in LDS; the keys are then read
// back with the element-per-thread mapping (tid + i*1024), whose wave maxima
// keep the candidate list short on plateaus (a masked map is mostly zeros:
// strip-wise wave maxima would admit thousands of zeros by index).  Otherwise
// thread tid computes its elements' masked values itself (masked_value).
template <int E, bool STRIP>
__global__ __launch_bounds__(kSelThreads) void nms_select_kernel(const float *__restrict__ prob, long long stride,
                                                                 int X, int Y, int K, int es,
                                                                 float *__restrict__ vals,
                                                                 int64_t *__restrict__ flat,
                                                                 int64_t *__restrict__ xy, ColGather cg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int M = X * Y;
    float *map = reinterpret_cast<float *>(smem);                                             // [M]
    unsigned long long *lkey = reinterpret_cast<unsigned long long *>(smem + (((size_t)M * 4 + 15) & ~(size_t)15));
    __shared__ unsigned long long wmax[kSelWaves];
    __shared__ unsigned long long gmax[4 * kSelWaves];  // maxima of the block's 16-lane rows
    __shared__ unsigned long long thr;
    __shared__ int count;
    __shared__ int widx[kSelWaves];  // winners' flat indices (K <= kSelWaves)
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float rY = 1.0f / (float)Y;
    const float *__restrict__ p = prob + (size_t)b * stride;
    {
        // all E loads in flight before the first LDS store (clamped addresses, no branches)
        float v[E];
#pragma unroll
        for (int i = 0; i < E; ++i) v[i] = p[min(tid + i * kSelThreads, M - 1)];
#pragma unroll
        for (int i = 0; i < E; ++i)
            if (tid + i * kSelThreads < M) map[tid + i * kSelThreads] = v[i];
    }
    if (tid == 0) {
        count = 0;
        thr = 0;  // stays 0 when fewer than K waves own elements
    }
    __syncthreads();

    unsigned long long key[E];
    unsigned long long best = 0;
    if constexpr (STRIP) {
        // the window maximum with NaN propagating (nanmax): NaN anywhere in the window makes c == m
        // false, as masked_value's nan flag does; otherwise m is its maximum (+-0 compare equal)
        const int xb = tid / Y, y = tid - xb * Y;
        const int x0 = xb * es;
        const bool act = xb < kSelThreads / Y;
        const int yl = y > 0 ? y - 1 : y, yr = y + 1 < Y ? y + 1 : y;  // (the centre stands in for a missing tap)
        // row r = x0 - 1 + r (clamped into the map; unused when outside): centre c and row maximum h,
        // a window of three rows rolled down the strip
        auto row_at = [&](int r, float &c, float &h) {
            const float *row = map + min(max(x0 - 1 + r, 0), X - 1) * Y;
            c = row[y];
            h = nanmax(nanmax(c, row[yl]), row[yr]);
        };
        float c0, h0, c1, h1, mv[E];
        row_at(0, c0, h0);
        row_at(1, c1, h1);
#pragma unroll
        for (int i = 0; i < E; ++i) {
            float c2, h2;
            row_at(i + 2, c2, h2);
            const int x = x0 + i;
            const float up = x > 0 ? h0 : h1, dn = x + 1 < X ? h2 : h1;
            const float m = nanmax(nanmax(h1, up), dn);
            mv[i] = (c1 == m ? 1.0f : 0.0f) * c1;
            h0 = h1;
            c1 = c2;
            h1 = h2;
        }
        __syncthreads();  // every window has read the raw map
#pragma unroll
        for (int i = 0; i < E; ++i)
            if (act && i < es && x0 + i < X) map[(x0 + i) * Y + y] = mv[i];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < E; ++i) {  // (E >= es >= ceil(M / 1024): every element has a slot)
            const int e = tid + i * kSelThreads;
            key[i] = e < M ? cand_key(Cand{map[e], e}) : 0ull;
            best = key[i] > best ? key[i] : best;
        }
    } else {
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int e = tid + i * kSelThreads;
            key[i] = e < M ? cand_key(Cand{masked_value(map, e, X, Y, rY), e}) : 0ull;
            best = key[i] > best ? key[i] : best;
        }
    }
    // the maxima of the 64 16-lane rows (DPP within rows: lane 15 of each row ends with its
    // row's maximum); the K-th largest of them is the threshold.  Rows rather than waves:
    // on a plateau of tied zeros the threshold is a zero's key, and the candidates are the
    // zeros of smaller index -- ~16 per row above it instead of ~64 per wave
    best = dpp_max<0x111, 0xf, 0xf>(best);
    best = dpp_max<0x112, 0xf, 0xf>(best);
    best = dpp_max<0x113, 0xf, 0xf>(best);
    best = dpp_max<0x114, 0xf, 0xe>(best);
    best = dpp_max<0x118, 0xf, 0xc>(best);
    if ((lane & 15) == 15) gmax[wave * 4 + (lane >> 4)] = best;
    __syncthreads();
    if (wave == 0) {
        const unsigned long long mine = gmax[lane];
        int rank = 0;
#pragma unroll 16
        for (int w = 0; w < 4 * kSelWaves; ++w) rank += gmax[w] > mine;
        if (rank == K - 1) thr = mine;
    }
    __syncthreads();
    const unsigned long long t = thr > 0 ? thr : 1ull;  // waves without elements hold the 0 sentinel

    // one LDS atomic per wave for all its candidates (the ballots first)
    int tot = 0;  // (the ballots are recomputed below rather than held: E of them would spill at E = 32)
#pragma unroll
    for (int i = 0; i < E; ++i) tot += (int)__builtin_popcountll(__builtin_amdgcn_ballot_w64(key[i] >= t));
    if (tot > 0) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&count, tot);
        base = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const unsigned long long bal = __builtin_amdgcn_ballot_w64(key[i] >= t);
            const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
            if (key[i] >= t && pos < kSelCap) lkey[pos] = key[i];
            base += (int)__builtin_popcountll(bal);
        }
    }
    __syncthreads();
    const int C = count;
    if (C <= kSelCap) {
        for (int c = tid; c < C; c += kSelThreads) {
            const unsigned long long k = lkey[c];
            // the list's keys 8 at a time, all 8 LDS reads in flight: on plateaus (a few
            // peaks on exact zeros, the threshold a zero's key) C reaches a few hundred and
            // one dependent read per key made this the kernel's longest phase
            int rank = 0, j = 0;
            for (; j + 8 <= C; j += 8) {
                unsigned long long q[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) q[u] = lkey[j + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) rank += q[u] > k;
            }
            for (; j < C; ++j) rank += lkey[j] > k;
            if (rank < K) {
                const int idx = (int)~(unsigned)k;
                write_winner(b, K, rank, idx, (STRIP ? map[idx] : masked_value(map, idx, X, Y, rY)), X, vals, flat, xy, widx);
            }
        }
    } else {  // K rounds, each the largest key below the previous winner
        unsigned long long prev = ~0ull;
        for (int r = 0; r < K; ++r) {
            unsigned long long mine = 0;
#pragma unroll
            for (int i = 0; i < E; ++i)
                if (key[i] < prev && key[i] > mine) mine = key[i];
            const unsigned long long wm = wave_max_key(mine);
            if (lane == 0) wmax[wave] = wm;
            __syncthreads();
            unsigned long long w = 0;
#pragma unroll
            for (int q = 0; q < kSelWaves; ++q) w = wmax[q] > w ? wmax[q] : w;
            if (tid == 0) {
                const int idx = (int)~(unsigned)w;
                write_winner(b, K, r, idx, (STRIP ? map[idx] : masked_value(map, idx, X, Y, rY)), X, vals, flat, xy, widx);
            }
            prev = w;
            __syncthreads();
        }
    }
    if (!cg.cols) return;
    __syncthreads();
    const int JZ = cg.J * cg.Z, KJZ = K * JZ;
    constexpr int CU = 4;  // column elements per thread in flight: the loads of a round issue together
    for (int e0 = tid; e0 < KJZ; e0 += CU * kSelThreads) {
        float cv[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            const int e = min(e0 + u * kSelThreads, KJZ - 1);
            const int k = e / JZ, r = e - k * JZ;
            const int j = r / cg.Z, z = r - j * cg.Z;
            cv[u] = cg.cube[(((size_t)b * cg.J + j) * M + widx[k]) * cg.Z + z];
        }
#pragma unroll
        for (int u = 0; u < CU; ++u)
            if (e0 + u * kSelThreads < KJZ) cg.cols[(size_t)b * KJZ + e0 + u * kSelThreads] = cv[u];
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
    // an index outside the map reads nothing and yields NaN (torch.gather raises)
    out[gid] = (f >= 0 && f < XY) ? cube[((b * J + j) * XY + f) * Z + z] : __builtin_nanf("");
}

__global__ __launch_bounds__(256) void gather_bbox_kernel(const float *__restrict__ size,
                                                          const int64_t *__restrict__ flat, float *__restrict__ out,
                                                          int XY, int K, long long total) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= total) return;
    const int c = (int)(gid & 1);
    const long long bk = gid >> 1;
    const long long b = bk / K;
    const int64_t f = flat[bk];
    out[gid] = (f >= 0 && f < XY) ? size[(b * 2 + c) * XY + f] : __builtin_nanf("");
}

// ProposalLayer.forward in test mode (human_detection_net.py:36-37, 99-124)
// fused with the z pick of HumanDetectionNet.forward (:208-215): per proposal
// z = argmax over the 1-D heatmap (topk(1): NaN first, then the largest value,
// lowest index on ties) and conf = conf_2d * hm1d[z] -- or, without a 1-D
// heatmap, z = index[...,2] and conf = conf_2d -- then centre = index * scale
// + bias (two fp32 ops, as torch), valid = (conf > min_score) - 1, bbox copied.
__global__ __launch_bounds__(256) void proposal_centers_kernel(const int64_t *__restrict__ index, int idims,
                                                               const float *__restrict__ hm1d,
                                                               const float *__restrict__ confs,
                                                               const float *__restrict__ bbox, int BK, int Z,
                                                               float3 scale, float3 bias, float min_score,
                                                               float *__restrict__ centers) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= BK) return;
    float conf = confs[t];
    float zi;
    if (hm1d) {
        const float *__restrict__ h = hm1d + (size_t)t * Z;
        Cand best{h[0], 0};
        for (int z = 1; z < Z; ++z) {
            const Cand c{h[z], z};
            if (before(c, best)) best = c;
        }
        conf = conf * best.v;
        zi = (float)best.i;
    } else {
        zi = (float)index[(size_t)t * idims + 2];
    }
    const float idx[3] = {(float)index[(size_t)t * idims + 0], (float)index[(size_t)t * idims + 1], zi};
    const float sc[3] = {scale.x, scale.y, scale.z}, bi[3] = {bias.x, bias.y, bias.z};
    float *__restrict__ o = centers + (size_t)t * 7;
#pragma unroll
    for (int a = 0; a < 3; ++a) o[a] = __fadd_rn(__fmul_rn(idx[a], sc[a]), bi[a]);
    o[3] = (conf > min_score ? 1.0f : 0.0f) - 1.0f;
    o[4] = conf;
    o[5] = bbox[(size_t)t * 2 + 0];
    o[6] = bbox[(size_t)t * 2 + 1];
}

}  // namespace fvp

namespace fvp {
static int nms_any(const float *prob, int B, int X, int Y, long long frame_stride, int K, float *vals, int64_t *flat,
                   int64_t *xy, const ColGather &cg, int Xc, int Yc, void *stream) {
    if (!prob || !vals || !flat) return FVP_ERR_NULL;
    if (B <= 0 || X <= 0 || Y <= 0 || K <= 0 || K > X * Y) return FVP_ERR_SHAPE;
    const size_t M = (size_t)X * Y;
    const size_t lds = M * 4 + ((M + 31) / 32) * 4;
    if (lds > 150 * 1024) return FVP_ERR_SHAPE;
    if (frame_stride == 0) frame_stride = (long long)M;
    if (frame_stride < (long long)M) return FVP_ERR_SHAPE;
    hipStream_t st = (hipStream_t)stream;
    const int E = (int)((M + kSelThreads - 1) / kSelThreads);
    const size_t sel_lds = ((M * 4 + 15) & ~(size_t)15) + (size_t)kSelCap * 8;
    if (K <= kSelWaves && E <= kSelMaxE && sel_lds <= 159 * 1024) {
        const dim3 g(B), blk(kSelThreads);
        // column strips when every column fits one thread row of the block and a strip <= 16
        const int nxb = Y <= kSelThreads ? kSelThreads / Y : 0;
        const int es = nxb ? (X + nxb - 1) / nxb : 0;
        auto go = [&](auto kernel, int e_arg) {
            hipLaunchKernelGGL(kernel, g, blk, sel_lds, st, prob, frame_stride, X, Y, K, e_arg, vals, flat, xy, cg);
        };
        if (nxb && es <= 16) {  // (strips of up to 16: at 32 the strip's values and keys spill)
            if (es <= 1) go(nms_select_kernel<1, true>, es);
            else if (es <= 2) go(nms_select_kernel<2, true>, es);
            else if (es <= 4) go(nms_select_kernel<4, true>, es);
            else if (es <= 8) go(nms_select_kernel<8, true>, es);
            else go(nms_select_kernel<16, true>, es);
        } else {
            if (E <= 1) go(nms_select_kernel<1, false>, 0);
            else if (E <= 2) go(nms_select_kernel<2, false>, 0);
            else if (E <= 4) go(nms_select_kernel<4, false>, 0);
            else if (E <= 8) go(nms_select_kernel<8, false>, 0);
            else if (E <= 16) go(nms_select_kernel<16, false>, 0);
            else go(nms_select_kernel<32, false>, 0);
        }
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(nms_topk_kernel, dim3(B), dim3(kNmsThreads), lds, st, prob, frame_stride, X, Y, K, vals, flat,
                       xy);
    if (cg.cols) {  // K > 16: the column gather as its own launch
        const long long total = (long long)B * K * cg.J * cg.Z;
        hipLaunchKernelGGL(gather_columns_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, cg.cube,
                           flat, cg.cols, cg.J, Xc * Yc, cg.Z, K, total);
    }
    return (int)hipGetLastError();
}
}  // namespace fvp

extern "C" int fvp_nms_topk(const float *prob, int B, int X, int Y, long long frame_stride, int K, float *vals,
                            int64_t *flat, int64_t *xy, void *stream) {
    return fvp::nms_any(prob, B, X, Y, frame_stride, K, vals, flat, xy, fvp::ColGather{nullptr, nullptr, 0, 0}, 0, 0,
                        stream);
}

extern "C" int fvp_nms_topk_columns(const float *prob, int B, int X, int Y, long long frame_stride, int K,
                                    float *vals, int64_t *flat, int64_t *xy, const float *cube, int J, int Z,
                                    float *columns, void *stream) {
    if (!cube || !columns) return FVP_ERR_NULL;
    if (J <= 0 || Z <= 0) return FVP_ERR_SHAPE;
    return fvp::nms_any(prob, B, X, Y, frame_stride, K, vals, flat, xy, fvp::ColGather{cube, columns, J, Z}, X, Y,
                        stream);
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

extern "C" int fvp_proposal_centers(const int64_t *index, int index_dims, const float *hm1d, const float *confs,
                                    const float *bbox, int B, int K, int Z, const float *scale3, const float *bias3,
                                    float min_score, float *centers, void *stream) {
    if (!index || !confs || !bbox || !scale3 || !bias3 || !centers) return FVP_ERR_NULL;
    if (B < 0 || K < 0 || (hm1d ? (index_dims != 2 || Z <= 0) : index_dims != 3)) return FVP_ERR_SHAPE;
    const int BK = B * K;
    if (BK == 0) return FVP_OK;
    hipLaunchKernelGGL(fvp::proposal_centers_kernel, dim3((unsigned)((BK + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, index, index_dims, hm1d, confs, bbox, BK, Z,
                       make_float3(scale3[0], scale3[1], scale3[2]), make_float3(bias3[0], bias3[1], bias3[2]),
                       min_score, centers);
    return (int)hipGetLastError();
}
