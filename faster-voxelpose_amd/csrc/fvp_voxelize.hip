// Whole-space voxelisation fused with the xy max-projection (A5-A7).
//
// Reference: project_whole.py:119-168 (grid_sample per frame, mean over all V
// cameras, clamp(0,1)) and cnns_2d.py:291 (max over z).
//
// Why a layout pass.  A bilinear tap of all J joints touches J separate
// [H][W] planes in the reference layout.  On gfx950 the texture addresser
// only merges ADJACENT lanes that fall in one 128-B line (a quad per clock);
// scattered per-joint taps cost ~64 clocks per wave load (tools/ta_probe.py),
// and a voxel-camera needs 2 rows x J planes of lines.  So each chunk of
// frames is first re-laid out, a pure streaming pass:
//   fp32: heatmaps_to_cl    [B][V][J][H][W] -> [b][V][H][W][JP] (JP = 4*LPV >= J, zero padded)
//         LPV lanes share one voxel; lane q loads 16 B = joints 4q..4q+3 of a
//         tap with one buffer_load_dwordx4, so a quad reads one 64-B pixel in
//         one clock: 4 loads per voxel-camera.
//   fp16: heatmaps_to_pairs [B][V][J][H][W] -> [b][V][H][W+1] 64-B entries
//         holding pixels x0 and x0+1 of a row (J <= 16): 2 loads per
//         voxel-camera, half the bytes through L1 (fp16 -> fp32 is exact).
// Out-of-image taps use an out-of-range offset and read 0 through the buffer
// descriptor's range check (= grid_sample's zero padding).  The chunk's copy
// stays in the 256 MB Infinity Cache between the two launches.
//
// Gather work decomposition: a 256-thread block owns COLS whole voxel columns
// (x, y..y+COLS, all z) of one frame -- a contiguous range of the cube --
// processed in passes of 256/LPV voxels; results are staged in LDS so the
// cube is written as contiguous runs per joint and the xy max over z is read
// back from LDS.  The sample grid is read voxel-major (fvp_pack_grid): each
// lane of a voxel group loads 2 cameras' coordinates with one 16-B load,
// computes their bilinear offsets/weights once, and the group picks them up
// per camera through lane broadcasts -- one grid load and one tap setup per
// 2*LPV voxel-cameras instead of per voxel-camera and lane.  Arithmetic per
// tap and the camera sum order are the reference's (fvp_device.h: torch's
// CPU mean over the views folds complete blocks of 16 cameras, CASC = V > 16),
// so the result is bit-exact.
#include <type_traits>

#include "fvp_layout.h"


namespace fvp {

// -- gather pass ----------------------------------------------------------------
// Where the sampling coordinates come from: a packed per-sequence grid
// (OTF = false), or the camera records, projected on the fly with the exact
// fp32 sequence of project_grid_kernel (OTF = true; used when the grid would
// not stay cache-resident, e.g. 31 cameras x 160x160x64 = 420 MB).
struct CoordSource {
    const float *grids;     // packed grids [S][N][GV][2]            (!OTF)
    const float *cams;      // camera records [S][V][FVP_CAM_STRIDE] (OTF)
    const float *resize_t;  // [2][3]                                (OTF)
    fvp_grid_spec gs;       // (OTF) the whole grid: x-row i of a launch is row x_off + i of gs
    ImageConsts im;
    int x_off;              // (OTF) first x-row of an x-slab launch (0: the whole grid)
};

// Epilogue of a gather block: the stage [NF][JP][SP] (clamped means, column-
// major within the block's columns) -> the cube runs and the xy max over z.
template <int NF, int JP>
__device__ __forceinline__ void store_stage(const float *__restrict__ stage, int SP, int T, int Z, long long N,
                                            long long n0, int c0, int ncols, int XY, int J, int Jst, int b,
                                            float *__restrict__ cube, float *__restrict__ xy, bool cube16) {
    // Epilogue.  When every run is 16-B aligned (T, SP, Z, N multiples of 4: the
    // C2 / C3 / C4 launches; cube16: the caller's cube pointer is 16-B aligned,
    // checked on the host) the cube goes out as float4 non-temporal stores and
    // the z-max reads 4 voxels per LDS load: a sixth of the store instructions
    // and independent LDS reads instead of a 20-long dependent chain
    // (tools/gather_probe.py FULL2: C2 8 frames 62.1 -> 59.8 us).
    const bool vec = ((T | SP | Z | (int)(N & 3)) & 3) == 0 && cube16;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        const float *fst = stage + f * JP * SP;
        const size_t bf = (size_t)(b + f);
        if (cube) {
            if (vec) {
                const int T4 = T >> 2;
                for (int e = threadIdx.x; e < J * T4; e += 256) {
                    const int j = e / T4, r = e - (e / T4) * T4;
                    const f32x4 v = *reinterpret_cast<const f32x4 *>(fst + j * SP + 4 * r);
                    __builtin_nontemporal_store(v, reinterpret_cast<f32x4 *>(cube + (bf * Jst + j) * N + n0) + r);
                }
            } else {
                for (int j = 0; j < J; ++j) {
                    float *__restrict__ dst = cube + (bf * Jst + j) * N + n0;
                    for (int e = threadIdx.x; e < T; e += 256) __builtin_nontemporal_store(fst[j * SP + e], dst + e);
                }
            }
        }
        if (xy) {
            for (int e = threadIdx.x; e < J * ncols; e += 256) {
                const int j = e / ncols, cc = e - (e / ncols) * ncols;
                const float *s = fst + j * SP + cc * Z;
                float m = -INFINITY;
                if (vec) {
                    const f32x4 *s4 = reinterpret_cast<const f32x4 *>(s);
#pragma unroll 4
                    for (int z = 0; z < (Z >> 2); ++z) {
                        const f32x4 v = s4[z];  // (torch.max's order is immaterial: max is exact, NaN wins)
                        m = nanmax(nanmax(m, v[0]), nanmax(nanmax(v[1], v[2]), v[3]));
                    }
                } else {
                    for (int z = 0; z < Z; ++z) m = nanmax(m, s[z]);
                }
                __builtin_nontemporal_store(m, xy + (bf * Jst + j) * XY + c0 + cc);
            }
        }
    }
}

template <int LPV, bool PAIR, bool OTF, bool CASC, int NF>
__device__ __forceinline__ void voxelize_body(const void *__restrict__ tab, const CoordSource &src_,
                                                       const int32_t *__restrict__ grid_index, int frame0,
                                                       float *__restrict__ cube, float *__restrict__ xy, int V, int J,
                                                       int Jst, int H, int W, int X, int Y, int Z, int cols,
                                                       int col_blocks, int SP, int band, unsigned pixb,
                                                       bool cube16) {
    static_assert(!PAIR || LPV == 4, "the fp16 pair table has 4 lanes per voxel");
    constexpr int JP = 4 * LPV;
    constexpr int VPP = 256 / LPV;  // voxels per pass
    constexpr int CPG = 2 * LPV;    // cameras per grid load (2 per lane)
    extern __shared__ __attribute__((aligned(16))) float stage[];  // [NF][JP][SP] (+ OTF camera records)
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int bl = L / col_blocks;   // frame group within the chunk (NF frames share each table entry)
    const int b = frame0 + bl * NF;  // first frame of the group within the batch (outputs, grid_index)
    const int XY = X * Y;
    int cb = L - bl * col_blocks;
    if (band > 0) {
        // bands of `band` x-rows walked column-group-major: consecutive blocks
        // (those resident together on an XCD) cover a compact x-y patch
        const int gpr = Y / cols;  // column groups per x-row (host: Y % cols == 0)
        const int per_band = band * gpr;
        const int bi = cb / per_band, r = cb - bi * per_band;
        const int rows = min(band, X - bi * band);
        const int gc = r / rows, xr = r - gc * rows;
        cb = (bi * band + xr) * gpr + gc;
    }
    const int c0 = cb * cols;  // the block's columns: c0 .. c0 + ncols - 1 (an x-row segment when banded)
    const int ncols = min(cols, XY - c0);
    const int T = ncols * Z;
    const long long N = (long long)XY * Z;
    const long long n0 = (long long)c0 * Z;
    const int q = threadIdx.x % LPV;
    const int GV = V + (V & 1);
    const unsigned qo = (unsigned)q * 16u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    const int gsel = grid_index ? grid_index[b] : 0;
    __amdgpu_buffer_rsrc_t grs;
    float *lcam = stage + ((NF * JP * SP + 3) & ~3);  // OTF: camera records [GV][FVP_CAM_STRIDE] after the stage
    float rt[6];
    if constexpr (OTF) {
        const float *cams = src_.cams + (size_t)gsel * V * FVP_CAM_STRIDE;
        for (int e = threadIdx.x; e < GV * FVP_CAM_STRIDE; e += 256) lcam[e] = e < V * FVP_CAM_STRIDE ? cams[e] : 0.0f;
#pragma unroll
        for (int k = 0; k < 6; ++k) rt[k] = src_.resize_t[k];
        __syncthreads();
    } else {
        grs = uniform_rsrc(src_.grids + (size_t)gsel * N * GV * 2, (unsigned)(N * GV * 8));
    }
    // per-camera image of this frame group in the workspace: each pixel / pair
    // entry holds the NF frames' copies back to back (one 128-B line at NF = 2)
    const unsigned pix = PAIR ? 64u : pixb;  // bytes of one frame's pixel (>= JP*4) / pair entry
    const unsigned unit = pix * NF;             // bytes per entry
    const unsigned img = (PAIR ? (unsigned)(H * (W + 1)) : (unsigned)(H * W)) * unit;  // bytes per camera
    const char *__restrict__ frame_tab = (const char *)tab + (size_t)bl * V * img;

    for (int i0 = 0; i0 < T; i0 += VPP) {
        const int i = i0 + threadIdx.x / LPV;
        const bool valid = i < T;
        // the slot's voxel, layer-major (a wave holds 16/ncols z-layers of all
        // the block's columns): column cl, layer zl; ii = its stage index
        // (column-major, as the cube), gn = its index in the cube
        const int sl = min(i, T - 1);
        const int zl = sl / ncols, cl = sl - zl * ncols;
        const int ii = cl * Z + zl;
        const long long gn = (long long)(c0 + cl) * Z + zl;
        float acc[NF][4], blk[NF][4];  // blk (CASC): completed 16-camera blocks (view_sum order)
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int m = 0; m < 4; ++m) acc[f][m] = blk[f][m] = 0.0f;
        float wx_ = 0.f, wy_ = 0.f, wz_ = 0.f;  // OTF: voxel centre (compute_grid, project_whole.py:43-79)
        if constexpr (OTF) {
            const int iz = zl;
            const long long r = c0 + cl;
            wx_ = axis_coord(src_.gs.start[0], src_.gs.end[0], src_.gs.bins[0], src_.x_off + (int)(r / Y),
                             src_.gs.center[0]);
            wy_ = axis_coord(src_.gs.start[1], src_.gs.end[1], Y, (int)(r % Y), src_.gs.center[1]);
            wz_ = axis_coord(src_.gs.start[2], src_.gs.end[2], Z, iz, src_.gs.center[2]);
        }
        for (int v0 = 0; v0 < V; v0 += CPG) {
            // cameras v0+2q, v0+2q+1 of voxel n0+ii (past V: padding, unused)
            float g[4];
            if constexpr (OTF) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const Cam c = load_cam(lcam + min(v0 + 2 * q + h, GV - 1) * FVP_CAM_STRIDE);
                    float px, py;
                    project_point(c, wx_, wy_, wz_, px, py);
                    pixel_to_sample(px, py, rt, src_.im, g[2 * h], g[2 * h + 1]);
                }
            } else {
                // slots v0+2q, v0+2q+1 (past the row: the next voxel's or 0)
                const u32x4 graw = __builtin_amdgcn_raw_buffer_load_b128(
                    grs, (unsigned)((gn * GV + v0 + 2 * q) * 8), 0, 0);
#pragma unroll
                for (int k = 0; k < 4; ++k) g[k] = __builtin_bit_cast(float, (unsigned)graw[k]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) g[k] = valid ? g[k] : -2.0f;
            const Taps4<PAIR> t0 = setup_taps<PAIR>(g[0], g[1], sxs, sys, W, H, unit);
            const Taps4<PAIR> t1 = setup_taps<PAIR>(g[2], g[3], sxs, sys, W, H, unit);
            static_for(std::make_integer_sequence<int, CPG>{}, [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = k >> 1;  // lane of the group that set this camera up
                const int v = v0 + k;
                if (v >= V) return;
                if constexpr (CASC) {
                    if ((v & 15) == 0 && v > 0) {  // a block of 16 cameras is complete: fold it (fvp_device.h)
#pragma unroll
                        for (int f = 0; f < NF; ++f)
#pragma unroll
                            for (int m = 0; m < 4; ++m) {
                                blk[f][m] = blk[f][m] + acc[f][m];
                                acc[f][m] = 0.0f;
                            }
                    }
                }
                const Taps4<PAIR> &src = (k & 1) ? t1 : t0;
                unsigned o[Taps4<PAIR>::NO];
                unsigned all = kOOB;
#pragma unroll
                for (int m = 0; m < Taps4<PAIR>::NO; ++m) {
                    o[m] = group_bcast<LPV, S>(src.o[m]);
                    all &= o[m];
                }
                // whole wave off-image (every tap's kOOB bit set): contributes exactly 0
                if (!__builtin_amdgcn_ballot_w64((all & kOOB) == 0u)) return;
                float w[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) w[m] = group_bcast<LPV, S>(src.w[m]);
                const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(frame_tab + (size_t)v * img, img);
                if constexpr (PAIR) {
                    // r0 = [a j0 j1 | a j2 j3 | b j0 j1 | b j2 j3] (row y0), r1 likewise (c, d; row y1)
                    u32x4 r0[NF], r1[NF];
#pragma unroll
                    for (int f = 0; f < NF; ++f) {
                        r0[f] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[0] + f * pix + qo, 0, 0);
                        r1[f] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[1] + f * pix + qo, 0, 0);
                    }
#pragma unroll
                    for (int f = 0; f < NF; ++f)
                        static_for(std::make_integer_sequence<int, 4>{}, [&](auto mc) {
                            constexpr int m = decltype(mc)::value, HI = m & 1;
                            const unsigned ua = r0[f][m >> 1], ub = r0[f][2 + (m >> 1)];
                            const unsigned uc = r1[f][m >> 1], ud = r1[f][2 + (m >> 1)];
                            // fd*w3 + (fc*w2 + (fb*w1 + fa*w0)), the fp16 taps converted inside the fmas
                            const float t = fma_h<HI>(ua, w[0], -0.0f);
                            acc[f][m] = acc[f][m] + fma_h<HI>(ud, w[3], fma_h<HI>(uc, w[2], fma_h<HI>(ub, w[1], t)));
                        });
                } else {
                    u32x4 a[NF], bq[NF], c[NF], d[NF];
#pragma unroll
                    for (int f = 0; f < NF; ++f) {
                        a[f] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[0] + f * pix + qo, 0, 0);
                        bq[f] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[1] + f * pix + qo, 0, 0);
                        c[f] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[2] + f * pix + qo, 0, 0);
                        d[f] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[3] + f * pix + qo, 0, 0);
                    }
#pragma unroll
                    for (int f = 0; f < NF; ++f)
#pragma unroll
                        for (int m = 0; m < 4; ++m) {
                            const float fa = __builtin_bit_cast(float, (unsigned)a[f][m]);
                            const float fb = __builtin_bit_cast(float, (unsigned)bq[f][m]);
                            const float fc = __builtin_bit_cast(float, (unsigned)c[f][m]);
                            const float fd = __builtin_bit_cast(float, (unsigned)d[f][m]);
                            acc[f][m] = acc[f][m] + __builtin_fmaf(fd, w[3], __builtin_fmaf(fc, w[2],
                                                                   __builtin_fmaf(fb, w[1], fa * w[0])));
                        }
                }
            });
        }
        // the sum's final levels (fvp_device.h): remainder + blocks, or + 0 (a -0 sum becomes +0)
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int m = 0; m < 4; ++m) acc[f][m] = acc[f][m] + (CASC ? blk[f][m] : 0.0f);
        if (valid) {
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    stage[(f * JP + 4 * q + m) * SP + ii] = clampf(acc[f][m] / fV, 0.0f, 1.0f);
        }
    }
    __syncthreads();
    store_stage<NF, JP>(stage, SP, T, Z, N, n0, c0, ncols, XY, J, Jst, b, cube, xy, cube16);
}

// The cube and xy plane are written with non-temporal stores: they are not
// re-read by this launch, and keeping them out of L2 leaves it to the taps
// (C2 -4 %, C4 -8 % gather time, measured).
// Cached-grid gather: <= 64 VGPRs so 8 waves/SIMD fit (32 waves/CU with the
// 20 KB stage); the on-the-fly variant keeps its registers (no spills).
template <int LPV, bool PAIR, bool OTF, bool CASC, int NF>
__global__ __launch_bounds__(256, NF == 1 ? 8 : NF == 2 ? 5 : 4) void voxelize_kernel(const void *__restrict__ tab, CoordSource src,
                                                          const int32_t *__restrict__ grid_index, int frame0,
                                                          float *__restrict__ cube, float *__restrict__ xy, int V,
                                                          int J, int Jst, int H, int W, int X, int Y, int Z,
                                                          int cols, int col_blocks, int SP, int band, unsigned pixb,
                                                          bool cube16) {
    static_assert(!OTF, "grid kernel");
    voxelize_body<LPV, PAIR, OTF, CASC, NF>(tab, src, grid_index, frame0, cube, xy, V, J, Jst, H, W, X, Y, Z, cols,
                                            col_blocks, SP, band, pixb, cube16);
}

template <int LPV, bool PAIR, bool OTF, bool CASC, int NF>
__global__ __launch_bounds__(256) void voxelize_cams_kernel(const void *__restrict__ tab, CoordSource src,
                                                            const int32_t *__restrict__ grid_index, int frame0,
                                                            float *__restrict__ cube, float *__restrict__ xy, int V,
                                                            int J, int Jst, int H, int W, int X, int Y, int Z,
                                                            int cols, int col_blocks, int SP, int band,
                                                            unsigned pixb, bool cube16) {
    static_assert(OTF, "on-the-fly kernel");
    voxelize_body<LPV, PAIR, OTF, CASC, NF>(tab, src, grid_index, frame0, cube, xy, V, J, Jst, H, W, X, Y, Z, cols,
                                            col_blocks, SP, band, pixb, cube16);
}

// [V][N][2] -> [N][GV][2], padding slots (-2,-2) (off-image)
__global__ __launch_bounds__(256) void pack_grid_kernel(const float2 *__restrict__ g, float2 *__restrict__ out, int V,
                                                        int GV, long long N) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= N * GV) return;
    const long long n = t / GV;
    const int v = (int)(t - n * GV);
    out[t] = v < V ? g[(size_t)v * N + n] : make_float2(-2.f, -2.f);
}

constexpr int kBandRows = 16;

// Cached-grid blocks of ~160 voxels at Z < 32 (C2 / C3: 8 columns of 20) and
// 256 from Z = 32 (C4: 8 of 32).  Measured on the same box against 320 / 200 /
// 100 (profiles/round3/block_voxels): C2 +2-3 %, C4 +2-5 % over 320 -- twice
// the blocks per chunk (6,400 at C2) leave a shorter last round on 2,048 block
// slots, and since the stage pitch keeps 16-B rows (stage_pitch) the smaller
// blocks keep the vector epilogue.  With layer-major slots C4 is 3-4 % faster
// at 8 columns than at 4 (a wave = 8 columns x 2 layers; 16: -13 %), C2 stays
// best at 8 (4: -11 %, 16: -3 %) (profiles/round3/slot_order/cols_sweep.txt).
static int cols_per_block(int Z) { return Z >= 256 ? 1 : Z >= 32 ? 256 / Z : 160 / Z; }

// LDS row pitch of the stage: padding against bank conflicts (a pitch of 0
// mod 32 dwords puts a voxel's 4 lanes on one bank), unless dropping it lets 8
// blocks (32 waves, full occupancy) share a CU's 160 KB.  When the block's
// voxel count is a multiple of 4 the pad is 4 floats, keeping the rows 16-B
// aligned for the vector epilogue (C4 / C5 / the one-frame launches, T = 256
// and 100: 2-way stage-write conflicts, as with the pad of 1).
static int stage_pitch(int LPV, int cols, int Z) {
    const int T = cols * Z;
    const int pad = T % 4 ? 1 : 4;
    const size_t padded = (size_t)16 * LPV * (T + pad), tight = (size_t)16 * LPV * T;
    return (padded > 20480 && tight <= 20480) ? T : T + pad;
}

static bool use_pairs(int J, bool half) { return half && J <= 16; }

// Frames per fp16 pair-table entry: 4 (two 128-B lines per entry), so each
// tap setup -- at C5 the on-the-fly projection of 31 cameras -- serves four
// frames.  Same box, C5 (profiles/round3/c5/pair_frames_ab.txt): B = 8 2.83 k
// -> 3.25 k frames/s, B = 32 3.11 k -> 3.43 k against 2 per entry.  A batch's
// remainder runs as a pair and / or a single frame (run_frames), so every
// grouping is exercised by batches of 2, 3, 5 and 7 frames.
constexpr int kPairFrames = 4;

static size_t frame_bytes(int V, int J, int H, int W, bool half) {
    return use_pairs(J, half) ? pair_frame_bytes(V, H, W) : cl_frame_bytes(V, J, H, W);
}

// Frames per chunk: keep a chunk's re-laid-out copy inside the 256 MB Infinity
// Cache.  fp32 layout: ~120 MB (C2 / C3 / C4: 12 frames) -- with layer-major
// slots 12 frames beat 8 by 5.5 % at C2, 3.5 % at C3, 1-3 % at C4, while 16+
// lose (C2: 4 / 8 / 10 / 12 / 16 / 20 / 32 frames = 83 / 96 / 98 / 101 / 96 /
// 80 / 81 k frames/s; profiles/round3/slot_order/chunk_sweep.txt; 8 was best
// with column-major slots).  fp16 pair table: ~128 MB, but at least one group
// of kPairFrames frames when that fits the cache: 4 frames = 245 MB at C5.
static int chunk_frames(int B, int V, int J, int H, int W, bool half) {
    const size_t per = frame_bytes(V, J, H, W, half);
    const bool pairs = use_pairs(J, half);
    const size_t budget = pairs ? (128ull << 20) : (120ull << 20);
    long long c = (long long)(budget / (per ? per : 1));
    if (pairs && c < kPairFrames && (size_t)kPairFrames * per <= (256ull << 20)) c = kPairFrames;
    if (c < 1) c = 1;
    if (c > B) c = B;
    return (int)c;
}

// Gather launch shape for `frames` frames per launch (NF per table entry).
struct GatherCfg {
    int cols, band, col_blocks, SP;
    size_t lds;
};

template <int LPV, bool OTF>
static int gather_cfg(int frames, int NF, int V, int X, int Y, int Z, GatherCfg &c) {
    // Column groups that tile the x-rows exactly (largest divisor of Y, if it
    // keeps at least half the columns), so the blocks can be walked in bands of
    // 16 x-rows: the blocks resident on an XCD at a time then cover a compact
    // x-y patch, whose heatmap footprint is smaller (C5 -8 %, C4 -4 %, C2 0).
    // Small grids (C1: 400 columns) keep their column groups (measured -6 % with bands).
    const bool big = (long long)X * Y >= 4096;
    auto snap = [&](int c) {
        if (big) {
            int cc = c;
            while (cc > 1 && Y % cc != 0) --cc;
            if (2 * cc >= c) c = cc;
        }
        return c;
    };
    auto blocks = [&](int c) { return (long long)frames / NF * ((X * Y + c - 1) / c); };
    // on the fly: 256-voxel blocks (C5: 4 columns of 64; 128-voxel blocks
    // measured 2-4 % slower, 64 -> 8 % slower, 512 -> 40 % slower, round 3);
    // 4 frames per entry: 128 (the stage holds NF frames)
    const int otf_vox = NF >= 4 ? 128 : 256;  // (4 frames: 256 -17 %, 64 -9 %; profiles/round3/c5/otf_voxels.txt)
    int cols = snap(OTF ? (Z >= otf_vox ? 1 : otf_vox / Z) : cols_per_block(Z));
    // latency (few frames): one pass of 256/LPV voxels per block, so a single
    // frame spreads over enough blocks to fill the CUs -- or two passes when
    // one-pass blocks would overflow one round of 8 blocks per CU (the counts
    // compared are those of the snapped column groups actually launched: C2/C3
    // B = 1, 80x80x20, LPV 4: one pass = 2 columns, 3,200 blocks; two passes =
    // 5 columns, 1,280 blocks -- 40 of a block's 64 voxel slots busy per pass
    // at one pass, 100 of 128 at two)
    if (blocks(cols) < 4 * 256) {
        cols = snap(max(1, (256 / LPV) / Z));
        if (blocks(cols) > 8 * 256) cols = snap(max(1, 2 * (256 / LPV) / Z));
    }
    c.cols = cols;
    c.band = (big && Y % cols == 0 && X > kBandRows) ? kBandRows : 0;
    c.col_blocks = (X * Y + cols - 1) / cols;
    c.SP = stage_pitch(LPV, cols, Z);
    c.lds = (size_t)NF * 4 * LPV * c.SP * sizeof(float);
    if (OTF) c.lds = ((c.lds / 4 + 3) & ~(size_t)3) * 4 + (size_t)FVP_GRID_SLOTS(V) * FVP_CAM_STRIDE * sizeof(float);
    return c.lds > 160 * 1024 ? FVP_ERR_SHAPE : FVP_OK;
}

template <int LPV, bool PAIR, bool OTF, bool CASC, int NF>
static void launch_gather(const void *tab, int f0, int nb, const GatherCfg &c, const CoordSource &src,
                          const int32_t *grid_index, int V, int J, int Jst, int H, int W, int X, int Y, int Z,
                          float *cube, float *xy, unsigned pixb, hipStream_t s) {
    const dim3 grid((unsigned)(nb / NF * c.col_blocks));
    const bool cube16 = ((unsigned long long)cube & 15ull) == 0;  // float4 epilogue stores
    if constexpr (OTF)
        hipLaunchKernelGGL((voxelize_cams_kernel<LPV, PAIR, true, CASC, NF>), grid, dim3(256), c.lds, s, tab, src,
                           grid_index, f0, cube, xy, V, J, Jst, H, W, X, Y, Z, c.cols, c.col_blocks, c.SP, c.band,
                           pixb, cube16);
    else
        hipLaunchKernelGGL((voxelize_kernel<LPV, PAIR, false, CASC, NF>), grid, dim3(256), c.lds, s, tab, src,
                           grid_index, f0, cube, xy, V, J, Jst, H, W, X, Y, Z, c.cols, c.col_blocks, c.SP, c.band,
                           pixb, cube16);
}

// One voxelize call's shapes.  Heatmaps with more than kJointSlice joints run
// in joint slices of kJointSlice (a layout pass + gather per slice): J is the
// slice's joint count, Jst the full count (the frame stride of the input
// planes and of the cube / xy outputs, whose pointers start at the slice).
constexpr int kJointSlice = 32;

struct VoxJob {
    int V, J, Jst, H, W, X, Y, Z;
    const int32_t *grid_index;
    float *cube, *xy;
};

// Frames [first, last) of the batch (a multiple of NF of them), chunk by chunk:
// layout pass into the workspace, then the gather, NF frames per table entry.
template <int LPV, bool PAIR, bool OTF, bool CASC, int NF, typename T>
static int run_chunks(const T *hm, int first, int last, const VoxJob &j, const CoordSource &src, void *ws,
                      hipStream_t s) {
    const bool half = sizeof(T) == 2;
    const int B = last - first;
    const int chunk = max(NF, chunk_frames(B, j.V, j.J, j.H, j.W, half) / NF * NF);
    GatherCfg c;
    if (gather_cfg<LPV, OTF>(min(chunk, B), NF, j.V, j.X, j.Y, j.Z, c) != FVP_OK) return FVP_ERR_SHAPE;
    const size_t frame_elems = (size_t)j.V * j.Jst * j.H * j.W;
    for (int f0 = first; f0 < last; f0 += chunk) {
        const int nb = min(chunk, last - f0);
        const T *hsrc = hm + (size_t)f0 * frame_elems;
        if constexpr (PAIR) {  // (J <= 16: never sliced)
            launch_pairs<NF>(reinterpret_cast<const _Float16 *>(hsrc), nb, j.V, j.J, j.H, j.W,
                             reinterpret_cast<uint4 *>(ws), s);
        } else {
            launch_layout<LPV, T, NF>(hsrc, nb, j.V, j.J, j.Jst, j.H, j.W, reinterpret_cast<float *>(ws), s);
        }
        launch_gather<LPV, PAIR, OTF, CASC, NF>(ws, f0, nb, c, src, j.grid_index, j.V, j.J, j.Jst, j.H, j.W, j.X, j.Y,
                                               j.Z, j.cube, j.xy, 4u * 4u * LPV, s);
    }
    return (int)hipGetLastError();
}

// Heatmaps already channels-last ([B][V][H][W][cp] fp32, the slice's joints
// from hm_cl on, e.g. the PoseResNet backbone's NHWC output): the gather reads
// them in place, one launch for the whole batch, no layout pass, no workspace.
template <bool OTF, bool CASC>
static int run_direct(const float *hm_cl, int cp, int B, const VoxJob &j, const CoordSource &src, hipStream_t s) {
    const unsigned pixb = (unsigned)cp * 4u;
    auto go = [&](auto lpv) -> int {
        constexpr int LPV = decltype(lpv)::value;
        GatherCfg c;
        if (gather_cfg<LPV, OTF>(B, 1, j.V, j.X, j.Y, j.Z, c) != FVP_OK) return FVP_ERR_SHAPE;
        launch_gather<LPV, false, OTF, CASC, 1>(hm_cl, 0, B, c, src, j.grid_index, j.V, j.J, j.Jst, j.H, j.W, j.X,
                                               j.Y, j.Z, j.cube, j.xy, pixb, s);
        return (int)hipGetLastError();
    };
    switch (lanes_per_voxel(j.J)) {
        case 1: return go(std::integral_constant<int, 1>{});
        case 2: return go(std::integral_constant<int, 2>{});
        case 4: return go(std::integral_constant<int, 4>{});
        default: return go(std::integral_constant<int, 8>{});
    }
}

// Frames per table entry: the fp16 pair table interleaves two frames per
// 128-B line (NF = 2), so each tap row of a voxel-camera serves both frames
// with one line and one tap setup: C5 3.97 -> 3.12 ms per 8 frames (the
// gather waits on L1 misses; measured).  The fp32 channels-last table keeps
// one frame per entry (NF = 2 measured 4 % slower at C2: the L2 working set
// doubles).  Four frames per entry (kPairFrames) amortise the tap setup
// further; the batch runs as groups of 4, then a pair, then a single frame.
// Frames of a group must share one sampling grid, so batches that mix
// sequences (grid_index given) run at NF = 1.
template <int LPV, bool PAIR, bool OTF, bool CASC, typename T>
static int run_frames(const T *hm, int B, const VoxJob &j, const CoordSource &src, void *ws, hipStream_t s) {
    if constexpr (PAIR) {
        const int cf = chunk_frames(B, j.V, j.J, j.H, j.W, sizeof(T) == 2);
        int done = 0;
        if (!j.grid_index && cf >= kPairFrames) {  // workspace holds >= 4 frames
            done = B / kPairFrames * kPairFrames;
            const int st = run_chunks<LPV, PAIR, OTF, CASC, kPairFrames, T>(hm, 0, done, j, src, ws, s);
            if (st != FVP_OK || done == B) return st;
        }
        if (!j.grid_index && cf >= 2 && B - done >= 2) {  // workspace holds >= 2 frames
            const int even = done + ((B - done) & ~1);
            const int st = run_chunks<LPV, PAIR, OTF, CASC, 2, T>(hm, done, even, j, src, ws, s);
            if (st != FVP_OK || even == B) return st;
            done = even;
        }
        if (done > 0) return run_chunks<LPV, PAIR, OTF, CASC, 1, T>(hm, done, B, j, src, ws, s);
    }
    return run_chunks<LPV, PAIR, OTF, CASC, 1, T>(hm, 0, B, j, src, ws, s);
}

template <bool OTF, bool CASC, typename T>
static int voxelize_lpv(const T *hm, int B, const VoxJob &j, const CoordSource &src, void *ws, hipStream_t s) {
    const bool half = sizeof(T) == 2;
    if (use_pairs(j.Jst, half)) return run_frames<4, true, OTF, CASC, T>(hm, B, j, src, ws, s);
    switch (lanes_per_voxel(j.J)) {
        case 1: return run_frames<1, false, OTF, CASC, T>(hm, B, j, src, ws, s);
        case 2: return run_frames<2, false, OTF, CASC, T>(hm, B, j, src, ws, s);
        case 4: return run_frames<4, false, OTF, CASC, T>(hm, B, j, src, ws, s);
        default: return run_frames<8, false, OTF, CASC, T>(hm, B, j, src, ws, s);
    }
}

// Joints of the first slice (all of them up to kJointSlice).
static int slice_joints(int J) { return J < kJointSlice ? J : kJointSlice; }

static size_t workspace_bytes(int B, int V, int J, int H, int W, bool half);

template <bool OTF, typename T>
static int voxelize_any(const T *hm, int B, int V, int J, int H, int W, const CoordSource &src,
                        const int32_t *grid_index, int X, int Y, int Z, float *cube, float *xy, void *ws,
                        size_t ws_bytes, hipStream_t s) {
    const bool half = sizeof(T) == 2;
    const int J1 = slice_joints(J);
    const size_t need = workspace_bytes(B, V, J, H, W, half);
    if (!ws || ws_bytes < need) return FVP_ERR_WORKSPACE;
    if (frame_bytes(1, J1, H, W, half) > 0x7fffffffull) return FVP_ERR_SHAPE;  // 32-bit tap offsets
    const size_t N = (size_t)X * Y * Z, XY = (size_t)X * Y, HW = (size_t)H * W;
    for (int j0 = 0; j0 < J; j0 += kJointSlice) {
        const VoxJob job{V, min(kJointSlice, J - j0), J, H, W, X, Y, Z, grid_index, cube ? cube + j0 * N : nullptr,
                         xy ? xy + j0 * XY : nullptr};
        const T *h = hm + j0 * HW;
        const int st = V > 16 ? voxelize_lpv<OTF, true, T>(h, B, job, src, ws, s)
                              : voxelize_lpv<OTF, false, T>(h, B, job, src, ws, s);
        if (st != FVP_OK) return st;
    }
    return FVP_OK;
}

// Channels-last input: the slice's channels start at hm_cl + j0 (cp >= j0 + 4 * LPV(slice) for every slice).
template <bool OTF>
static int voxelize_cl_any(const float *hm_cl, int cp, int B, int V, int J, int H, int W, const CoordSource &src,
                           const int32_t *grid_index, int X, int Y, int Z, float *cube, float *xy, hipStream_t s) {
    const int jl = ((J - 1) / kJointSlice) * kJointSlice;  // first joint of the last slice
    if (cp % 4 || cp < jl + 4 * lanes_per_voxel(J - jl)) return FVP_ERR_SHAPE;
    if ((size_t)H * W * cp * 4 > 0x7fffffffull) return FVP_ERR_SHAPE;  // 32-bit tap offsets per camera image
    const size_t N = (size_t)X * Y * Z, XY = (size_t)X * Y;
    for (int j0 = 0; j0 < J; j0 += kJointSlice) {
        const VoxJob job{V, min(kJointSlice, J - j0), J, H, W, X, Y, Z, grid_index, cube ? cube + j0 * N : nullptr,
                         xy ? xy + j0 * XY : nullptr};
        const int st = V > 16 ? run_direct<OTF, true>(hm_cl + j0, cp, B, job, src, s)
                              : run_direct<OTF, false>(hm_cl + j0, cp, B, job, src, s);
        if (st != FVP_OK) return st;
    }
    return FVP_OK;
}

static int check_args(const void *heatmaps, int B, int V, int J, int H, int W, const float *grids, int X, int Y, int Z) {
    if (!heatmaps || !grids) return FVP_ERR_NULL;
    if (B <= 0 || V <= 0 || V > FVP_MAX_VIEWS || J <= 0 || J > FVP_MAX_JOINTS || H < 2 || W < 2 || X <= 0 ||
        Y <= 0 || Z <= 0)
        return FVP_ERR_SHAPE;
    // packed grid of one sequence addressed with 32-bit byte offsets
    if ((long long)X * Y * Z * FVP_GRID_SLOTS(V) * 8 > 0xfffff000LL) return FVP_ERR_SHAPE;
    return FVP_OK;
}

static size_t workspace_bytes(int B, int V, int J, int H, int W, bool half) {
    if (B <= 0 || V <= 0 || J <= 0 || J > FVP_MAX_JOINTS || H <= 0 || W <= 0) return 0;
    const int J1 = slice_joints(J);  // one joint slice's copy at a time
    return (size_t)chunk_frames(B, V, J1, H, W, half) * frame_bytes(V, J1, H, W, half);
}

// -- winners' columns without the cube ----------------------------------------
// columns[b,k,j,z] = cube[b,j,flat[b,k],z] (human_detection_net.py:199-200)
// recomputed for the K winners only, so an HDN forward that needs the cube
// just for these columns can skip writing it (7.7 MB per C2 frame): the same
// per-voxel arithmetic as voxelize_body -- coordinates from the packed grid or
// projected on the fly, setup_taps, fma(d,w3, fma(c,w2, fma(b,w1, a*w0))) per
// camera in view order with the 16-camera block fold, + 0 / + blocks, / V,
// clamp -- hence bit-identical to the cube's voxels.  The heatmaps are read
// in place through strides: planar [B][V][J][H][W] (joint stride H*W, pixel
// stride 1) or channels-last [B][V][H][W][cp] (joint stride 1, pixel stride
// cp).  One thread per output element (z fastest).
template <typename T, bool OTF, bool CASC>
__global__ __launch_bounds__(256) void voxel_columns_kernel(const T *__restrict__ hm, long long vstride,
                                                            long long jstride, int pstride, CoordSource src,
                                                            const int32_t *__restrict__ grid_index,
                                                            const int64_t *__restrict__ flat, int K, int V, int J,
                                                            int H, int W, int X, int Y, int Z,
                                                            float *__restrict__ cols, long long total) {
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= total) return;
    const int z = (int)(gid % Z);
    long long r = gid / Z;
    const int j = (int)(r % J);
    r /= J;
    const int k = (int)(r % K);
    const long long b = r / K;
    const int64_t f = flat[b * K + k];
    if (f < 0 || f >= (int64_t)X * Y) {  // an index outside the map reads nothing (as gather_columns)
        cols[gid] = __builtin_nanf("");
        return;
    }
    const long long n = f * Z + z;
    const long long N = (long long)X * Y * Z;
    const int GV = V + (V & 1);
    const int gsel = grid_index ? grid_index[b] : 0;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    float wx_ = 0.f, wy_ = 0.f, wz_ = 0.f, rt[6];
    if constexpr (OTF) {
        wx_ = axis_coord(src.gs.start[0], src.gs.end[0], X, (int)(f / Y), src.gs.center[0]);
        wy_ = axis_coord(src.gs.start[1], src.gs.end[1], Y, (int)(f % Y), src.gs.center[1]);
        wz_ = axis_coord(src.gs.start[2], src.gs.end[2], Z, z, src.gs.center[2]);
#pragma unroll
        for (int q = 0; q < 6; ++q) rt[q] = src.resize_t[q];
    }
    // cameras in groups of G: all coordinates, then all 4G taps in flight, then
    // the sums in view order (the latency of one group instead of one per camera)
    constexpr int G = OTF ? 4 : 8;  // (OTF: 21 floats of camera record per camera in registers)
    float acc = 0.0f, blk = 0.0f;
    for (int v0 = 0; v0 < V; v0 += G) {
        float tv[G][4], w[G][4];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const int v = min(v0 + u, V - 1);
            float gx, gy;
            if constexpr (OTF) {
                const Cam c = load_cam(src.cams + ((size_t)gsel * V + v) * FVP_CAM_STRIDE);
                float px, py;
                project_point(c, wx_, wy_, wz_, px, py);
                pixel_to_sample(px, py, rt, src.im, gx, gy);
            } else {
                const float2 gp = *reinterpret_cast<const float2 *>(src.grids + (((size_t)gsel * N + n) * GV + v) * 2);
                gx = gp.x;
                gy = gp.y;
            }
            const Taps4<false> t = setup_taps<false>(gx, gy, sxs, sys, W, H, 1u);  // offsets in pixels
            const T *__restrict__ im = hm + ((size_t)b * V + v) * vstride + (size_t)j * jstride;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                w[u][m] = t.w[m];
                tv[u][m] = t.o[m] == kOOB ? 0.0f : to_f32(im[(size_t)t.o[m] * pstride]);
            }
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const int v = v0 + u;
            if (v >= V) break;
            if (CASC && (v & 15) == 0 && v > 0) {  // a complete block of 16 cameras (fvp_device.h)
                blk = blk + acc;
                acc = 0.0f;
            }
            acc = acc + __builtin_fmaf(tv[u][3], w[u][3],
                                       __builtin_fmaf(tv[u][2], w[u][2], __builtin_fmaf(tv[u][1], w[u][1], tv[u][0] * w[u][0])));
        }
    }
    acc = acc + (CASC ? blk : 0.0f);
    cols[gid] = clampf(acc / (float)V, 0.0f, 1.0f);
}

}  // namespace fvp

extern "C" int fvp_voxel_columns(const void *heatmaps, int half, long long view_stride, long long joint_stride,
                                 int pix_stride, int B, int V, int J, int H, int W, const float *packed_grids,
                                 const float *cams, const float *resize_t, const fvp_grid_spec *grid,
                                 const fvp_image_spec *img, const int32_t *grid_index, int X, int Y, int Z,
                                 const int64_t *flat, int K, float *columns, void *stream) {
    if (!heatmaps || !flat || !columns) return FVP_ERR_NULL;
    if (B < 0 || K < 0 || V <= 0 || V > FVP_MAX_VIEWS || J <= 0 || H < 2 || W < 2 || X <= 0 || Y <= 0 || Z <= 0 ||
        view_stride <= 0 || joint_stride <= 0 || pix_stride <= 0)
        return FVP_ERR_SHAPE;
    if ((long long)H * W > 0x7fffffffLL) return FVP_ERR_SHAPE;  // 32-bit pixel offsets
    fvp::CoordSource src{};
    const bool otf = packed_grids == nullptr;
    if (otf) {
        if (!cams || !resize_t || !grid || !img) return FVP_ERR_NULL;
        if (grid->bins[0] != X || grid->bins[1] != Y || grid->bins[2] != Z || img->hm_w != W || img->hm_h != H)
            return FVP_ERR_SHAPE;
        src.cams = cams;
        src.resize_t = resize_t;
        src.gs = *grid;
        src.im = fvp::image_consts(*img);
    } else {
        src.grids = packed_grids;
    }
    const long long total = (long long)B * K * J * Z;
    if (total == 0) return FVP_OK;
    const dim3 g((unsigned)((total + 255) / 256)), blk(256);
    hipStream_t st = (hipStream_t)stream;
    auto go = [&](auto tag, auto o, auto c) {
        using T = decltype(tag);
        hipLaunchKernelGGL((fvp::voxel_columns_kernel<T, decltype(o)::value, decltype(c)::value>), g, blk, 0, st,
                           reinterpret_cast<const T *>(heatmaps), view_stride, joint_stride, pix_stride, src,
                           grid_index, flat, K, V, J, H, W, X, Y, Z, columns, total);
    };
    using TT = std::true_type;
    using FF = std::false_type;
    const bool casc = V > 16;
    if (half) {
        if (otf) casc ? go(_Float16{}, TT{}, TT{}) : go(_Float16{}, TT{}, FF{});
        else casc ? go(_Float16{}, FF{}, TT{}) : go(_Float16{}, FF{}, FF{});
    } else {
        if (otf) casc ? go(0.0f, TT{}, TT{}) : go(0.0f, TT{}, FF{});
        else casc ? go(0.0f, FF{}, TT{}) : go(0.0f, FF{}, FF{});
    }
    return (int)hipGetLastError();
}

extern "C" int fvp_pack_grid(const float *sample_grid, int V, long long N, float *packed, void *stream) {
    if (!sample_grid || !packed) return FVP_ERR_NULL;
    if (V <= 0 || N <= 0) return FVP_ERR_SHAPE;
    const int GV = FVP_GRID_SLOTS(V);
    const long long tot = N * GV;
    hipLaunchKernelGGL(fvp::pack_grid_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float2 *>(sample_grid), reinterpret_cast<float2 *>(packed), V, GV, N);
    return (int)hipGetLastError();
}

extern "C" size_t fvp_voxelize_workspace_bytes(int B, int V, int J, int H, int W) {
    return fvp::workspace_bytes(B, V, J, H, W, false);
}

extern "C" size_t fvp_voxelize_f16_workspace_bytes(int B, int V, int J, int H, int W) {
    return fvp::workspace_bytes(B, V, J, H, W, true);
}

extern "C" int fvp_voxelize(const float *heatmaps, int B, int V, int J, int H, int W, const float *packed_grids,
                            const int32_t *grid_index, int X, int Y, int Z, float *cube, float *xy, void *workspace,
                            size_t workspace_bytes, void *stream) {
    const int st = fvp::check_args(heatmaps, B, V, J, H, W, packed_grids, X, Y, Z);
    if (st != FVP_OK) return st;
    if (!cube && !xy) return FVP_OK;
    fvp::CoordSource src{};
    src.grids = packed_grids;
    return fvp::voxelize_any<false, float>(heatmaps, B, V, J, H, W, src, grid_index, X, Y, Z, cube, xy, workspace,
                                           workspace_bytes, (hipStream_t)stream);
}

extern "C" int fvp_voxelize_f16(const void *heatmaps, int B, int V, int J, int H, int W, const float *packed_grids,
                                const int32_t *grid_index, int X, int Y, int Z, float *cube, float *xy,
                                void *workspace, size_t workspace_bytes, void *stream) {
    const int st = fvp::check_args(heatmaps, B, V, J, H, W, packed_grids, X, Y, Z);
    if (st != FVP_OK) return st;
    if (!cube && !xy) return FVP_OK;
    fvp::CoordSource src{};
    src.grids = packed_grids;
    return fvp::voxelize_any<false, _Float16>(reinterpret_cast<const _Float16 *>(heatmaps), B, V, J, H, W, src,
                                              grid_index, X, Y, Z, cube, xy, workspace, workspace_bytes,
                                              (hipStream_t)stream);
}

namespace fvp {

// The on-the-fly entry points, for the whole grid or for x-rows [x0, x1) of it
// (the large-frame mode): every voxel's coordinates come from
// its global indices, so a slab is bit-identical to the same rows of the
// whole-grid launch, and no rank builds or reads a sample grid.
static int voxelize_cams_rows(const void *heatmaps, bool half, const float *hm_cl, int cp, int B, int V, int J, int H,
                              int W, const float *cams, const int32_t *grid_index, const float *resize_t,
                              const fvp_grid_spec *grid, const fvp_image_spec *img, int x0, int x1, float *cube,
                              float *xy, void *workspace, size_t workspace_bytes, hipStream_t s) {
    if (!cams || !resize_t || !grid || !img) return FVP_ERR_NULL;
    const int Y = grid->bins[1], Z = grid->bins[2];
    if (x0 < 0 || x1 > grid->bins[0] || x0 >= x1) return FVP_ERR_SHAPE;
    const int X = x1 - x0;  // the launch's x-rows
    const int st = check_args(hm_cl ? (const void *)hm_cl : heatmaps, B, V, J, H, W, cams, X, Y, Z);
    if (st != FVP_OK) return st;
    if (img->hm_w != W || img->hm_h != H) return FVP_ERR_SHAPE;
    if (!cube && !xy) return FVP_OK;
    CoordSource src{};
    src.cams = cams;
    src.resize_t = resize_t;
    src.gs = *grid;
    src.im = fvp::image_consts(*img);
    src.x_off = x0;
    if (hm_cl) return voxelize_cl_any<true>(hm_cl, cp, B, V, J, H, W, src, grid_index, X, Y, Z, cube, xy, s);
    if (half)
        return voxelize_any<true, _Float16>(reinterpret_cast<const _Float16 *>(heatmaps), B, V, J, H, W, src,
                                            grid_index, X, Y, Z, cube, xy, workspace, workspace_bytes, s);
    return voxelize_any<true, float>(reinterpret_cast<const float *>(heatmaps), B, V, J, H, W, src, grid_index, X, Y,
                                     Z, cube, xy, workspace, workspace_bytes, s);
}

}  // namespace fvp

extern "C" int fvp_voxelize_cams(const void *heatmaps, int half, int B, int V, int J, int H, int W,
                                 const float *cams, const int32_t *grid_index, const float *resize_t,
                                 const fvp_grid_spec *grid, const fvp_image_spec *img, float *cube, float *xy,
                                 void *workspace, size_t workspace_bytes, void *stream) {
    if (!grid) return FVP_ERR_NULL;
    return fvp::voxelize_cams_rows(heatmaps, half != 0, nullptr, 0, B, V, J, H, W, cams, grid_index, resize_t, grid,
                                   img, 0, grid->bins[0], cube, xy, workspace, workspace_bytes, (hipStream_t)stream);
}

extern "C" int fvp_voxelize_cams_slab(const void *heatmaps, int half, int B, int V, int J, int H, int W,
                                      const float *cams, const int32_t *grid_index, const float *resize_t,
                                      const fvp_grid_spec *grid, const fvp_image_spec *img, int x_begin, int x_end,
                                      float *cube, float *xy, void *workspace, size_t workspace_bytes, void *stream) {
    return fvp::voxelize_cams_rows(heatmaps, half != 0, nullptr, 0, B, V, J, H, W, cams, grid_index, resize_t, grid,
                                   img, x_begin, x_end, cube, xy, workspace, workspace_bytes, (hipStream_t)stream);
}

extern "C" int fvp_voxelize_cl(const float *heatmaps_cl, int cp, int B, int V, int J, int H, int W,
                               const float *packed_grids, const int32_t *grid_index, int X, int Y, int Z, float *cube,
                               float *xy, void *stream) {
    const int st = fvp::check_args(heatmaps_cl, B, V, J, H, W, packed_grids, X, Y, Z);
    if (st != FVP_OK) return st;
    if (!cube && !xy) return FVP_OK;
    fvp::CoordSource src{};
    src.grids = packed_grids;
    return fvp::voxelize_cl_any<false>(heatmaps_cl, cp, B, V, J, H, W, src, grid_index, X, Y, Z, cube, xy,
                                       (hipStream_t)stream);
}

extern "C" int fvp_voxelize_cl_cams(const float *heatmaps_cl, int cp, int B, int V, int J, int H, int W,
                                    const float *cams, const int32_t *grid_index, const float *resize_t,
                                    const fvp_grid_spec *grid, const fvp_image_spec *img, float *cube, float *xy,
                                    void *stream) {
    if (!heatmaps_cl) return FVP_ERR_NULL;
    if (!grid) return FVP_ERR_NULL;
    return fvp::voxelize_cams_rows(nullptr, false, heatmaps_cl, cp, B, V, J, H, W, cams, grid_index, resize_t, grid,
                                   img, 0, grid->bins[0], cube, xy, nullptr, 0, (hipStream_t)stream);
}

extern "C" int fvp_voxelize_cl_cams_slab(const float *heatmaps_cl, int cp, int B, int V, int J, int H, int W,
                                         const float *cams, const int32_t *grid_index, const float *resize_t,
                                         const fvp_grid_spec *grid, const fvp_image_spec *img, int x_begin,
                                         int x_end, float *cube, float *xy, void *stream) {
    if (!heatmaps_cl) return FVP_ERR_NULL;
    return fvp::voxelize_cams_rows(nullptr, false, heatmaps_cl, cp, B, V, J, H, W, cams, grid_index, resize_t, grid,
                                   img, x_begin, x_end, cube, xy, nullptr, 0, (hipStream_t)stream);
}
