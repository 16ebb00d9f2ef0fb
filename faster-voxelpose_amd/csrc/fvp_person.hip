// Per-person voxel cubes from the cached fine sample grid (A11-A13) and the
// JLN xy/xz/yz max-projections (A8).
//
// fvp_person_planes replaces project_individual.ProjectLayer.forward
// (project_individual.py:222-293) and, fused, the max-projections of
// joint_localization_net.py:158-160, for every proposal of a batch in one
// launch and without host syncs: each block recomputes its proposal's window
// (centers_tl, margins, start/end, skip flag, :255-275) from the proposal
// row.  The frames are first re-laid out channels-last (fvp_layout.h) so the
// taps are quad-coalesced (see fvp_voxelize.hip).
//
// max_planes (planes of an already materialised cube) replaces torch.cat([max(c,4), max(c,3), max(c,2)])
// (joint_localization_net.py:158-160): one block per (person, joint) reads the
// S^3 cube once; lane = z, each wave owns S/4 y-rows; yz is a register max
// over x, xz a register + LDS max over y, xy a wave reduction over z.
#include "fvp_layout.h"

namespace fvp {

struct Window {
    int ctl[3], start[3], end[3];
    bool skip;
};

__device__ __forceinline__ Window person_window(const float *__restrict__ pc, const fvp_person_spec &s) {
    Window w;
    // centers_tl = round(center * scale + bias).int()   (:255, round half to even)
#pragma unroll
    for (int a = 0; a < 3; ++a) w.ctl[a] = (int)rintf(pc[a] * s.scale[a] + s.bias[a]);
    // mask = ((1 - bbox) / 2 * (vpa[0:2] - 1)).int(), negatives -> 0, z margin 0  (:262-265)
    int m[3];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const float f = ((1.0f - pc[5 + a]) / 2.0f) * (float)(s.bins[a] - 1);
        int mi = (int)f;  // trunc toward zero, as .int()
        m[a] = mi < 0 ? 0 : mi;
    }
    m[2] = 0;
    w.skip = false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int lo = w.ctl[a] + m[a];
        const int hi = w.ctl[a] + s.bins[a] - m[a];
        w.start[a] = lo >= 0 ? lo : 0;                   // :268
        w.end[a] = hi <= s.fine[a] ? hi : s.fine[a];     // :269
        w.skip |= (w.start[a] >= w.end[a]);              // :274-275
    }
    return w;
}

// planes: [3P][J][S][S]; block (p, j); 256 threads = 4 waves, lane = z.
__global__ __launch_bounds__(256) void max_planes_kernel(const float *__restrict__ cubes, float *__restrict__ planes,
                                                         int P, int J, int S) {
    __shared__ float xz_part[4][64];
    const int p = blockIdx.x / J, j = blockIdx.x % J;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool zok = lane < S;
    const size_t SS = (size_t)S * S;
    const float *__restrict__ c = cubes + ((size_t)p * J + j) * SS * S;
    float *__restrict__ pxy = planes + ((size_t)(0 * P + p) * J + j) * SS;
    float *__restrict__ pxz = planes + ((size_t)(1 * P + p) * J + j) * SS;
    float *__restrict__ pyz = planes + ((size_t)(2 * P + p) * J + j) * SS;
    constexpr int kRows = 16;  // y rows per wave (S <= 64)
    float yz[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) yz[r] = -INFINITY;

    for (int x = 0; x < S; ++x) {
        float xzm = -INFINITY;
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            const int y = wave + 4 * r;
            const bool ok = zok && y < S;
            const float v = ok ? c[((size_t)x * S + y) * S + lane] : -INFINITY;
            yz[r] = nanmax(yz[r], v);
            xzm = nanmax(xzm, v);
            // xy[x][y] = max over z (wave reduction; y is wave-uniform)
            float m = v;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) m = nanmax(m, __shfl_xor(m, off));
            if (lane == 0 && y < S) pxy[(size_t)x * S + y] = m;
        }
        xz_part[wave][lane] = xzm;
        __syncthreads();
        if (wave == 0 && zok) {
            float m = xz_part[0][lane];
            m = nanmax(m, xz_part[1][lane]);
            m = nanmax(m, xz_part[2][lane]);
            m = nanmax(m, xz_part[3][lane]);
            pxz[(size_t)x * S + lane] = m;
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int y = wave + 4 * r;
        if (zok && y < S) pyz[(size_t)y * S + lane] = yz[r];
    }
}

// Planes of cubes deeper than 64 (one thread per plane cell, a loop over the
// reduced axis; NaN-propagating like torch.max).
__global__ __launch_bounds__(256) void max_planes_generic_kernel(const float *__restrict__ cubes,
                                                                 float *__restrict__ planes, int P, int J, int S) {
    const size_t SS = (size_t)S * S;
    const size_t per_plane = (size_t)P * J * SS;
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= 3 * per_plane) return;
    const int k = (int)(e / per_plane);  // 0 xy (max z), 1 xz (max y), 2 yz (max x)
    const size_t r = e - k * per_plane;
    const size_t pj = r / SS;
    const int a = (int)((r - pj * SS) / S), b = (int)(r - pj * SS - (size_t)a * S);
    const float *__restrict__ c = cubes + pj * SS * S;
    const size_t base = k == 0 ? ((size_t)a * S + b) * S : k == 1 ? (size_t)a * SS + b : (size_t)a * S + b;
    const size_t step = k == 0 ? 1 : k == 1 ? (size_t)S : SS;
    float m = -INFINITY;
    for (int t = 0; t < S; ++t) m = nanmax(m, c[base + t * step]);
    planes[e] = m;
}

// Channels-last per-person kernel (batched over frames, optional fused planes).
// Block = (proposal p, one y-row, x part, 64-deep z chunk); threads = 64 z-lanes
// x LPV joint quads.  The block walks the x-planes of its row:
//   xy[x][y] = max_z   -> per-wave z maxima in VALU (slot_umax), then either kept
//                         in LDS and stored once per (x, joint) at the block's end
//                         (xy_direct: the block owns the row's xy cells) or one
//                         atomicMax per wave into the pre-zeroed plane
//   yz[y][z] = max_x   -> registers (the block owns its row), stored at the end
//                         (atomics into a pre-zeroed plane when x is split)
//   xz[x][z] = max_y   -> one atomicMax per (x, z, joint) into the pre-zeroed plane
// (values are clamped to [0,1] or NaN, so unsigned order == float order.)
// Outside-window voxels are 0 exactly as in the reference cube.
// Sampling coordinates of the fine grid: the packed per-sequence grid
// (OTF = false) or projected on the fly from the camera records with the fp32
// sequence of fvp_project_grid (OTF = true: no 197 MB fine grid to stream).
struct PersonCoords {
    const float *cams;      // [V][FVP_CAM_STRIDE]   (OTF)
    const float *resize_t;  // [2][3]                (OTF)
    fvp_grid_spec fine;     // fine whole-space grid (OTF)
    ImageConsts im;         //                       (OTF)
};

// The clamped-mean input of one fine voxel of the person cube: the V cameras'
// bilinear taps summed in the reference's order (project_individual.py:278-283,
// fvp_device.h), before the division.  A group of LPV lanes shares the voxel
// (lane q holds joints 4q..4q+3); `valid` false (outside the window or the
// cube) gives 0.  Coordinates from the packed fine grid or projected on the fly.
template <int LPV, bool OTF, bool CASC, int MODE>
__device__ __forceinline__ void person_voxel_sum(float (&acc)[4], bool valid, int gx, int gy, int gz,
                                                 const __amdgpu_buffer_rsrc_t &grs, const float *lcam, const float *rt,
                                                 const PersonCoords &pc, const fvp_person_spec &s,
                                                 const char *__restrict__ frame_cl, unsigned img, unsigned qo, int q,
                                                 int V, int GV, int W, int H, float sxs, float sys,
                                                 unsigned pix_bytes) {
    constexpr int CPG = 2 * LPV;  // cameras per packed-grid load (2 per lane)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = 0.0f;
    float blk[4] = {0.f, 0.f, 0.f, 0.f};  // CASC: completed 16-camera blocks (fvp_device.h)
    if (__builtin_amdgcn_ballot_w64(valid)) {
        const long long gn = valid ? ((long long)gx * s.fine[1] + gy) * s.fine[2] + gz : 0;
        float wxc = 0.f, wyc = 0.f, wzc = 0.f;  // OTF: fine voxel centre (compute_grid at fine resolution)
        if constexpr (OTF) {
            wxc = axis_coord(pc.fine.start[0], pc.fine.end[0], s.fine[0], valid ? gx : 0, pc.fine.center[0]);
            wyc = axis_coord(pc.fine.start[1], pc.fine.end[1], s.fine[1], valid ? gy : 0, pc.fine.center[1]);
            wzc = axis_coord(pc.fine.start[2], pc.fine.end[2], s.fine[2], valid ? gz : 0, pc.fine.center[2]);
        }
        for (int v0 = 0; v0 < V; v0 += CPG) {
            float g[4];
            if constexpr (OTF) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const Cam c = load_cam(lcam + min(v0 + 2 * q + h, GV - 1) * FVP_CAM_STRIDE);
                    float px, py;
                    project_point(c, wxc, wyc, wzc, px, py);
                    pixel_to_sample(px, py, rt, pc.im, g[2 * h], g[2 * h + 1]);
                }
            } else {
                // slots v0+2q, v0+2q+1 of fine voxel gn (packed grid, fvp_pack_grid)
                const u32x4 graw =
                    __builtin_amdgcn_raw_buffer_load_b128(grs, (unsigned)((gn * GV + v0 + 2 * q) * 8), 0, 0);
#pragma unroll
                for (int k = 0; k < 4; ++k) g[k] = __builtin_bit_cast(float, (unsigned)graw[k]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) g[k] = valid ? g[k] : -2.0f;
            const Taps4<false> t0 = setup_taps<false>(g[0], g[1], sxs, sys, W, H, pix_bytes);
            const Taps4<false> t1 = setup_taps<false>(g[2], g[3], sxs, sys, W, H, pix_bytes);
            static_for(std::make_integer_sequence<int, CPG>{}, [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int S = k >> 1;
                const int v = v0 + k;
                if (v >= V) return;
                if constexpr (CASC) {
                    if ((v & 15) == 0 && v > 0) {
#pragma unroll
                        for (int m = 0; m < 4; ++m) {
                            blk[m] = blk[m] + acc[m];
                            acc[m] = 0.0f;
                        }
                    }
                }
                const Taps4<false> &src = (k & 1) ? t1 : t0;
                unsigned o[4];
                unsigned all = kOOB;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    o[m] = group_bcast<LPV, S>(src.o[m]);
                    all &= o[m];
                }
                if (!__builtin_amdgcn_ballot_w64((all & kOOB) == 0u)) return;
                float wt[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) wt[m] = group_bcast<LPV, S>(src.w[m]);
                if constexpr (MODE == 4) {
#pragma unroll
                    for (int m = 0; m < 4; ++m) acc[m] = acc[m] + wt[m] + __builtin_bit_cast(float, o[m]);
                    return;
                }
                if constexpr (MODE == 3) {
#pragma unroll
                    for (int m = 0; m < 4; ++m) o[m] = kOOB;
                }
                const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(frame_cl + (size_t)v * img, img);
                u32x4 ta = {0u, 0u, 0u, 0u}, tb = ta, tc = ta, td = ta;
                if constexpr (MODE != 2) {
                    ta = __builtin_amdgcn_raw_buffer_load_b128(rs, o[0] + qo, 0, 0);
                    tb = __builtin_amdgcn_raw_buffer_load_b128(rs, o[1] + qo, 0, 0);
                    tc = __builtin_amdgcn_raw_buffer_load_b128(rs, o[2] + qo, 0, 0);
                    td = __builtin_amdgcn_raw_buffer_load_b128(rs, o[3] + qo, 0, 0);
                }
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float fa = __builtin_bit_cast(float, (unsigned)ta[m]);
                    const float fb = __builtin_bit_cast(float, (unsigned)tb[m]);
                    const float fc = __builtin_bit_cast(float, (unsigned)tc[m]);
                    const float fd = __builtin_bit_cast(float, (unsigned)td[m]);
                    acc[m] = acc[m] + __builtin_fmaf(fd, wt[3], __builtin_fmaf(fc, wt[2],
                                                                              __builtin_fmaf(fb, wt[1], fa * wt[0])));
                }
            });
        }
    }
    // the sum's final levels (fvp_device.h): remainder + blocks, or + 0 (a -0 sum becomes +0)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = acc[m] + (CASC ? blk[m] : 0.0f);
}

// MODE (replay probe, tools/person_probe.hip; the product launches 0): 1 = no
// plane reductions / stores (the sums folded into `offset`), 2 = zeros instead
// of the tap loads, 3 = every tap offset off-image (range-checked loads, no
// memory access), 4 = grid loads and tap setup only (no tap loads, no planes),
// 5 / 6 = no xz / xy plane atomics or stores, 7 = xz atomics from even z lanes only,
// 8 = plain stores instead of the xz atomics (timing only: wrong maxima).
template <int LPV, bool OTF, bool CASC, int MODE = 0>
__global__ __launch_bounds__(64 * LPV) void person_cl_kernel(const float *__restrict__ cl,
                                                             const float *__restrict__ fgrid, PersonCoords pc,
                                                             const float *__restrict__ props,
                                                             const int32_t *__restrict__ frame_of, fvp_person_spec s,
                                                             float *__restrict__ cubes, float *__restrict__ planes,
                                                             float *__restrict__ offset, int P, int V, int J, int Jst,
                                                             int H, int W, int xmap, int xsplit, int zsplit,
                                                             unsigned pix_bytes, int xy_direct) {
    __shared__ float lcam[OTF ? 64 * FVP_CAM_STRIDE : 1];  // OTF: camera records (V <= 64)
    // xy_direct: [wave][x][joint slot] per-wave z maxima, stored at the block's end
    constexpr bool DXY = LPV <= 4;
    __shared__ unsigned lxy[DXY ? LPV * 64 * 4 * LPV : 1];
    const int SX = s.bins[0], SY = s.bins[1], SZ = s.bins[2];
    // XCD-aware: each XCD runs whole proposals, so the rows of one proposal
    // (walking x together) share that XCD's L2 footprint (L2 hit 35 % with
    // round-robin placement)
    const int L = xmap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    // block -> (proposal, row, x part, z chunk): a proposal's blocks stay contiguous
    const int parts = xsplit * zsplit;
    const int p = L / (SY * parts);
    const int rem = L - p * SY * parts;
    const int y = rem / parts;
    const int part = rem - y * parts;
    const int xpart = part % xsplit, zc = part / xsplit;
    const Window w = person_window(props + (size_t)p * 7, s);
    if (offset && y == 0 && part == 0 && threadIdx.x < 3) {
        const int a = threadIdx.x;
        offset[(size_t)p * 3 + a] =
            ((float)w.ctl[a] / (float)(s.fine[a] - 1)) * s.whole_size[a] - s.whole_size[a] / 2.0f + s.ind_size[a] / 2.0f;
    }
    const int lane = threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    const int zl = zc * 64 + (int)threadIdx.x / LPV, q = threadIdx.x % LPV;
    const int b = frame_of ? frame_of[p] : 0;
    const unsigned HW = (unsigned)(H * W);
    const unsigned img = HW * pix_bytes;  // pix_bytes >= JP * 4: one channels-last pixel
    const unsigned qo = (unsigned)q * 16u;
    const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
    const float fV = (float)V;
    const int GV = V + (V & 1);
    const long long FN = (long long)s.fine[0] * s.fine[1] * s.fine[2];
    __amdgpu_buffer_rsrc_t grs;
    float rt[6];
    if constexpr (OTF) {
        for (int e = threadIdx.x; e < GV * FVP_CAM_STRIDE; e += 64 * LPV)
            lcam[e] = e < V * FVP_CAM_STRIDE ? pc.cams[e] : 0.0f;
#pragma unroll
        for (int k = 0; k < 6; ++k) rt[k] = pc.resize_t[k];
        __syncthreads();
    } else {
        grs = uniform_rsrc(fgrid, (unsigned)(FN * GV * 8));
    }
    const char *__restrict__ frame_cl = (const char *)cl + (size_t)b * V * img;
    const size_t SS = (size_t)SY * SZ;
    const size_t S3 = (size_t)SX * SS;
    // (planes / cubes start at this joint slice; Jst joints per proposal)
    float *xy_pl = planes ? planes + (size_t)p * Jst * SX * SY : nullptr;
    float *xz_pl = planes ? planes + ((size_t)P + p) * Jst * SX * SZ : nullptr;
    float *yz_pl = planes ? planes + ((size_t)2 * P + p) * Jst * SY * SZ : nullptr;
    const bool zok = zl < SZ;
    const int gz = w.ctl[2] + zl;
    const bool zin = zok && gz >= w.start[2] && gz < w.end[2];
    const int gy = w.ctl[1] + y;
    const bool row_in = gy >= w.start[1] && gy < w.end[1];  // block-uniform

    // plane maxima on the float bits: every voxel value is +0 .. 1 or NaN (the
    // mean is clamped and +0.0f turns a -0 into +0), so unsigned order is float
    // order with NaN on top (torch.max: NaN wins) -- one v_max_u32 per step
    // instead of a NaN-aware float max (compares + select); +0 is neutral
    unsigned yzacc[4] = {0u, 0u, 0u, 0u};

    // xy_direct (host: one x part, one z chunk, S <= 64, LPV <= 4 for every joint
    // slice): the block owns its row's xy cells, so the per-wave z maxima go to LDS
    // and leave as plain stores at the block's end -- no atomics (one per wave and x
    // step cost ~0.6 us per proposal, probe mode 6: non-returning atomics count in
    // vmcnt and the next taps wait on them)
    const bool defer = DXY && planes && xy_direct;
    if (defer) {
        for (int e = lane; e < 64 * 4 * LPV; e += 64) lxy[wave * 64 * 4 * LPV + e] = 0u;
    }
    int x_lo = xpart * SX / xsplit, x_hi = (xpart + 1) * SX / xsplit;
    if (!cubes) {
        // planes only: the x-planes outside the window are all 0, which changes none
        // of the maxima (pre-zeroed xy / xz planes, yzacc >= 0)
        // -- walk the window only
        if (w.skip || !row_in) {
            x_hi = x_lo;
        } else {
            x_lo = max(x_lo, w.start[0] - w.ctl[0]);
            x_hi = min(x_hi, w.end[0] - w.ctl[0]);
        }
    }
    for (int x = x_lo; x < x_hi; ++x) {
        const int gx = w.ctl[0] + x;
        const bool xin = !w.skip && gx >= w.start[0] && gx < w.end[0];
        const bool valid = xin && zin && row_in;
        float acc[4];
        person_voxel_sum<LPV, OTF, CASC, MODE>(acc, valid, gx, gy, gz, grs, lcam, rt, pc, s, frame_cl, img, qo, q, V, GV,
                                               W, H, sxs, sys, pix_bytes);
        float o[4];
        unsigned ou[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // clamp(0,1) of the mean; +0.0f turns a -0 into +0 (unsigned max order below)
            o[k] = valid ? clampf(acc[k] / fV, 0.0f, 1.0f) + 0.0f : 0.0f;
            ou[k] = zok ? __builtin_bit_cast(unsigned, o[k]) : 0u;  // beyond the cube: neutral
        }
        if constexpr (MODE == 1 || MODE == 4) {  // probe: keep the sums live, no planes
            if (offset && zok && (acc[0] + acc[1] + acc[2] + acc[3]) == -1.0f) offset[(size_t)p * 3] = o[0];
            continue;
        }
        if (cubes && zok) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (4 * q + k < J) cubes[((size_t)p * Jst + 4 * q + k) * S3 + ((size_t)x * SY + y) * SZ + zl] = o[k];
        }
        if (planes) {
#pragma unroll
            for (int k = 0; k < 4; ++k) yzacc[k] = max(yzacc[k], ou[k]);
            // this wave's z-range maxima (all lanes: their slot's), four independent
            // VALU chains; lane L < 4 LPV then holds joint 4 (L % LPV) + L / LPV
            unsigned zm[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) zm[k] = slot_umax<LPV>(ou[k]);
            const int kk = lane / LPV;  // q == lane % LPV
            const unsigned mv = kk == 0 ? zm[0] : kk == 1 ? zm[1] : kk == 2 ? zm[2] : zm[3];
            if (defer) {
                if (lane < 4 * LPV) lxy[(wave * 64 + x) * (4 * LPV) + 4 * q + kk] = mv;
            } else if (MODE != 6 && lane < 4 * LPV && 4 * q + kk < J && mv != 0u) {
                // into the pre-zeroed plane (+0 cannot raise it)
                atomicMax(reinterpret_cast<unsigned *>(xy_pl) + ((size_t)(4 * q + kk) * SX + x) * SY + y, mv);
            }
            if (zok) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    // +0 cannot raise the pre-zeroed plane: skip those atomics (most of the 64^3 cube)
                    const unsigned u = ou[k];
                    if (MODE == 8 && 4 * q + k < J && u != 0u)  // probe: plain stores instead (wrong maxima)
                        reinterpret_cast<unsigned *>(xz_pl)[((size_t)(4 * q + k) * SX + x) * SZ + zl] = u;
                    else if (MODE != 5 && MODE != 8 && (MODE != 7 || (zl & 1) == 0) && 4 * q + k < J && u != 0u)
                        atomicMax(reinterpret_cast<unsigned *>(xz_pl) + ((size_t)(4 * q + k) * SX + x) * SZ + zl, u);
                }
            }
        }
    }
    if (planes && zok) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (4 * q + k >= J) continue;
            float *dst = yz_pl + ((size_t)(4 * q + k) * SY + y) * SZ + zl;
            const unsigned u = yzacc[k];
            if (xsplit == 1) *dst = __builtin_bit_cast(float, u);
            else if (u != 0u) atomicMax(reinterpret_cast<unsigned *>(dst), u);  // pre-zeroed plane
        }
    }
    if (defer) {  // xy[j][x][y] = max over the block's waves (z ranges); the plane is pre-zeroed
        __syncthreads();
        // (only the walked x range and values above +0: a row's cells are SY floats
        // apart, and storing the zeros as well -- instead of the memset -- measured
        // slower: 5.45 -> 5.73 us per proposal)
        const int n = (x_hi - x_lo) * J;
        for (int e = threadIdx.x; e < n; e += 64 * LPV) {
            const int xi = x_lo + e / J, j = e - (e / J) * J;
            unsigned m = 0u;
#pragma unroll
            for (int wv = 0; wv < LPV; ++wv) m = max(m, lxy[(wv * 64 + xi) * (4 * LPV) + j]);
            if (MODE != 6 && m != 0u) xy_pl[((size_t)j * SX + xi) * SY + y] = __builtin_bit_cast(float, m);
        }
    }
}

// Small launches (per-frame calls) split each row's x walk over 2-4 blocks.
static int person_xsplit(int P, int SY) {
    const long long rows = (long long)P * SY;
    return rows >= 4096 ? 1 : rows >= 1024 ? 2 : 4;
}

template <int LPV, bool OTF, bool CASC>
static void launch_person_cl(const float *cl, const float *fgrid, const PersonCoords &pc, const float *props,
                             const int32_t *frame_of, const fvp_person_spec &s, float *cubes, float *planes,
                             float *offset, int P, int V, int J, int Jst, int H, int W, unsigned pix_bytes,
                             int xy_direct, hipStream_t st) {
    const int SY = s.bins[1];
    // one y-row per block: with the planes-only fast path for x-planes outside the
    // window, rows are the finer and better balanced unit -- measured (C3, 320
    // proposals): 1 row 6.24, 2 rows 6.85, 4 rows 7.4, 8 rows 8.8 us per proposal
    // (round 2); two rows per block again in round 4 (sequential: 6.04 vs 5.86; two
    // halves combining xz in LDS: 5.98 vs 5.45).  XCD-aware placement keeps a
    // proposal's rows on one XCD.  Small launches (per-frame calls) split each row's
    // x walk over 2-4 blocks (the yz maxima then go through atomics into a
    // pre-zeroed plane).  Cubes deeper than 64 run as 64-deep z chunks, one block
    // each (the xy and xz maxima combine across blocks through atomics; yz is per
    // (y, z)).
    const int xmap = 1, xsplit = person_xsplit(P, SY), zsplit = (s.bins[2] + 63) / 64;
    hipLaunchKernelGGL((person_cl_kernel<LPV, OTF, CASC>), dim3((unsigned)((long long)P * SY * xsplit * zsplit)),
                       dim3(64 * LPV), 0, st, cl, fgrid, pc, props, frame_of, s, cubes, planes, offset, P, V, J, Jst, H,
                       W, xmap, xsplit, zsplit, pix_bytes, xy_direct);
}

}  // namespace fvp

extern "C" int fvp_max_planes(const float *cubes, int P, int J, int S, float *planes, void *stream) {
    if (!cubes || !planes) return FVP_ERR_NULL;
    if (P <= 0) return FVP_OK;
    if (J <= 0 || S <= 0 || S > 4096) return FVP_ERR_SHAPE;
    if (S > 64) {
        const size_t n = (size_t)3 * P * J * S * S;
        hipLaunchKernelGGL(fvp::max_planes_generic_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, cubes, planes, P, J, S);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(fvp::max_planes_kernel, dim3(P * J), dim3(256), 0, (hipStream_t)stream, cubes, planes, P, J,
                       S);
    return (int)hipGetLastError();
}

extern "C" size_t fvp_person_workspace_bytes(int B, int V, int J, int H, int W) {
    if (B <= 0 || V <= 0 || J <= 0 || J > FVP_MAX_JOINTS || H <= 0 || W <= 0) return 0;
    return (size_t)B * fvp::cl_frame_bytes(V, J < 32 ? J : 32, H, W);  // one joint slice at a time
}

namespace fvp {

// heatmaps: planar [B][V][J][H][W] (cp == 0: re-laid out into the workspace
// first) or channels-last [B][V][H][W][cp] (read in place, no workspace).
// More than kPersonSlice joints run in joint slices (layout + launch each).
constexpr int kPersonSlice = 32;

static int person_planes_any(const float *heatmaps, int cp, int B, int V, int J, int H, int W,
                             const float *fine_grid, const PersonCoords *pc, const fvp_person_spec *spec,
                             const float *proposals, const int32_t *frame_of, int P, float *cubes, float *planes,
                             float *offset, void *workspace, size_t workspace_bytes, void *stream) {
    if (!heatmaps || !spec || (!fine_grid && !pc)) return FVP_ERR_NULL;
    if (P <= 0) return FVP_OK;
    if (!proposals) return FVP_ERR_NULL;
    if (B <= 0 || V <= 0 || V > FVP_MAX_VIEWS || J <= 0 || J > FVP_MAX_JOINTS || H < 2 || W < 2) return FVP_ERR_SHAPE;
    if (pc && V > 64) return FVP_ERR_SHAPE;  // camera records staged in LDS
    const int SX = spec->bins[0], SY = spec->bins[1], SZ = spec->bins[2];
    if (SX <= 0 || SY <= 0 || SZ <= 0 || SX > 4096 || SY > 4096 || SZ > 4096 || spec->fine[0] <= 1 ||
        spec->fine[1] <= 1 || spec->fine[2] <= 1)
        return FVP_ERR_SHAPE;
    if (planes && !(SX == SY && SY == SZ)) return FVP_ERR_SHAPE;  // torch.cat of the planes needs a cubic volume
    // packed fine grid addressed with 32-bit byte offsets
    if (!pc && (long long)spec->fine[0] * spec->fine[1] * spec->fine[2] * FVP_GRID_SLOTS(V) * 8 > 0xfffff000LL)
        return FVP_ERR_SHAPE;
    const int J1 = J < kPersonSlice ? J : kPersonSlice;
    if (cp) {
        const int jl = ((J - 1) / kPersonSlice) * kPersonSlice;
        if (cp % 4 || cp < jl + 4 * lanes_per_voxel(J - jl) || (size_t)H * W * cp * 4 > 0x7fffffffull)
            return FVP_ERR_SHAPE;
    } else {
        const size_t need = (size_t)B * cl_frame_bytes(V, J1, H, W);
        if (!workspace || workspace_bytes < need) return FVP_ERR_WORKSPACE;
    }
    hipStream_t st = (hipStream_t)stream;
    // xy maxima stored by their row's block without atomics (person_cl_kernel
    // xy_direct): one x part, one z chunk, S <= 64 and every joint slice at <= 4
    // lanes per voxel
    const int xsplit = person_xsplit(P, SY);
    const int xy_direct = (planes && xsplit == 1 && SZ <= 64 && SX <= 64 && J <= 16) ? 1 : 0;
    if (planes) {  // xy, xz (and yz when x is split) hold maxima over non-negative floats: from +0
        const size_t n = (xsplit > 1 ? 3 : 2) * (size_t)P * J * SX * SY;
        const hipError_t e = hipMemsetAsync(planes, 0, n * 4, st);
        if (e != hipSuccess) return (int)e;
    }
    const PersonCoords none{};
    const PersonCoords &c = pc ? *pc : none;
    const size_t HW = (size_t)H * W, S2 = (size_t)SX * SY, S3 = S2 * SZ;
    for (int j0 = 0; j0 < J; j0 += kPersonSlice) {
        const int Jc = J - j0 < kPersonSlice ? J - j0 : kPersonSlice;
        const float *cl = cp ? heatmaps + j0 : reinterpret_cast<const float *>(workspace);
        const unsigned pix_bytes = 4u * (unsigned)(cp ? cp : 4 * lanes_per_voxel(Jc));
        float *cb = cubes ? cubes + j0 * S3 : nullptr;
        float *pl = planes ? planes + j0 * S2 : nullptr;
#define FVP_PERSON_CASE(L)                                                                                            \
    if (!cp) launch_layout<L, float>(heatmaps + j0 * HW, B, V, Jc, J, H, W, reinterpret_cast<float *>(workspace), st); \
    if (pc && V > 16)                                                                                                 \
        launch_person_cl<L, true, true>(cl, nullptr, c, proposals, frame_of, *spec, cb, pl, offset, P, V, Jc, J, H,   \
                                        W, pix_bytes, xy_direct, st);                                                            \
    else if (pc)                                                                                                      \
        launch_person_cl<L, true, false>(cl, nullptr, c, proposals, frame_of, *spec, cb, pl, offset, P, V, Jc, J, H,  \
                                         W, pix_bytes, xy_direct, st);                                                           \
    else if (V > 16)                                                                                                  \
        launch_person_cl<L, false, true>(cl, fine_grid, c, proposals, frame_of, *spec, cb, pl, offset, P, V, Jc, J,   \
                                         H, W, pix_bytes, xy_direct, st);                                                        \
    else                                                                                                              \
        launch_person_cl<L, false, false>(cl, fine_grid, c, proposals, frame_of, *spec, cb, pl, offset, P, V, Jc, J,  \
                                          H, W, pix_bytes, xy_direct, st);                                                       \
    break;
        switch (lanes_per_voxel(Jc)) {
            case 1: FVP_PERSON_CASE(1)
            case 2: FVP_PERSON_CASE(2)
            case 4: FVP_PERSON_CASE(4)
            default: FVP_PERSON_CASE(8)
        }
#undef FVP_PERSON_CASE
    }
    return (int)hipGetLastError();
}

}  // namespace fvp

extern "C" int fvp_person_planes(const float *heatmaps, int B, int V, int J, int H, int W, const float *fine_grid,
                                 const fvp_person_spec *spec, const float *proposals, const int32_t *frame_of, int P,
                                 float *cubes, float *planes, float *offset, void *workspace, size_t workspace_bytes,
                                 void *stream) {
    if (!fine_grid) return FVP_ERR_NULL;
    return fvp::person_planes_any(heatmaps, 0, B, V, J, H, W, fine_grid, nullptr, spec, proposals, frame_of, P,
                                  cubes, planes, offset, workspace, workspace_bytes, stream);
}

extern "C" int fvp_person_planes_cams(const float *heatmaps, int B, int V, int J, int H, int W, const float *cams,
                                      const float *resize_t, const fvp_grid_spec *fine_grid_spec,
                                      const fvp_image_spec *img, const fvp_person_spec *spec, const float *proposals,
                                      const int32_t *frame_of, int P, float *cubes, float *planes, float *offset,
                                      void *workspace, size_t workspace_bytes, void *stream) {
    if (!cams || !resize_t || !fine_grid_spec || !img) return FVP_ERR_NULL;
    if (img->hm_w != W || img->hm_h != H) return FVP_ERR_SHAPE;
    for (int a = 0; a < 3; ++a)
        if (fine_grid_spec->bins[a] != spec->fine[a]) return FVP_ERR_SHAPE;
    const fvp::PersonCoords pc{cams, resize_t, *fine_grid_spec, fvp::image_consts(*img)};
    return fvp::person_planes_any(heatmaps, 0, B, V, J, H, W, nullptr, &pc, spec, proposals, frame_of, P, cubes,
                                  planes, offset, workspace, workspace_bytes, stream);
}

extern "C" int fvp_person_planes_cl(const float *heatmaps_cl, int cp, int B, int V, int J, int H, int W,
                                    const float *fine_grid, const fvp_person_spec *spec, const float *proposals,
                                    const int32_t *frame_of, int P, float *cubes, float *planes, float *offset,
                                    void *stream) {
    if (!fine_grid) return FVP_ERR_NULL;
    if (cp <= 0) return FVP_ERR_SHAPE;
    return fvp::person_planes_any(heatmaps_cl, cp, B, V, J, H, W, fine_grid, nullptr, spec, proposals, frame_of, P,
                                  cubes, planes, offset, nullptr, 0, stream);
}
