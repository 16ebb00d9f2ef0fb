/*
 * fvp.h -- C ABI of the MI355X-native Faster-VoxelPose voxel-projection path.
 *
 * One shared library (libfvp.so, built from faster-voxelpose_amd/csrc) exports
 * these entry points.  They are plain C: device pointers, sizes and a HIP
 * stream handle (hipStream_t passed as void*).  Every call is asynchronous on
 * that stream, allocates nothing, never synchronises, and returns a status
 * (0 = success, otherwise a hipError_t value; FVP_ERR_* for argument errors).
 *
 * The reference has no FFI: its boundary is Python nn.Module classes reached
 * by module path.  Each entry point below names the
 * reference code it replaces (paths relative to the reference repo).  The
 * Python mirror of the reference interface (faster-voxelpose_amd/fvp) binds
 * these with ctypes and registers them as torch.ops.fvp.* custom ops.
 *
 * Layouts (all row-major, fp32 unless noted):
 *   heatmaps      [B][V][J][H][W]      (as handed to ProjectLayer.forward)
 *   cams          [V][FVP_CAM_STRIDE]  packed camera records (see below)
 *   sample_grid   [V][N][2]            N = X*Y*Z, voxel n = (ix*Y+iy)*Z+iz
 *   packed grid   [N][FVP_GRID_SLOTS(V)][2]  voxel-major copy read by fvp_voxelize
 *   cube          [B][J][X][Y][Z]
 *   xy            [B][J][X][Y]
 */
#ifndef FVP_H
#define FVP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FVP_ABI_VERSION 22
/* Joints per heatmap set: the voxelize and person kernels run up to 32 joints
 * per pass (one channels-last pixel of 32 floats per tap) and more in joint
 * slices of 32. */
#define FVP_MAX_JOINTS 1024
/* Cameras per frame: torch's CPU mean over the views (the sum order every
 * kernel reproduces) folds blocks of 16 into a second accumulator, and past
 * 255 views into a third; up to 255 views are supported. */
#define FVP_MAX_VIEWS 255
#define FVP_CAM_STRIDE 24 /* R[9] T[3] fx fy cx cy k[3] p[2] pad[3] */
/* Camera slots per voxel in a packed grid (V rounded up to even). */
#define FVP_GRID_SLOTS(V) ((V) + ((V) & 1))

/* Argument errors (distinct from hipError_t values, which are < 1000). */
#define FVP_OK 0
#define FVP_ERR_NULL 1001     /* a required pointer is NULL */
#define FVP_ERR_SHAPE 1002    /* a size is <= 0 or exceeds a kernel limit */
#define FVP_ERR_WORKSPACE 1003 /* workspace missing or smaller than fvp_voxelize_workspace_bytes() */

/* Voxel-grid description: centre_i = linspace(start, end, bins)[i] + center
 * per axis, fp32, exactly as compute_grid (lib/models/project_whole.py:43-79). */
typedef struct fvp_grid_spec {
    float start[3];  /* -SPACE_SIZE/2 */
    float end[3];    /* +SPACE_SIZE/2 */
    float center[3]; /* SPACE_CENTER */
    int32_t bins[3]; /* VOXELS_PER_AXIS (or fine_voxels_per_axis) */
} fvp_grid_spec;

/* Image geometry used when building a sample grid (project_whole.py:81-117). */
typedef struct fvp_image_spec {
    float ori_max;  /* max(ORI_IMAGE_SIZE): the upper clamp, project_whole.py:100 */
    float img_w, img_h; /* IMAGE_SIZE */
    int32_t hm_w, hm_h; /* HEATMAP_SIZE */
} fvp_image_spec;

/* Per-person layer constants (lib/models/project_individual.py:43-85). */
typedef struct fvp_person_spec {
    int32_t fine[3];      /* fine_voxels_per_axis, e.g. 253,253,64 */
    float scale[3];       /* (fine-1)/whole_space_size */
    float bias[3];
    float whole_size[3];  /* CAPTURE_SPEC.SPACE_SIZE */
    float ind_size[3];    /* INDIVIDUAL_SPEC.SPACE_SIZE */
    int32_t bins[3];      /* INDIVIDUAL_SPEC.VOXELS_PER_AXIS, e.g. 64,64,64 */
} fvp_person_spec;

int fvp_abi_version(void);
const char *fvp_status_string(int status);

/* Sample grid of one sequence: for each camera v and voxel n, project the
 * voxel centre (lib/utils/cameras.py:30-56), clamp to [-1, ori_max], apply
 * resize_transform (lib/utils/transforms.py:59-63), scale to heatmap pixels,
 * normalise to [-1,1] and clamp to +-1.1.
 * Replaces ProjectLayer.project_grid x V (project_whole.py:81-117, :151-156)
 * and compute_sample_grid (project_individual.py:192-220).
 *   cams        device [V][FVP_CAM_STRIDE]
 *   resize_t    device [2][3]
 *   sample_grid device [V][N][2] (output) */
int fvp_project_grid(const float *cams, int V, const float *resize_t,
                     const fvp_grid_spec *grid, const fvp_image_spec *img,
                     float *sample_grid, void *stream);

/* Voxel-major copy of a sample grid, the layout fvp_voxelize reads:
 *   packed[n][v][:] = sample_grid[v][n][:] for v < V; padding slots = (-2,-2)
 * (off-image).  Built once per sequence, like the grid itself.  The LPV lanes
 * that share a voxel read 2*LPV cameras' coordinates with one 16-B load each.
 *   sample_grid device [V][N][2];  packed device [N][FVP_GRID_SLOTS(V)][2] */
int fvp_pack_grid(const float *sample_grid, int V, long long N, float *packed, void *stream);

/* Whole-space voxelisation fused with the xy max-projection:
 *   cube[b,j,n] = clamp(mean_v grid_sample(heatmaps[b,v,j], sample_grid[g(b),v,n]), 0, 1)
 *   xy[b,j,x,y] = max_z cube[b,j,x,y,z]
 * Replaces ProjectLayer.forward (project_whole.py:119-168) and the first line
 * of CenterNet.forward (lib/models/cnns_2d.py:291).
 *   packed_grids device [n_grids][N][FVP_GRID_SLOTS(V)][2] (fvp_pack_grid)
 *   grid_index   device int32 [B] (grid of frame b, 0 <= g < n_grids: a precondition,
 *                checked by fvp.ops on host tensors) or NULL (all frames use grid 0)
 *   cube, xy     device outputs; either may be NULL to skip it
 *   workspace    device scratch of >= fvp_voxelize_workspace_bytes(B,V,J,H,W)
 *                bytes (channels-last copy of a chunk of frames; of one 32-joint slice
 *                when J > 32); J <= FVP_MAX_JOINTS */
size_t fvp_voxelize_workspace_bytes(int B, int V, int J, int H, int W);
int fvp_voxelize(const float *heatmaps, int B, int V, int J, int H, int W,
                 const float *packed_grids, const int32_t *grid_index,
                 int X, int Y, int Z, float *cube, float *xy,
                 void *workspace, size_t workspace_bytes, void *stream);
/* Same with fp16 heatmaps (IEEE binary16), computed in fp32 (exact upcast).
 * For J <= 16 the chunk is re-laid out as an fp16 pixel-pair table (each
 * 64-B entry holds pixels x and x+1 of a row), so a voxel-camera is 2 loads
 * per frame, with 4 frames interleaved per entry (a batch's remainder in
 * entries of 2 and 1); the workspace size differs from the fp32 one and depends
 * on the arguments only. */
size_t fvp_voxelize_f16_workspace_bytes(int B, int V, int J, int H, int W);
int fvp_voxelize_f16(const void *heatmaps, int B, int V, int J, int H, int W,
                     const float *packed_grids, const int32_t *grid_index,
                     int X, int Y, int Z, float *cube, float *xy,
                     void *workspace, size_t workspace_bytes, void *stream);

/* Same operation with the sampling coordinates projected on the fly from the
 * camera records (the exact fp32 sequence of fvp_project_grid) instead of read
 * from a cached grid: for configurations whose grid would not stay
 * cache-resident (e.g. 31 cameras x 160x160x64 = 420 MB per sequence).
 *   half       0: heatmaps fp32, 1: fp16 (workspace as fvp_voxelize[_f16])
 *   cams       device [n_seq][V][FVP_CAM_STRIDE]; grid_index selects the sequence
 *   resize_t   device [2][3];  grid, img as for fvp_project_grid
 *              (X,Y,Z = grid->bins; img->hm_w/hm_h must equal W/H) */
int fvp_voxelize_cams(const void *heatmaps, int half, int B, int V, int J, int H, int W,
                      const float *cams, const int32_t *grid_index, const float *resize_t,
                      const fvp_grid_spec *grid, const fvp_image_spec *img, float *cube, float *xy,
                      void *workspace, size_t workspace_bytes, void *stream);

/* fvp_voxelize_cams for the voxels of x-rows [x_begin, x_end) of the grid only
 * (0 <= x_begin < x_end <= grid->bins[0]): cube [B][J][x_end-x_begin][Y][Z],
 * xy [B][J][x_end-x_begin][Y].  Every voxel's coordinates come from its global
 * indices, so the slab equals the same rows of the whole-grid call bit for bit,
 * without any sample grid -- the large-frame mode of SURVEY.md §8(e), where each
 * rank of a group voxelises one x-slab of every frame (the per-sequence cache
 * of project_whole.py:151-156 is never built). */
int fvp_voxelize_cams_slab(const void *heatmaps, int half, int B, int V, int J, int H, int W,
                           const float *cams, const int32_t *grid_index, const float *resize_t,
                           const fvp_grid_spec *grid, const fvp_image_spec *img, int x_begin, int x_end,
                           float *cube, float *xy, void *workspace, size_t workspace_bytes, void *stream);

/* fvp_voxelize / fvp_voxelize_cams on heatmaps that are already channels-last,
 * [B][V][H][W][cp] fp32 with cp >= 4*ceil(J/4) rounded to {4, 8, 16, 32} and
 * cp % 4 == 0 (joints j < J in channels 0..J-1, the rest ignored) -- the NHWC
 * output of the PoseResNet backbone's final layer (fvp.backbone; resnet.py:122-128,
 * "emit heatmaps directly in the kernel's channels-last
 * layout, removing a transpose pass").  Same results bit for bit as the planar
 * entry points on the same values; no layout pass, no workspace, one launch. */
int fvp_voxelize_cl(const float *heatmaps_cl, int cp, int B, int V, int J, int H, int W,
                    const float *packed_grids, const int32_t *grid_index, int X, int Y, int Z, float *cube,
                    float *xy, void *stream);
int fvp_voxelize_cl_cams(const float *heatmaps_cl, int cp, int B, int V, int J, int H, int W, const float *cams,
                         const int32_t *grid_index, const float *resize_t, const fvp_grid_spec *grid,
                         const fvp_image_spec *img, float *cube, float *xy, void *stream);
int fvp_voxelize_cl_cams_slab(const float *heatmaps_cl, int cp, int B, int V, int J, int H, int W,
                              const float *cams, const int32_t *grid_index, const float *resize_t,
                              const fvp_grid_spec *grid, const fvp_image_spec *img, int x_begin, int x_end,
                              float *cube, float *xy, void *stream);

/* Peak NMS + top-K on a [B,1,X,Y] map: 3x3 max-pool keep mask, top-K of the
 * masked map (value descending, flat index ascending on ties), and
 * get_index2D's (flat // X, flat % X) decode.
 * Replaces nms2D / max_pool2D / get_index2D (lib/core/proposal.py:13-76).
 *   prob         frame b's X*Y map starts at prob + b*frame_stride (0 = X*Y),
 *                so one channel of the xy planes can be passed without a copy
 *   vals [B][K] fp32, flat [B][K] int64, xy [B][K][2] int64 (xy may be NULL) */
int fvp_nms_topk(const float *prob, int B, int X, int Y, long long frame_stride, int K,
                 float *vals, int64_t *flat, int64_t *xy, void *stream);

/* ProposalLayer.forward in test mode (lib/models/human_detection_net.py:
 * 36-37, 99-124), optionally fused with the z pick of HumanDetectionNet.forward
 * (:208-215).  With hm1d (index_dims == 2):
 *   z    = argmax_z hm1d[b,k,:] (torch.topk(1): NaN first, lowest index on ties)
 *   conf = confs[b,k] * hm1d[b,k,z]
 * without (hm1d NULL, index_dims == 3): z = index[b,k,2], conf = confs[b,k]; then
 *   centers[b,k] = [ix*sx+bx, iy*sy+by, z*sz+bz, (conf > min_score) - 1, conf, bbox[b,k,0:2]]
 *   index  device int64 [B][K][index_dims] (nms2D topk_index, or the full 3-D index)
 *   hm1d   device [B][K][Z] or NULL;  confs device [B][K];  bbox device [B][K][2]
 *   scale3 / bias3 HOST float[3] = SPACE_SIZE/(VOXELS-1) and SPACE_CENTER-SPACE_SIZE/2 (fp32)
 *   centers device [B][K][7]. */
int fvp_proposal_centers(const int64_t *index, int index_dims, const float *hm1d, const float *confs,
                         const float *bbox, int B, int K, int Z, const float *scale3, const float *bias3,
                         float min_score, float *centers, void *stream);

/* fvp_nms_topk fused with fvp_gather_columns for a map of the cube's own
 * X x Y grid: the winners' z-columns columns[b,k,j,:] = cube[b,j,flat[b,k],:]
 * come from the same launch (K <= 16; larger K: two launches).
 *   cube device [B][J][X][Y][Z];  columns device [B][K][J][Z] */
int fvp_nms_topk_columns(const float *prob, int B, int X, int Y, long long frame_stride, int K, float *vals,
                         int64_t *flat, int64_t *xy, const float *cube, int J, int Z, float *columns, void *stream);
/* z-columns of the top-K proposals: columns[b,k,j,:] = cube[b,j,flat[b,k],:]
 * (an index outside [0, X*Y) reads nothing and yields NaN; torch.gather raises)
 * Replaces the torch.gather at lib/models/human_detection_net.py:199-200. */
int fvp_gather_columns(const float *cube, int B, int J, int X, int Y, int Z,
                       const int64_t *flat, int K, float *columns, void *stream);

/* The same z-columns recomputed from the heatmaps for the K winners only, so
 * a caller that needs the cube just for them (HumanDetectionNet.forward,
 * human_detection_net.py:162-200) can run fvp_voxelize without the cube:
 * bit-identical to fvp_gather_columns on the cube fvp_voxelize (packed_grids
 * != NULL) or fvp_voxelize_cams (packed_grids == NULL: cams, resize_t, grid,
 * img as there) would write.  Heatmaps are read in place through strides, in
 * elements: planar [B][V][J][H][W] -> (J*H*W, H*W, 1), channels-last
 * [B][V][H][W][cp] -> (H*W*cp, 1, cp) (from the first joint's element);
 * half = fp16 heatmaps.  columns device [B][K][J][Z] (NaN for an index
 * outside the map).  Precondition (as fvp_voxelize): a device grid_index holds
 * 0 <= grid_index[b] < the number of sequences packed in packed_grids / cams;
 * it is not range-checked on the device (the Python wrapper checks host
 * indices). */
int fvp_voxel_columns(const void *heatmaps, int half, long long view_stride, long long joint_stride,
                      int pix_stride, int B, int V, int J, int H, int W, const float *packed_grids,
                      const float *cams, const float *resize_t, const fvp_grid_spec *grid,
                      const fvp_image_spec *img, const int32_t *grid_index, int X, int Y, int Z,
                      const int64_t *flat, int K, float *columns, void *stream);

/* bbox sizes at the top-K: out[b,k,c] = size[b,c,flat[b,k]] (c = 0,1; NaN for an index outside the map)
 * Replaces the torch.gather at lib/models/human_detection_net.py:191-192. */
int fvp_gather_bbox(const float *size, int B, int X, int Y,
                    const int64_t *flat, int K, float *out, void *stream);

/* Per-person voxelisation of a batch of proposals from the cached fine
 * sample grid, optionally fused with the JLN max-projections.
 * Replaces project_individual.ProjectLayer.forward (project_individual.py:222-293)
 * and torch.cat([max(c,4), max(c,3), max(c,2)]) (joint_localization_net.py:158-160).
 *   heatmaps    device [B][V][J][H][W] (the frames the proposals refer to)
 *   fine_grid   device packed fine grid [FX*FY*FZ][FVP_GRID_SLOTS(V)][2] (fvp_pack_grid)
 *   proposals   device [P][7] (x,y,z mm, gt, conf, bbox_w, bbox_h)
 *   frame_of    device int32 [P]: frame of each proposal in [0,B) (NULL: all frame 0)
 *   cubes       device [P][J][SX][SY][SZ] or NULL (outside-window voxels are 0)
 *   planes      device [3P][J][S][S] or NULL: xy (max over z) for p < P, then xz
 *               (max over y), then yz (max over x); needs SX == SY == SZ (any size:
 *               cubes deeper than 64 run in 64-deep z chunks, joints in slices of 32)
 *   offset      device [P][3] or NULL
 *   workspace   >= fvp_person_workspace_bytes(B,V,J,H,W) bytes (channels-last frames) */
size_t fvp_person_workspace_bytes(int B, int V, int J, int H, int W);
int fvp_person_planes(const float *heatmaps, int B, int V, int J, int H, int W,
                      const float *fine_grid, const fvp_person_spec *spec,
                      const float *proposals, const int32_t *frame_of, int P,
                      float *cubes, float *planes, float *offset,
                      void *workspace, size_t workspace_bytes, void *stream);
/* Same with the fine-grid sampling coordinates projected on the fly from the
 * camera records (the fp32 sequence of fvp_project_grid over the fine
 * whole-space grid) instead of read from the 197 MB (5 cameras) packed fine
 * grid -- no per-sequence fine-grid build.
 *   cams            device [V][FVP_CAM_STRIDE] (V <= 64)
 *   resize_t        device [2][3]
 *   fine_grid_spec  the fine whole-space grid (bins == spec->fine)
 *   img             image geometry (hm_w/hm_h == W/H) */
int fvp_person_planes_cams(const float *heatmaps, int B, int V, int J, int H, int W,
                           const float *cams, const float *resize_t, const fvp_grid_spec *fine_grid_spec,
                           const fvp_image_spec *img, const fvp_person_spec *spec,
                           const float *proposals, const int32_t *frame_of, int P,
                           float *cubes, float *planes, float *offset,
                           void *workspace, size_t workspace_bytes, void *stream);
/* fvp_person_planes on channels-last heatmaps [B][V][H][W][cp] (cp as
 * fvp_voxelize_cl; e.g. the backbone's NHWC output): read in place, no
 * layout pass, no workspace. */
int fvp_person_planes_cl(const float *heatmaps_cl, int cp, int B, int V, int J, int H, int W, const float *fine_grid,
                         const fvp_person_spec *spec, const float *proposals, const int32_t *frame_of, int P,
                         float *cubes, float *planes, float *offset, void *stream);

/* xy / xz / yz max-projections of per-person cubes [P][J][S][S][S] into
 * planes [3P][J][S][S] (xy block first, then xz, then yz).
 * Replaces torch.cat([max(c,4), max(c,3), max(c,2)]) at
 * lib/models/joint_localization_net.py:158-160.  S <= 4096 (S > 64: one thread per plane cell). */
int fvp_max_planes(const float *cubes, int P, int J, int S, float *planes, void *stream);

/* JLN soft-argmax of the per-plane joint maps plus the offset shift:
 *   softmax(beta * x) over the S2 = S*S cells of each (plane, proposal, joint),
 *   pose = expectation of center_grid[plane] + offset (xy: x,y; xz: x,z; yz: y,z)
 *   maxprob = max of the softmax
 * Replaces SoftArgmaxLayer.forward (lib/models/joint_localization_net.py:32-56)
 * and the offset additions of JointLocalizationNet.forward (:170-174).
 *   features    device [3][P][J][S2] (P2PNet output, chunked and stacked by plane)
 *   center_grid device [3][S2][2] (project_individual.ProjectLayer.center_grid)
 *   offset      device [P][3] or NULL;  pose [3][P][J][2], maxprob [3][P][J] outputs */
int fvp_soft_argmax(const float *features, int P, int J, int S2, const float *center_grid,
                    const float *offset, float beta, float *pose, float *maxprob, void *stream);

/* Three-plane fusion and the per-proposal confidence:
 *   fused[p,j] = weighted (x from xy/xz, y from xy/yz, z from xz/yz), weights
 *   normalised per axis; confs[p] = mean over planes and joints of maxprob.
 * Replaces fuse_pose_preds (joint_localization_net.py:83-120) and the confs
 * mean of SoftArgmaxLayer.forward (:49-50).
 *   weights device [3P][J] (WeightNet output);  fused [P][J][3], confs [P] (either may be NULL) */
int fvp_fuse_poses(const float *pose, const float *weights, const float *maxprob, int P, int J,
                   float *fused, float *confs, void *stream);
/* torch.nonzero of a [rows][cols] bool mask (uint8, contiguous), one launch:
 * idx [rows*cols][2] int64 receives the (row, col) of the true entries in
 * row-major order (the first *count rows are written), count device int
 * (joint_localization_net.py:136-137's boolean selections as indices). */
int fvp_mask_nonzero(const unsigned char *mask, int rows, int cols, long long *idx, int *count, void *stream);
/* The same, plus (each optional) frame_of [rows*cols] int32 = the row of each selected entry and
 * rowdst [rows*cols][width] = rowsrc[row * rs0 + col * rs1 + 0 .. width) (floats): the JLN's
 * selected frames and proposal rows (joint_localization_net.py:140-151) from the same launch,
 * so that after its one host sync only views remain. */
int fvp_mask_select(const unsigned char *mask, int rows, int cols, long long *idx, int *count, int *frame_of,
                    const float *rowsrc, long long rs0, long long rs1, int width, float *rowdst, void *stream);
/* The JLN's result scatters (joint_localization_net.py:176-180) in one launch:
 * for p < P with (b, k) = idx[p]: all_fused [B][K][J][3] <- fused [P][J][3],
 * all_pose [3][B][K][J][2] <- pose [3][P][J][2], and (centers non-NULL)
 * centers[b * cs0 + k * cs1 + conf_col] <- confs[p]. */
int fvp_scatter_poses(const long long *idx, int P, int B, int K, int J, const float *fused, const float *pose,
                      const float *confs, float *all_fused, float *all_pose, float *centers, long long cs0,
                      long long cs1, int conf_col, void *stream);

/* Dense 2-D convolution on the fp32 matrix cores (v_mfma_f32_32x32x2_f32),
 * implicit GEMM over NHWC activations, for the HDN / JLN CNNs
 * (lib/models/cnns_2d.py:12-295, weight_net.py:48-80):
 *   out = act(conv(in, W) * scale + shift + res_pre) + res_post
 * with eval-mode BatchNorm and the conv bias folded into scale/shift, act =
 * ReLU when relu != 0.  Stride 1, zero padding (K-1)/2, odd KH/KW.
 * upsample2 == 1: ConvTranspose2d(k=2, s=2) as a 1x1 conv with 4*Cpo packed
 * outputs n = (dy*2+dx)*Cpo + co, scattered to the 2H x 2W output.
 * upsample2 == 2: ConvTranspose1d(k=2, s=2) (cnns_1d.py:96-123) on rows of
 * H == 1 (1-D tensors [N][C][L] run as [N][1][L][Cp]): 2*Cpo packed outputs
 * n = dx*Cpo + co, scattered to the H x 2W output.  Conv1d(k) is KH = 1, KW = k.
 *   in        device [N][H][W][Cpi], Cpi % 16 == 0 (padding channels zero)
 *   wpack     device [KH*KW*Cpi][Cpo_w], row (ky*KW+kx)*Cpi+ci, Cpo_w % 128 == 0
 *   scale, shift device [Cpo];  res_pre, res_post device [N][Ho][Wo][Cpo] or NULL
 *   out       device [N][Ho][Wo][Cpo], Cpo % 16 == 0 */
int fvp_conv2d_nhwc(const float *in, int N, int H, int W, int Cpi, const float *wpack, int KH, int KW,
                    int Cpo, int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                    const float *res_post, int relu, int upsample2, float *out, void *stream);
/* Kernel selection of fvp_conv2d_nhwc_ws (every choice computes the same
 * convolution; they differ in tiling only, and tests run each of them):
 *   FVP_CONV_AUTO            halo-tiled KxK kernel where measured faster,
 *                            per-tap kernel elsewhere, split-K where a per-tap
 *                            launch is under-filled (what fvp_conv2d_nhwc runs)
 *   FVP_CONV_PER_TAP         per-tap kernel on every layer (split-K as AUTO)
 *   FVP_CONV_HALO            halo-tiled kernel on every eligible layer
 *   FVP_CONV_PER_TAP_NOSPLIT per-tap kernel, never split */
#define FVP_CONV_AUTO 0
#define FVP_CONV_PER_TAP 1
#define FVP_CONV_HALO 2
#define FVP_CONV_PER_TAP_NOSPLIT 3
/* Same with a kernel choice and a device scratch for split-K: launches under
 * one block per CU with a long K walk (small maps, many channels) split the K
 * loop over blocks and combine the partial sums in a fixed order.  workspace
 * may be NULL or smaller than fvp_conv2d_workspace_bytes() of the same algo
 * (then no split); 0 bytes = the layer does not split. */
size_t fvp_conv2d_workspace_bytes(int N, int H, int W, int Cpi, int KH, int KW, int Cpo, int upsample2, int algo);
int fvp_conv2d_nhwc_ws(const float *in, int N, int H, int W, int Cpi, const float *wpack, int KH, int KW,
                       int Cpo, int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                       const float *res_post, int relu, int upsample2, float *out, int algo, void *workspace,
                       size_t workspace_bytes, void *stream);
/* Same convolution with bf16 operands (opt-in precision): activations are
 * rounded to bf16 when staged, weights given as bf16 [Cpo_w][KH*KW*Cpi]
 * (output-channel major), products accumulated in fp32 on
 * v_mfma_f32_32x32x16_bf16.  Other arguments as fvp_conv2d_nhwc. */
int fvp_conv2d_nhwc_bf16(const float *in, int N, int H, int W, int Cpi, const void *wpack_bf16, int KH, int KW,
                         int Cpo, int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                         const float *res_post, int relu, int upsample2, float *out, void *stream);
/* Generalised convolution geometry (same kernels), for the PoseResNet heatmap
 * backbone (lib/models/resnet.py:98-201, called at faster_voxelpose.py:73-75;
 * SURVEY.md §8(f) rank 4) as well as the CNNs above:
 *   mode 0  Conv2d with stride (sy, sx) in 1..4 and zero padding (py, px) < K
 *           (any KH, KW): output Ho = (H + 2py - KH)/sy + 1, Wo likewise
 *           (resnet.py:105 7x7/s2/p3, :64 3x3/s2/p1, :134 1x1/s2, :62/:67 1x1);
 *   mode 1  ConvTranspose2d(k=2, s=2)  (upsample2 == 1 above)
 *   mode 2  ConvTranspose1d(k=2, s=2)  (upsample2 == 2 above)
 *   mode 3  ConvTranspose2d(k=4, s=2, p=1, output_padding 0) (resnet.py:173-180,
 *           NUM_DECONV_KERNELS = 4): Ho = 2H, Wo = 2W, as four 2x2 convolutions
 *           over the input grid, one per output parity g = ry*2 + rx; KH = KW = 2,
 *           wpack [4][Krows][Cpo_w] with row (i*2+j)*Cpi+ci of group g holding
 *           W[ci][co][3-2i-ry][3-2j-rx]; sy, sx, py, px are ignored.
 *   in     device [N][H][W][Cpi]: Cpi % 16 == 0, or Cpi in {4, 8, 12} (an RGB
 *          input padded to 4 channels; a K chunk then spans several taps)
 *   wpack  fp32: [G][Krows][Cpo_w], Krows = KH*KW*Cpi rounded up to 16 (zero
 *          rows), G = 4 for mode 3 else 1;  bf16 & FVP_CONV_BF16: bf16 operands,
 *          wpack bf16 [G][Cpo_w][Krows] (no split-K; a 4/8/12-channel input
 *          must be fp32); with
 *          them, FVP_CONV_BF16_IN: `in` holds bf16 activations, FVP_CONV_BF16_OUT:
 *          `out`, res_pre and res_post hold bf16 (the pointers are reinterpreted)
 *   out    device [N][Ho][Wo][Cpo];  res_pre / res_post likewise or NULL
 *   algo   FVP_CONV_* (the halo kernel serves stride-1 "same" fp32 convolutions);
 *   workspace as fvp_conv2d_nhwc_ws, sized by fvp_conv2d_ex_workspace_bytes. */
int fvp_conv2d_nhwc_ex(const float *in, int N, int H, int W, int Cpi, const void *wpack, int KH, int KW, int Cpo,
                       int Cpo_w, const float *scale, const float *shift, const float *res_pre,
                       const float *res_post, int relu, int mode, int sy, int sx, int py, int px, int bf16,
                       int algo, float *out, void *workspace, size_t workspace_bytes, void *stream);
#define FVP_CONV_BF16 1
#define FVP_CONV_BF16_IN 2
#define FVP_CONV_BF16_OUT 4
/* fp32 operands with the weights given k-contiguous, wpack fp32
 * [G][Cpo_w][Krows] (the bf16 layout): runs the LDS-DMA staged kernel
 * (Cpi % 16 == 0, activations and weights under 2 GiB, KH*KW <= 32, N*Hm*Wm
 * < 2^24, else FVP_ERR_SHAPE; no split-K, algo ignored).  Same fp32 products,
 * summed in another order than the [Krows][Cpo_w] kernels. */
#define FVP_CONV_F32_KC 8
size_t fvp_conv2d_ex_workspace_bytes(int N, int H, int W, int Cpi, int KH, int KW, int Cpo, int mode, int sy,
                                     int sx, int py, int px, int algo);
/* 3x3 stride-1 padding-1 Conv2d (cnns_2d.py:12-64 Basic2DBlock / Res2DBlock
 * 3x3 layers; resnet.py:60-95 Bottleneck conv2 at stride 1) by Winograd
 * F(2x2, 3x3) on the fp32 matrix cores, with the epilogue of
 * fvp_conv2d_nhwc_ex (out = act(acc * scale + shift + res_pre) + res_post):
 *   in    device [N][H][W][Cpi] fp32, Cpi % 16 == 0
 *   u     device [16][Cpi/16][4][Cpo][4] fp32: U = G g G^T of the [Cout][Cin][3][3]
 *         weights, G = [[1,0,0],[1/2,1/2,1/2],[1/2,-1/2,1/2],[0,0,1]], element
 *         (xi = 4r + s, step k, cm, co, c4) = U[co][ci = 16k + 4c4 + cm][r][s]
 *         (zero for padding channels)
 *   out   device [N][H][W][Cpo] fp32, Cpo % 32 == 0
 *   pool  device [N][H/2][W/2][Cpo] fp32 or NULL: F.max_pool2d(out, 2, 2) (NaN-propagating,
 *         the window order of fvp_maxpool_nhwc) written by the same launch
 * The transforms are exact sums and differences (the weight transform is the
 * caller's, in fp64): the result equals the direct convolution up to their
 * rounding.  FVP_ERR_SHAPE otherwise. */
int fvp_conv3x3_wino_nhwc(const float *in, int N, int H, int W, int Cpi, const float *u, int Cpo, const float *scale,
                          const float *shift, const float *res_pre, const float *res_post, int relu, float *out,
                          float *pool, void *stream);
/* ConvTranspose2d(kernel 4, stride 2, padding 1) (resnet.py:147-158, the
 * PoseResNet deconvolution head) by Winograd F(2x2, 2x2) on the fp32 matrix
 * cores, one 2x2 convolution per output parity (ry, rx): output (2y+ry, 2x+rx)
 * = sum_{i,j} W[ci][co][3-2i-ry][3-2j-rx] in[y-1+ry+i][x-1+rx+j], with the
 * epilogue of fvp_conv2d_nhwc_ex.
 *   in   device [N][H][W][Cpi] fp32, Cpi % 16 == 0;  out  device [N][2H][2W][Cpo], Cpo % 32 == 0
 *   u    device [4][9][Cpi/16][4][Cpo][4] fp32: per class c = 2 ry + rx, U = G g G^T
 *        (G = [[1,0],[1,1],[0,1]]) of its 2x2 taps, element (c, xi = 3a + b, k, cm, co, c4)
 *        = U[co][ci = 16k + 4c4 + cm][a][b] (zero for padding channels)
 * Exact sums and differences around fp32 products (the weight transform is the
 * caller's, in fp64). */
int fvp_deconv4s2_wino_nhwc(const float *in, int N, int H, int W, int Cpi, const float *u, int Cpo,
                            const float *scale, const float *shift, const float *res_pre, const float *res_post,
                            int relu, float *out, void *stream);
/* The launch fvp_conv3x3_wino_nhwc makes for a shape (host only): plan[0..5] =
 * {tile rows, tile columns (Winograd 2x2 tiles per block), 32-column blocks
 * per block (1 or 2), waves sets splitting the 16 transform positions (1 or 2),
 * blocks, 1000 x (tile slots x 4 px) / (H x W)} -- the last is the MFMA work
 * over the useful work, what the AUTO rule of fvp/cnn.py reads. */
int fvp_conv3x3_wino_plan(int N, int H, int W, int Cpo, int *plan);
/* A whole 1-D conv net in one launch (csrc/fvp_c2c.hip): C2CNet
 * (cnns_1d.py:182-241) on ncols columns x [ncols][cin0][L0] fp32 -> y
 * [ncols][cout_final][Lfinal]; one block per column, every activation in LDS.
 * prog: device int32 [nops][12] = {kind (0 conv, 1 ConvTranspose1d(2, 2),
 * 2 max_pool1d(2, 2)), cin, cout, k, L (input length), src, dst, res_pre,
 * res_post (activation buffers 0 .. nbuf-1 of slot floats each; -1 none),
 * relu, w_off, cic}; params: device fp32, at w_off (% 4 == 0) W [cin][k][cout]
 * then the folded BN scale [cout] and shift [cout]; a conv's weights stream
 * through LDS in chunks of cic input channels (cic * k * cout % 4 == 0,
 * <= wchunk floats; wchunk in {4096, 8192, 12288}: two chunk buffers share the
 * LDS with the activations, so longer columns take smaller chunks).
 * out = act(scale * sum W x + shift (+ res_pre)) (+ res_post);
 * the input is buffer 0, the output buffer out_buf.  lg in {4, 8}:
 * output positions per thread item, cout * ceil(Lout / lg) <= 1024 for every
 * conv.  fvp/cnn.py Net1D builds the program. */
size_t fvp_conv1d_net_lds_bytes(int slot, int nbuf, int wchunk, int lg);
int fvp_conv1d_net(const float *x, int ncols, int cin0, int L0, const int *prog, int nops, const float *params,
                   int slot, int nbuf, int wchunk, int out_buf, int cout_final, int Lfinal, int lg, float *y,
                   void *stream);
/* 1x1 convolution of NHWC activations [N][H][W][Cpi] (16-B aligned) written NCHW:
 * out[n][co][y][x] = act(scale[co] * sum_ci in[n][y][x][ci] w[ci * ldw + co] + shift[co]),
 * Cout <= 64; 4, 8 or 16 float4s of input are read per pixel (<= Cpi), so w holds
 * that many rows (zero past Cin; the padded GEMM weights of fvp/cnn.py do).
 * P2PNet's output layer (lib/models/cnns_2d.py:185-232) without the NHWC -> NCHW pass. */
int fvp_conv1x1_nchw(const float *in, int N, int H, int W, int Cpi, int Cin, const float *w, int ldw, int Cout,
                     const float *scale, const float *shift, int relu, float *out, void *stream);
/* P2PNet's tail in one launch (lib/models/cnns_2d.py:178-180 and 209): the
 * decoder's last Upsample2DBlock plus its skip and the output 1x1 conv,
 *   y[n][2y+ry][2x+rx][co] = max(scale[co] * sum_ci in[n][y][x][ci] W[ci][co][ry][rx] + shift[co], 0)
 *                            + (co < Cs ? skip[n][2y+ry][2x+rx][co] : 0)      (co < 32)
 *   out[n][j][oy][ox] = hscale[j] * sum_co y[n][oy][ox][co] Wh[j][co] + hshift[j]  (j < J <= 16)
 * with y never written to memory.  in: NHWC [N][H][W][Cpi] (16-B aligned, Cpi % 16 == 0, <= 128,
 * W % 32 == 0); skip: NHWC [N][2H][2W][Cps] (16-B aligned, Cps % 4 == 0); wd: [Cpi/16][4][128][4] with
 * wd[s][kq][(2 ry + rx) 32 + co][c4] = W[16 s + 4 c4 + kq][co][ry][rx] (zero past Cin / Cout);
 * wh: [2][4][16][4], wh[s][kq][j][c4] = Wh[j][16 s + 4 c4 + kq]; out: NCHW [N][J][2H][2W]
 * (fvp/cnn.py FvpCNN packs both). */
int fvp_up2_head_nchw(const float *in, int N, int H, int W, int Cpi, const float *wd, const float *scale,
                      const float *shift, const float *skip, int Cps, int Cs, const float *wh, const float *hscale,
                      const float *hshift, int J, float *out, void *stream);
/* Output size of a geometry (host only): out_hw = {Ho, Wo}; FVP_ERR_SHAPE if invalid. */
int fvp_conv2d_geom(int H, int W, int Cpi, int KH, int KW, int mode, int sy, int sx, int py, int px, int *out_hw);
/* MaxPool2d(K, S, P) of NHWC activations (C % 4 == 0) with implicit -inf
 * padding, NaN-propagating (resnet.py:109: 3, 2, 1).  Ho = (H + 2P - K)/S + 1. */
int fvp_maxpool_pad_nhwc(const float *in, int N, int H, int W, int C, int K, int S, int P, float *out, void *stream);
/* The same on bf16 NHWC activations (C % 8 == 0; exact: the maximum is one
 * of the inputs) -- the bf16 backbone's max pool after its bf16 stem. */
/* PoseResNet's conv1 + BN + ReLU (resnet.py:105-107, 109: 7x7, stride 2,
 * pad 3, C <= 4 input channels -> 64) on bf16 MFMA straight from the NCHW
 * fp32 images [N][C][H][W] to bf16 NHWC [N][Ho][Wo][64], Ho = (H - 1)/2 + 1.
 * wpack: bf16 [64][7][8][4] = W[co][c][ky][kx] at (co, ky, kx, c), zero for
 * kx = 7 and c >= C; scale / shift: fp32 [64] (BN folded).  Opt-in precision
 * (bf16 operands, fp32 accumulation). */
int fvp_conv_stem7_bf16(const float *img, int N, int C, int H, int W, const void *wpack, const float *scale,
                        const float *shift, void *out, void *stream);
/* The same stem on the fp32 matrix cores (exact fp32 products, fp32 sums; the
 * default precision), C <= 3 NCHW fp32 images -> fp32 NHWC [N][Ho][Wo][64]:
 * K = the 147 (tap, channel) pairs kk = 21 ky + 3 kx + c plus one zero row.
 * wpack: fp32 [148][80] = W[co][c][ky][kx] at (kk, co), zero for co >= 64,
 * c >= C and kk = 147; scale / shift: fp32 [64] (BN folded).  wpack, scale,
 * shift and out 16-B aligned.  Replaces the NHWC conversion + the generic
 * 4-channel-pitch conv of resnet.py:105-107 (fvp/backbone.py). */
int fvp_conv_stem7_f32(const float *img, int N, int C, int H, int W, const float *wpack, const float *scale,
                       const float *shift, float *out, void *stream);
/* The CNNs' front Basic2DBlock (cnns_2d.py: 7x7, stride 1, pad 3, C <= 16
 * planes -> 16 channels) + BN + ReLU on bf16 MFMA, straight from the NCHW
 * fp32 maps [N][C][H][W] to bf16 NHWC [N][H][W][16].  wpack: bf16
 * [16][50][16] = W[co][c][ky][kx] at (co, 7*ky + kx, c), zero for tap 49 and
 * c >= C; scale / shift: fp32 [16].  Opt-in precision. */
int fvp_conv_front7_bf16(const float *x, int N, int C, int H, int W, const void *wpack, const float *scale,
                         const float *shift, void *out, void *stream);
/* The same front Basic2DBlock on the fp32 matrix cores (exact fp32 products,
 * fp32 sums), NCHW fp32 maps [N][C][H][W] -> fp32 NHWC [N][H][W][16]: wpack
 * fp32 [49][16][16] = W[co][c][ky][kx] at (7*ky + kx, co, c), zero for c >= C;
 * scale / shift: fp32 [16] (BN folded).  The default fp32 front layer of
 * fvp/cnn.py FvpCNN (P2PNet, CenterNet). */
int fvp_conv_front7_f32(const float *x, int N, int C, int H, int W, const float *wpack, const float *scale,
                        const float *shift, float *out, void *stream);
int fvp_maxpool_pad_nhwc_bf16(const void *in, int N, int H, int W, int C, int K, int S, int P, void *out,
                              void *stream);
/* 2x2 / stride-2 max pool of NHWC activations (C % 4 == 0), NaN-propagating. */
int fvp_maxpool2_nhwc(const float *in, int N, int H, int W, int C, float *out, void *stream);
/* KH x KW / stride-(KH, KW) max pool, KH, KW in {1, 2} (floor); KH = 1, KW = 2
 * is F.max_pool1d(x, 2, 2) of Pool1DBlock (cnns_1d.py:77-93) on H == 1 rows. */
int fvp_maxpool_nhwc(const float *in, int N, int H, int W, int C, int KH, int KW, float *out, void *stream);
/* The same on bf16 NHWC activations (C % 8 == 0; exact) -- the bf16 CNNs' pools. */
int fvp_maxpool_nhwc_bf16(const void *in, int N, int H, int W, int C, int KH, int KW, void *out, void *stream);

/* WeightNet.forward (lib/models/weight_net.py:48-80) fused into one launch,
 * one block per joint map:
 *   conv3x3(1 -> C, pad 1) -> BatchNorm -> MaxPool2d(2) -> ReLU ->
 *   adaptive_avg_pool2d(1) -> Linear(C, Hd) -> ReLU -> Linear(Hd, 1) -> Sigmoid
 * without materialising the [C][H][W] conv maps.
 *   features device [Nimg][H][W] (the [3P][J] joint maps; Nimg = 3*P*J)
 *   conv_w   device [C][9];  scale, shift device [C] (conv bias + BatchNorm folded)
 *   fc1_w    device [Hd][C], fc1_b [Hd];  fc2_w device [Hd], fc2_b device [1]
 *   out      device [Nimg] fusion weights in (0, 1)
 * C <= 64; (H+2)*(W+2) floats must fit 64 KB of LDS. */
int fvp_weight_net(const float *features, int Nimg, int H, int W, const float *conv_w, const float *scale,
                   const float *shift, int C, const float *fc1_w, const float *fc1_b, int Hd, const float *fc2_w,
                   const float *fc2_b, float *out, void *stream);
/* NCHW [N][C][H][W] <-> NHWC [N][H][W][Cp] (Cp >= C, padding channels zero). */
int fvp_nchw_to_nhwc(const float *in, int N, int C, int H, int W, int Cp, float *out, void *stream);
int fvp_nhwc_to_nchw(const float *in, int N, int C, int H, int W, int Cp, float *out, void *stream);

/* Roofline calibration (not on the product path): a float4 streaming copy of
 * `bytes` (multiple of 16) from src to dst; bench.py reports the op's HBM
 * rate as a fraction of this kernel's measured rate besides the nominal peak. */
int fvp_copy_f4(const void *src, void *dst, size_t bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* FVP_H */
