"""Drop-in for ``models.project_whole.ProjectLayer`` (lib/models/project_whole.py).

Same constructor ``ProjectLayer(cfg)``, same ``forward(heatmaps, meta,
cameras, resize_transform) -> cube[B,J,X,Y,Z]``, same public attributes
(``grid``, ``sample_grid`` cache keyed by sequence, the cfg copies), same two
assertions (project_whole.py:147-148).  The arithmetic runs in two HIP
kernels (faster-voxelpose_amd/csrc): ``fvp_project_grid`` builds a sequence's
sample grid once (project_whole.py:151-156), ``fvp_voxelize`` samples, averages
over cameras, clamps and (optionally) emits the xy max-plane in the same pass
for every frame of the batch in one launch -- no Python loop over frames.

Registers no parameters or buffers, so checkpoints load unchanged.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn

from . import geometry, ops
from .heatmaps import channels_last_of

# Above this size a packed grid streams from HBM once per frame (MI355X: 4 MB
# L2 per XCD, 256 MB Infinity Cache) and the coordinates are projected on the
# fly instead (fvp_voxelize_cams).  Measured on the C5 geometry with the first
# V ring cameras (tools/c5_views.py, 8 frames): V=16 (210 MB grid) 1.63 ms
# cached vs 2.07 on the fly, V=24 (314 MB) 2.77 vs ~3.0, V=31 (406 MB) 3.76 vs
# 3.84 (B=32: 2,124 vs 2,106 frames/s) -- a tie, so the 406 MB grid is not kept.
ON_THE_FLY_GRID_BYTES = 384 << 20


def _as_list3(v, kind=float):
    if isinstance(v, (int, float)):
        return [kind(v)] * 3
    return [kind(x) for x in v]


# default of ProjectLayer.columns_on_the_fly (FVP_COLUMNS_ON_THE_FLY=1)
_COLUMNS_ON_THE_FLY_ENV = os.environ.get("FVP_COLUMNS_ON_THE_FLY", "0") != "0"


class ProjectLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.device = torch.device(cfg.DEVICE)
        self.image_size = cfg.DATASET.IMAGE_SIZE
        self.heatmap_size = cfg.DATASET.HEATMAP_SIZE
        self.ori_image_size = cfg.DATASET.ORI_IMAGE_SIZE
        self.space_size = cfg.CAPTURE_SPEC.SPACE_SIZE
        self.space_center = cfg.CAPTURE_SPEC.SPACE_CENTER
        self.voxels_per_axis = cfg.CAPTURE_SPEC.VOXELS_PER_AXIS
        self._grid = None
        self.sample_grid = {}  # seq -> [V, 1, N, 2] fp32 (the reference's cache layout; a view of _packed)
        self._packed = {}      # seq -> [N, GV, 2] voxel-major copy read by the voxelize kernel
        self._packed_of = {}   # seq -> (sample_grid entry, its packed grid, entry is a view of it, entry._version)
        self._cams = {}        # seq -> [V, FVP_CAM_STRIDE] camera records (on-the-fly projection)
        self._stacked = (None, None)  # (key, [S,N,GV,2]) grids of the last mixed-sequence batch
        self.on_the_fly = None  # None: decide by grid size; True/False: force
        # columns(): project the winners' voxels from the camera records even when
        # a packed grid is cached (bit-identical; measured slower at C3 B=8, 15.1
        # vs 11.6 us: the projection's VALU and 21-float records outweigh the
        # round trip it saves)
        self.columns_on_the_fly = _COLUMNS_ON_THE_FLY_ENV
        self.verbose = True

    # -- reference attribute: voxel centres [N,3] (compute_grid, :43-79) -------------
    @property
    def grid(self) -> torch.Tensor:
        if self._grid is None:
            S = _as_list3(self.space_size)
            C = _as_list3(self.space_center)
            nb = _as_list3(self.voxels_per_axis, int)
            axes = [torch.linspace(-S[a] / 2, S[a] / 2, nb[a]) + C[a] for a in range(3)]
            gx, gy, gz = torch.meshgrid(*axes, indexing="ij")
            self._grid = torch.stack([gx.reshape(-1), gy.reshape(-1), gz.reshape(-1)], dim=1).to(self.device)
        return self._grid

    def grid_spec(self):
        S = _as_list3(self.space_size)
        C = _as_list3(self.space_center)
        nb = _as_list3(self.voxels_per_axis, int)
        start = [float(np.float32(-s / 2)) for s in S]
        end = [float(np.float32(s / 2)) for s in S]
        return start, end, [float(np.float32(c)) for c in C], nb

    def build_sample_grid(self, cameras, seq, resize_transform, device) -> torch.Tensor:
        """project_grid x V for one sequence (project_whole.py:81-117,151-156) on device.

        Returns the reference's [V,1,N,2] layout as a view of the voxel-major
        packed grid (fvp_pack_grid) that the voxelize kernel reads."""
        cams = torch.from_numpy(geometry.pack_cameras(cameras, seq)).to(device)
        start, end, center, nb = self.grid_spec()
        w, h = self.heatmap_size
        sg = ops.project_grid(cams, resize_transform.to(device=device, dtype=torch.float32), start, end, center, nb,
                              float(max(self.ori_image_size[0], self.ori_image_size[1])),
                              float(self.image_size[0]), float(self.image_size[1]), int(w), int(h))
        packed = ops.pack_grid(sg)
        self._packed[seq] = packed
        return ops.packed_as_reference(packed, sg.shape[0])

    def _packed_grid(self, seq) -> torch.Tensor:
        sg = self.sample_grid[seq]
        hit = self._packed_of.get(seq)
        # the same tensor object, and either a view of the packed grid itself (in-place
        # writes land in the packed grid) or unchanged since it was packed (_version)
        if hit is not None and hit[0] is sg and (hit[2] or hit[3] == sg._version):
            return hit[1]
        pg = self._packed.get(seq)
        own = pg is not None and ops.packed_as_reference(pg, sg.shape[0]).data_ptr() == sg.data_ptr()
        if not own:
            # a grid assigned from outside (e.g. a reference-layout tensor): pack it, and
            # again whenever it is modified in place
            pg = ops.pack_grid(sg[:, 0].to(torch.float32).contiguous())
            self._packed[seq] = pg
        self._packed_of[seq] = (sg, pg, own, sg._version)
        return pg

    def _grids_for_batch(self, heatmaps, meta, cameras, resize_transform):
        device = heatmaps.device
        n = heatmaps.shape[1]
        seqs = list(meta["seq"])[: heatmaps.shape[0]]
        uniq = list(dict.fromkeys(seqs))
        # project_whole.py:147-156 per frame; the checks and the cache depend on
        # the sequence alone, so each distinct sequence is checked once, in order
        for curr_seq in uniq:
            assert curr_seq in cameras.keys(), "missing camera parameters for the current sequence"
            assert len(cameras[curr_seq]) == n, "inconsistent number of cameras"
            if curr_seq not in self.sample_grid:
                if self.verbose:
                    print("=> save the sampling grid in HDN for sequence", curr_seq)
                self.sample_grid[curr_seq] = self.build_sample_grid(cameras, curr_seq, resize_transform, device)
        if len(uniq) == 1:
            return self._packed_grid(uniq[0]), None
        index = torch.tensor([uniq.index(s) for s in seqs], dtype=torch.int32).to(device, non_blocking=True)
        return self._stacked_grids(uniq), index

    def _stacked_grids(self, uniq, n0: int = 0, n1: int | None = None) -> torch.Tensor:
        """[S, n1-n0, GV, 2]: the packed grids of the sequences `uniq` (voxels
        n0..n1) in one tensor for the kernel, kept across calls while the same
        sequences come back (a stack is a full copy of every grid)."""
        grids = [self._packed_grid(s) for s in uniq]
        n1 = grids[0].shape[0] if n1 is None else n1
        key = (tuple(uniq), tuple(g.data_ptr() for g in grids), n0, n1)
        if self._stacked[0] != key:
            self._stacked = (None, None)  # release the previous stack first
            self._stacked = (key, torch.stack([g[n0:n1] for g in grids]))
        return self._stacked[1]

    def _project_on_the_fly(self, V) -> bool:
        if self.on_the_fly is not None:
            return bool(self.on_the_fly)
        X, Y, Z = _as_list3(self.voxels_per_axis, int)
        return X * Y * Z * ops.grid_slots(V) * 8 > ON_THE_FLY_GRID_BYTES

    def _cams_for_batch(self, heatmaps, meta, cameras):
        device = heatmaps.device
        n = heatmaps.shape[1]
        seqs = list(meta["seq"])[: heatmaps.shape[0]]
        uniq = list(dict.fromkeys(seqs))
        for curr_seq in uniq:
            assert curr_seq in cameras.keys(), "missing camera parameters for the current sequence"
            assert len(cameras[curr_seq]) == n, "inconsistent number of cameras"
            if curr_seq not in self._cams:
                self._cams[curr_seq] = torch.from_numpy(geometry.pack_cameras(cameras, curr_seq)).to(device)
        if len(uniq) == 1:
            return self._cams[uniq[0]], None
        index = torch.tensor([uniq.index(s) for s in seqs], dtype=torch.int32).to(device, non_blocking=True)
        return torch.stack([self._cams[s] for s in uniq]), index

    def prepare(self, heatmaps, meta, cameras, resize_transform):
        """Build the per-sequence caches forward_fused will use (grid or camera records)."""
        if self._project_on_the_fly(heatmaps.shape[1]):
            self._cams_for_batch(heatmaps, meta, cameras)
        else:
            self._grids_for_batch(heatmaps, meta, cameras, resize_transform)

    def forward_fused(self, heatmaps, meta, cameras, resize_transform, want_cube=True, want_xy=True):
        """One launch for the whole batch: (cube[B,J,X,Y,Z] or empty, xy[B,J,X,Y] or empty).

        heatmaps: [B,V,J,H,W] tensor, or fvp.heatmaps.ChannelsLastHeatmaps (or a
        tensor carrying one, fvp.heatmaps.attach) -- then the gather reads the
        channels-last copy in place (fvp_voxelize_cl), bit-identical results."""
        ops.forward_only(heatmaps)
        X, Y, Z = _as_list3(self.voxels_per_axis, int)
        if heatmaps.shape[0] == 0:  # empty batch: the reference's frame loop yields empty outputs
            return self._empty(heatmaps, X, want_cube, want_xy)
        cl = channels_last_of(heatmaps)
        if self._project_on_the_fly(heatmaps.shape[1]):
            cams, index = self._cams_for_batch(heatmaps, meta, cameras)
            start, end, center, nb = self.grid_spec()
            rt = resize_transform.to(device=heatmaps.device, dtype=torch.float32)
            geo = (start, end, center, nb, float(max(self.ori_image_size[0], self.ori_image_size[1])),
                   float(self.image_size[0]), float(self.image_size[1]), want_cube, want_xy)
            if cl is not None:
                return ops.voxelize_cl_cams(cl.t, cl.J, cams, index, rt, *geo)
            return ops.voxelize_cams(heatmaps, cams, index, rt, *geo)
        grids, index = self._grids_for_batch(heatmaps, meta, cameras, resize_transform)
        if cl is not None:
            return ops.voxelize_cl(cl.t, cl.J, grids, index, X, Y, Z, want_cube, want_xy)
        return ops.voxelize(heatmaps, grids, index, X, Y, Z, want_cube, want_xy)

    def columns(self, heatmaps, meta, cameras, resize_transform, flat):
        """columns[b,k,j,:] = forward_fused(...)[0][b,j,flat[b,k],:] -- the z-columns
        at the proposals (human_detection_net.py:199-200) recomputed for the K
        winners only, bit-identical, so the cube need not be written."""
        ops.forward_only(heatmaps)
        X, Y, Z = _as_list3(self.voxels_per_axis, int)
        cl = channels_last_of(heatmaps)
        src, J = (cl.t, cl.J) if cl is not None else (heatmaps, 0)
        if self._project_on_the_fly(heatmaps.shape[1]) or self.columns_on_the_fly:
            # the coordinates projected from the camera records (bit-identical to the
            # packed grid; their loads do not wait for `flat`)
            cams, index = self._cams_for_batch(heatmaps, meta, cameras)
            start, end, center, nb = self.grid_spec()
            rt = resize_transform.to(device=heatmaps.device, dtype=torch.float32)
            return ops.voxel_columns(src, J, None, cams, index, rt, start, end, center, nb,
                                     float(max(self.ori_image_size[0], self.ori_image_size[1])),
                                     float(self.image_size[0]), float(self.image_size[1]), flat)
        grids, index = self._grids_for_batch(heatmaps, meta, cameras, resize_transform)
        return ops.voxel_columns(src, J, grids, None, index, None, [0.0] * 3, [0.0] * 3, [0.0] * 3, [X, Y, Z],
                                 0.0, 0.0, 0.0, flat)

    def _empty(self, heatmaps, X, want_cube, want_xy):
        _, Y, Z = _as_list3(self.voxels_per_axis, int)
        J = heatmaps.shape[2]
        f = dict(dtype=torch.float32, device=heatmaps.device)  # (a tensor or ChannelsLastHeatmaps)
        return (torch.zeros((0, J, X, Y, Z) if want_cube else (0,), **f),
                torch.zeros((0, J, X, Y) if want_xy else (0,), **f))

    def forward_slab(self, heatmaps, meta, cameras, resize_transform, x_begin: int, x_end: int,
                     want_cube=True, want_xy=True):
        """Voxels with x in [x_begin, x_end) only: (cube[B,J,x_end-x_begin,Y,Z], xy[B,J,x_end-x_begin,Y]).

        The large-frame mode of SURVEY.md §8(e): each rank of a group owns an
        x-slab of every frame (fvp.parallel.shard_slab); every voxel and every
        (x, y) column lies wholly in one slab, so the slabs are bit-identical
        to the same rows of forward_fused.  The coordinates come from where
        forward_fused would take them: for a grid that would not stay cached
        (C5: 406 MB per sequence) they are projected on the fly from the
        camera records for the slab's rows only (fvp_voxelize_cams_slab), so
        no rank builds or reads a sample grid; otherwise the packed grid is
        voxel-major with x slowest, a slab is a contiguous slice of it, and
        the kernel runs unchanged on the slab's rows."""
        ops.forward_only(heatmaps)
        X, Y, Z = _as_list3(self.voxels_per_axis, int)
        if not 0 <= x_begin < x_end <= X:
            raise ValueError(f"x-slab [{x_begin}, {x_end}) outside [0, {X})")
        if heatmaps.shape[0] == 0:
            return self._empty(heatmaps, x_end - x_begin, want_cube, want_xy)
        cl = channels_last_of(heatmaps)
        if self._project_on_the_fly(heatmaps.shape[1]):
            cams, index = self._cams_for_batch(heatmaps, meta, cameras)
            start, end, center, nb = self.grid_spec()
            rt = resize_transform.to(device=heatmaps.device, dtype=torch.float32)
            geo = (start, end, center, nb, float(max(self.ori_image_size[0], self.ori_image_size[1])),
                   float(self.image_size[0]), float(self.image_size[1]), want_cube, want_xy, x_begin, x_end)
            if cl is not None:
                return ops.voxelize_cl_cams(cl.t, cl.J, cams, index, rt, *geo)
            return ops.voxelize_cams(heatmaps, cams, index, rt, *geo)
        grids, index = self._grids_for_batch(heatmaps, meta, cameras, resize_transform)
        n0, n1 = x_begin * Y * Z, x_end * Y * Z
        if grids.dim() == 3:
            slab = grids[n0:n1]
        else:  # mixed sequences: the stacked slab rows (kept across calls)
            slab = self._stacked_grids(list(dict.fromkeys(list(meta["seq"])[: heatmaps.shape[0]])), n0, n1)
        if cl is not None:
            return ops.voxelize_cl(cl.t, cl.J, slab, index, x_end - x_begin, Y, Z, want_cube, want_xy)
        return ops.voxelize(heatmaps, slab, index, x_end - x_begin, Y, Z, want_cube, want_xy)

    def forward(self, heatmaps, meta, cameras, resize_transform):
        cube, _ = self.forward_fused(heatmaps, meta, cameras, resize_transform, want_cube=True, want_xy=False)
        return cube
