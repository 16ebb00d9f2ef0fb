"""Drop-in for ``models.project_individual.ProjectLayer``
(lib/models/project_individual.py).

Same constructor and ``forward(heatmaps, index, meta, proposal_centers,
cameras, resize_transform) -> (cubes[P,J,64,64,64], offset[P,3])``, same public
attributes (``center_grid`` is read by JointLocalizationNet's soft-argmax,
joint_localization_net.py:165; ``fine_voxels_per_axis``, ``scale``, ``bias``,
``fine_grid``, ``sample_grid``).  The per-sequence fine sample grid is built
by ``fvp_project_grid`` over the fine whole-space grid; all proposals of the
frame are voxelised by ONE ``fvp_person_planes`` launch that evaluates each
proposal's window on the device (no per-proposal loop, no host syncs --
project_individual.py:272-275 read ``torch.sum(start >= end)`` back per
proposal).  ``forward_planes`` returns the xy/xz/yz max-projections
JointLocalizationNet concatenates (joint_localization_net.py:158-160) without
materialising the 64^3 cubes; ``forward_batch`` does that for every valid
proposal of a batch of frames in one launch.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import geometry, ops
from .heatmaps import ChannelsLastHeatmaps, channels_last_of


# Fine-grid sampling coordinates: read from the per-sequence packed fine grid
# (197 MB for 5 cameras; measured faster: C3, 320 proposals, 10.7 vs 11.7 us
# each) unless that grid would exceed this size (e.g. 31 cameras: 1 GB), then
# projected on the fly (fvp_person_planes_cams).  layer.on_the_fly forces.
PERSON_OTF_GRID_BYTES = 512 << 20


class ProjectLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.device = torch.device(cfg.DEVICE)
        self.image_size = cfg.DATASET.IMAGE_SIZE
        self.heatmap_size = cfg.DATASET.HEATMAP_SIZE
        self.ori_image_size = cfg.DATASET.ORI_IMAGE_SIZE
        c = geometry.individual_constants(cfg.CAPTURE_SPEC.SPACE_SIZE, cfg.CAPTURE_SPEC.SPACE_CENTER,
                                          cfg.INDIVIDUAL_SPEC.SPACE_SIZE, cfg.INDIVIDUAL_SPEC.VOXELS_PER_AXIS)
        self._const = c
        dev = self.device
        self.whole_space_center = torch.from_numpy(c["whole_center"]).to(dev)
        self.whole_space_size = torch.from_numpy(c["whole_size"]).to(dev)
        self.ind_space_size = torch.from_numpy(c["ind_size"]).to(dev)
        self.voxels_per_axis = torch.from_numpy(c["ind_bins"]).to(dev)
        self.fine_voxels_per_axis = torch.from_numpy(c["fine"]).to(dev)
        self.scale = torch.from_numpy(c["scale"]).to(dev)
        self.bias = torch.from_numpy(c["bias"]).to(dev)
        self.center_grid = self._center_grid().to(dev)  # project_individual.py:101-107
        self._fine_grid = None
        self.sample_grid = {}  # seq -> [V, FX, FY, FZ, 2] (the reference's cache; a view of _packed)
        self._packed = {}      # seq -> [FX*FY*FZ, GV, 2] voxel-major copy read by the person kernel
        self._cams = {}        # seq -> [V, FVP_CAM_STRIDE] camera records (on-the-fly projection)
        self.on_the_fly = None  # None: by fine-grid size (PERSON_OTF_GRID_BYTES); True/False: force
        self.verbose = True

    @staticmethod
    def _axis(size, centre, n):
        s = float(size)
        return torch.linspace(float(np.float32(-s / 2)), float(np.float32(s / 2)), int(n)) + float(centre)

    def _grid3(self, size, centre, bins):
        axes = [self._axis(size[a], centre[a], bins[a]) for a in range(3)]
        gx, gy, gz = torch.meshgrid(*axes, indexing="ij")
        return torch.stack([gx.reshape(-1), gy.reshape(-1), gz.reshape(-1)], dim=1)

    def _center_grid(self):
        c = self._const
        b = [int(v) for v in c["ind_bins"]]
        g = self._grid3(c["ind_size"], c["whole_center"], b).view(b[0], b[1], b[2], 3)
        return torch.stack([g[:, :, 0, :2].reshape(-1, 2), g[:, 0, :, ::2].reshape(-1, 2),
                            g[0, :, :, 1:].reshape(-1, 2)])

    @property
    def fine_grid(self) -> torch.Tensor:
        """Fine whole-space voxel centres [FX*FY*FZ, 3] (project_individual.py:110).
        Built lazily: the kernels rebuild centres on the fly and never read it."""
        if self._fine_grid is None:
            c = self._const
            self._fine_grid = self._grid3(c["whole_size"], c["whole_center"], c["fine"]).to(self.device)
        return self._fine_grid

    def build_sample_grid(self, cameras, seq, resize_transform, device) -> torch.Tensor:
        """compute_sample_grid (project_individual.py:192-220) on device -> [V,FX,FY,FZ,2]."""
        c = self._const
        cams = torch.from_numpy(geometry.pack_cameras(cameras, seq)).to(device)
        start = [float(np.float32(-float(s) / 2)) for s in c["whole_size"]]
        end = [float(np.float32(float(s) / 2)) for s in c["whole_size"]]
        fine = [int(v) for v in c["fine"]]
        w, h = self.heatmap_size
        sg = ops.project_grid(cams, resize_transform.to(device=device, dtype=torch.float32), start, end,
                              [float(v) for v in c["whole_center"]], fine,
                              float(max(self.ori_image_size[0], self.ori_image_size[1])),
                              float(self.image_size[0]), float(self.image_size[1]), int(w), int(h))
        packed = ops.pack_grid(sg)  # voxel-major [FN, GV, 2], read by the person kernel
        self._packed[seq] = packed
        return ops.packed_as_reference(packed, sg.shape[0])[:, 0].view(sg.shape[0], fine[0], fine[1], fine[2], 2)

    def _seq_grid(self, heatmaps, index, meta, cameras, resize_transform):
        """Packed fine grid of frame ``index``'s sequence (built once per sequence)."""
        curr_seq = meta["seq"][index]
        if curr_seq not in self.sample_grid:
            if self.verbose:
                print("=> save the sampling grid in JLN for sequence", curr_seq)
            self.sample_grid[curr_seq] = self.build_sample_grid(cameras, curr_seq, resize_transform, heatmaps.device)
        sg = self.sample_grid[curr_seq]
        pg = self._packed.get(curr_seq)
        if pg is None or pg.data_ptr() != sg.data_ptr():
            # a grid assigned from outside (the reference's [V,FX,FY,FZ,2] layout): pack it once
            pg = ops.pack_grid(sg.reshape(sg.shape[0], -1, 2).to(torch.float32).contiguous())
            self._packed[curr_seq] = pg
        return pg

    def _otf(self, V: int) -> bool:
        if self.on_the_fly is not None:
            return bool(self.on_the_fly)
        fine = [int(v) for v in self._const["fine"]]
        return fine[0] * fine[1] * fine[2] * ops.grid_slots(V) * 8 > PERSON_OTF_GRID_BYTES

    def _run(self, heatmaps, index, meta, cameras, resize_transform, props, frame_of, cubes, planes):
        """One fvp_person_planes[_cams|_cl] launch for ``props`` of the frames of ``heatmaps``
        (the coordinates of ``meta['seq'][index]``'s cameras).  heatmaps: a tensor
        or fvp.heatmaps.ChannelsLastHeatmaps (read in place on the cached-grid path)."""
        cl = channels_last_of(heatmaps)
        if self._otf(heatmaps.shape[1]):
            if isinstance(heatmaps, ChannelsLastHeatmaps):
                heatmaps = heatmaps.planar()
            seq = meta["seq"][index]
            if seq not in self._cams:
                self._cams[seq] = torch.from_numpy(geometry.pack_cameras(cameras, seq)).to(heatmaps.device)
            c = self._const
            start = [float(np.float32(-float(v) / 2)) for v in c["whole_size"]]
            end = [float(np.float32(float(v) / 2)) for v in c["whole_size"]]
            return ops.person_planes_cams(heatmaps, self._cams[seq],
                                          resize_transform.to(device=heatmaps.device, dtype=torch.float32),
                                          start, end, [float(v) for v in c["whole_center"]],
                                          float(max(self.ori_image_size[0], self.ori_image_size[1])),
                                          float(self.image_size[0]), float(self.image_size[1]), props, frame_of,
                                          *self._args(), cubes, planes)
        grid = self._seq_grid(heatmaps, index, meta, cameras, resize_transform)
        if cl is not None:
            return ops.person_planes_cl(cl.t, cl.J, grid, props, frame_of, *self._args(), cubes, planes)
        return ops.person_planes(heatmaps, grid, props, frame_of, *self._args(), cubes, planes)

    @staticmethod
    def _frame(heatmaps, index):
        """Frame ``index`` of the batch (keeping a channels-last copy, if any)."""
        cl = channels_last_of(heatmaps)
        if cl is not None:
            return ChannelsLastHeatmaps(cl.t[index:index + 1], cl.J)
        return heatmaps[index:index + 1]

    def _args(self):
        c = self._const
        return ([int(v) for v in c["fine"]], [float(v) for v in c["scale"]], [float(v) for v in c["bias"]],
                [float(v) for v in c["whole_size"]], [float(v) for v in c["ind_size"]],
                [int(v) for v in c["ind_bins"]])

    def forward(self, heatmaps, index, meta, proposal_centers, cameras, resize_transform):
        ops.forward_only(heatmaps, proposal_centers)
        cubes, _, offset = self._run(self._frame(heatmaps, index), index, meta, cameras, resize_transform,
                                     proposal_centers, None, True, False)
        return cubes, offset

    def forward_planes(self, heatmaps, index, meta, proposal_centers, cameras, resize_transform):
        """(planes[3P,J,S,S], offset[P,3]) without materialising the cubes: the JLN
        input at joint_localization_net.py:158-160 for frame ``index``."""
        ops.forward_only(heatmaps, proposal_centers)
        _, planes, offset = self._run(self._frame(heatmaps, index), index, meta, cameras, resize_transform,
                                      proposal_centers, None, False, True)
        return planes, offset

    def forward_batch(self, heatmaps, meta, proposal_centers, mask, cameras, resize_transform, idx=None, sel=None):
        """Every valid proposal of the batch in one launch per sequence (the
        reference loops frames and proposals with host syncs,
        joint_localization_net.py:148-151, project_individual.py:272-275).
        proposal_centers [B,K,7], mask [B,K] bool.  Returns (planes [3P,J,S,S]
        in (frame, proposal) order of ``mask``, offset [P,3], frame_of [P]).
        idx: ``mask.nonzero()`` if the caller already has it (its one host sync); sel: the
        (idx, frame_of int32, proposal_centers[mask]) triple of ops.mask_select instead."""
        ops.forward_only(heatmaps, proposal_centers)
        seqs = list(meta["seq"])[: heatmaps.shape[0]]
        if sel is not None:
            idx, frame_of, props = sel
        else:
            if idx is None:
                idx = mask.nonzero()  # one host sync for the whole batch
            frame_of = idx[:, 0].to(torch.int32)
            props = proposal_centers[idx[:, 0], idx[:, 1]]
        uniq = list(dict.fromkeys(seqs))
        if len(uniq) == 1:
            _, planes, offset = self._run(heatmaps, 0, meta, cameras, resize_transform, props, frame_of, False, True)
            return planes, offset, frame_of
        # frames of several sequences: one launch per sequence over its proposals,
        # scattered back into the (frame, proposal) order
        P = props.shape[0]
        J = heatmaps.shape[2]
        S = [int(v) for v in self._const["ind_bins"]]
        planes = torch.zeros((3 * P, J, S[0], S[1]), dtype=torch.float32, device=heatmaps.device)
        offset = torch.zeros((P, 3), dtype=torch.float32, device=heatmaps.device)
        seq_of = torch.tensor([uniq.index(s) for s in seqs], dtype=torch.int64, device=heatmaps.device)
        owner = seq_of[idx[:, 0]] if P else seq_of[:0]
        for u, seq in enumerate(uniq):
            sel = (owner == u).nonzero()[:, 0]
            if sel.numel() == 0:
                continue
            first = seqs.index(seq)  # any frame of the sequence names its cameras
            _, pl, off = self._run(heatmaps, first, meta, cameras, resize_transform, props[sel],
                                   frame_of[sel], False, True)
            n = sel.numel()
            for k in range(3):  # xy, xz, yz blocks of the reference's cat order
                planes[k * P + sel] = pl[k * n:(k + 1) * n]
            offset[sel] = off
        return planes, offset, frame_of
