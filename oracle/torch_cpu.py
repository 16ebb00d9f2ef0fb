"""The reference's CPU execution of the hot path, restated with the same torch
ops in the same order (TEST INFRASTRUCTURE / BASELINE ONLY).

Used by bench.py's ``cpu_baseline`` leg (kind "port"): it is what the
reference costs on the host cores -- the per-frame F.grid_sample loop and
mean/clamp of project_whole.py:139-167, torch.max over z (cnns_2d.py:291),
nms2D (proposal.py:34-76) and the column gather (human_detection_net.py:199-200).
Validated against the reference's golden vectors in tests/test_oracle_golden.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def voxelize(heatmaps: torch.Tensor, sample_grid: torch.Tensor, vpa) -> torch.Tensor:
    """heatmaps [B,V,J,H,W], sample_grid [V,1,N,2] -> cube [B,J,X,Y,Z]."""
    B, V, J = heatmaps.shape[:3]
    N = sample_grid.shape[2]
    cubes = torch.zeros(B, J, 1, N)
    for i in range(B):
        cubes[i] = torch.mean(F.grid_sample(heatmaps[i], sample_grid, align_corners=True), dim=0).squeeze(0)
    cubes = cubes.clamp(0.0, 1.0)
    return cubes.view(B, J, vpa[0], vpa[1], vpa[2])


def nms2d(prob: torch.Tensor, K: int):
    B = prob.shape[0]
    mx = F.max_pool2d(prob, kernel_size=3, stride=1, padding=1)
    nms = ((prob == mx).float() * prob).reshape(B, -1)
    vals, flat = nms.topk(K)
    shape1 = prob[0].shape[1]
    xy = torch.stack([torch.div(flat, shape1, rounding_mode="trunc"), flat % shape1], dim=2)
    return vals, xy, flat


def hot_path(heatmaps: torch.Tensor, sample_grid: torch.Tensor, vpa, K: int, root: int = 2):
    """One frame batch through voxelise -> xy -> NMS top-K -> columns."""
    cube = voxelize(heatmaps, sample_grid, vpa)
    xy = torch.max(cube, dim=4)[0]
    vals, idx, flat = nms2d(xy[:, root:root + 1].contiguous(), K)
    B, J = cube.shape[:2]
    cols = torch.gather(torch.flatten(cube, 2, 3).permute(0, 2, 1, 3), dim=1,
                        index=flat.view(B, -1, 1, 1).repeat(1, 1, J, cube.shape[4]))
    return cube, xy, vals, flat, cols
