"""Drop-in for ``core.proposal`` (lib/core/proposal.py): ``nms2D`` and
``get_index2D`` with the reference's signatures, the two gathers of
HumanDetectionNet.forward (human_detection_net.py:191-192, :199-200), and
``ProposalLayer`` (human_detection_net.py:14-125; A14 of SURVEY.md §8(a)).

``nms2D(prob_map[B,1,X,Y], max_num) -> (topk_values[B,K], topk_index[B,K,2],
topk_flatten_index[B,K])`` runs in one HIP launch (``fvp_nms_topk``).  Ties
are ordered value-descending then flat-index-ascending (torch.topk leaves tie
order unspecified); the 2-D decode divides by ``shape[1] == X`` exactly as
get_index2D does (proposal.py:27-29,75).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import ops


def get_index2D(indices: torch.Tensor, shape) -> torch.Tensor:
    """proposal.py:13-32 (host-side integer decode, kept for API parity)."""
    batch_size, num_people = indices.shape[0], indices.shape[1]
    ix = torch.div(indices, shape[1], rounding_mode="trunc").reshape(batch_size, num_people, -1)
    iy = (indices % shape[1]).reshape(batch_size, num_people, -1)
    return torch.cat([ix, iy], dim=2)


def nms2D(prob_map: torch.Tensor, max_num: int):
    prob_map = prob_map.detach()  # human_detection_net.py:188 passes .detach(); the op is forward-only
    vals, xy, flat = ops.nms_topk(prob_map, int(max_num))
    return vals, xy, flat


def nms2D_columns(prob_map: torch.Tensor, max_num: int, feature_cubes: torch.Tensor):
    """nms2D followed by gather_columns at its winners (human_detection_net.py:188,
    :199-200) in one launch: (topk_values, topk_index, topk_flatten_index, feature_1d [B,K,J,Z])."""
    return ops.nms_topk_columns_joint(prob_map.detach(), int(max_num), feature_cubes)


def gather_columns(feature_cubes: torch.Tensor, topk_flatten_index: torch.Tensor) -> torch.Tensor:
    """feature_1d [B,K,J,Z] of human_detection_net.py:199-200."""
    return ops.gather_columns(feature_cubes, topk_flatten_index)


def gather_bbox(bbox_preds: torch.Tensor, topk_flatten_index: torch.Tensor) -> torch.Tensor:
    """match_bbox_preds [B,K,2] of human_detection_net.py:191-192 (bbox_preds [B,2,X,Y])."""
    return ops.gather_bbox(bbox_preds, topk_flatten_index)


class ProposalLayer(nn.Module):
    """Drop-in for ``models.human_detection_net.ProposalLayer`` (:14-125).

    Same constructor and attributes (``max_people``, ``min_score``, ``device``,
    ``scale``, ``bias``), same ``forward(topk_index, topk_confs,
    match_bbox_preds, meta) -> proposal_centers [B,K,7]``.  Eval / test mode
    runs on the device (``fvp_proposal_centers``: index -> mm, confidence
    threshold, bbox); in training with ground truth, the GT matching of
    ``filter_proposal`` (:38-70) -- a per-frame loop over a handful of people --
    stays in torch, with the reference's semantics, including its in-place
    update of ``match_bbox_preds``."""

    def __init__(self, cfg):
        super().__init__()
        self.max_people = cfg.CAPTURE_SPEC.MAX_PEOPLE
        self.min_score = cfg.CAPTURE_SPEC.MIN_SCORE
        self.device = torch.device(cfg.DEVICE)
        self.scale = (torch.tensor(cfg.CAPTURE_SPEC.SPACE_SIZE) /
                      (torch.tensor(cfg.CAPTURE_SPEC.VOXELS_PER_AXIS) - 1)).to(self.device)
        self.bias = (torch.tensor(cfg.CAPTURE_SPEC.SPACE_CENTER) -
                     torch.tensor(cfg.CAPTURE_SPEC.SPACE_SIZE) / 2.0).to(self.device)

    def filter_proposal(self, topk_index, bbox_preds, gt_3d, gt_bbox, num_person):
        """human_detection_net.py:38-70: nearest ground-truth root per proposal
        (-1 beyond 500 mm); predicted bbox raised to the matched GT box where
        any side falls short by more than 0.1."""
        batch_size = topk_index.shape[0]
        proposal2gt = torch.zeros(batch_size, self.max_people, device=topk_index.device)
        for i in range(batch_size):
            n = int(num_person[i])
            proposals = topk_index[i].reshape(self.max_people, 1, -1)
            gt = gt_3d[i, :n].reshape(1, n, -1)
            dist = torch.sqrt(torch.sum((proposals - gt) ** 2, dim=-1))
            min_dist, min_gt = torch.min(dist, dim=-1)
            proposal2gt[i] = min_gt
            proposal2gt[i][min_dist > 500.0] = -1.0
            for k in range(self.max_people):
                if proposal2gt[i, k] < 0:
                    continue
                g = gt_bbox[i, proposal2gt[i, k].long()]
                if torch.sum(bbox_preds[i, k] < g - 0.1):
                    bbox_preds[i, k] = g
        return proposal2gt

    def forward(self, topk_index, topk_confs, match_bbox_preds, meta):
        if self.training and ("roots_3d" in meta and "num_person" in meta):
            device = topk_index.device
            B = topk_index.shape[0]
            idx = topk_index.float() * self.scale.to(device) + self.bias.to(device)
            centers = torch.zeros(B, self.max_people, 7, device=device)
            centers[:, :, 0:3] = idx
            centers[:, :, 4] = topk_confs
            centers[:, :, 3] = self.filter_proposal(idx, match_bbox_preds, meta["roots_3d"].float().to(device),
                                                    meta["bbox"].float().to(device), meta["num_person"])
            centers[:, :, 5:7] = match_bbox_preds
            return centers
        return proposal_centers(self, topk_index, None, topk_confs, match_bbox_preds)


def _consts(layer):
    """(scale, bias, min_score) of a ProposalLayer as fp32 host values, read once
    per layer (no device sync per call)."""
    c = getattr(layer, "_fvp_consts", None)
    if c is None:
        f = lambda t: [float(np.float32(v)) for v in torch.as_tensor(t).detach().to("cpu", torch.float32).tolist()]
        c = (f(layer.scale), f(layer.bias), float(np.float32(layer.min_score)))
        layer._fvp_consts = c
    return c


def proposal_centers(layer, index, hm1d, confs, match_bbox):
    """ProposalLayer.forward in test mode (:99-124) as ONE device launch with
    ``layer``'s scale, bias and min_score (the reference's ProposalLayer or this
    one).  hm1d [B,K,Z] given: the z pick of HumanDetectionNet.forward
    (:208-215) is fused in and ``index`` is the 2-D [B,K,2] nms2D index."""
    scale, bias, min_score = _consts(layer)
    return ops.proposal_centers(index, hm1d, confs, match_bbox, scale, bias, min_score)
