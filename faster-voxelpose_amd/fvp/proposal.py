"""Drop-in for ``core.proposal`` (lib/core/proposal.py): ``nms2D`` and
``get_index2D`` with the reference's signatures, plus the two gathers of
HumanDetectionNet.forward (human_detection_net.py:191-192, :199-200).

``nms2D(prob_map[B,1,X,Y], max_num) -> (topk_values[B,K], topk_index[B,K,2],
topk_flatten_index[B,K])`` runs in one HIP launch (``fvp_nms_topk``).  Ties
are ordered value-descending then flat-index-ascending (torch.topk leaves tie
order unspecified); the 2-D decode divides by ``shape[1] == X`` exactly as
get_index2D does (proposal.py:27-29,75).
"""
from __future__ import annotations

import torch

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


def gather_columns(feature_cubes: torch.Tensor, topk_flatten_index: torch.Tensor) -> torch.Tensor:
    """feature_1d [B,K,J,Z] of human_detection_net.py:199-200."""
    return ops.gather_columns(feature_cubes, topk_flatten_index)


def gather_bbox(bbox_preds: torch.Tensor, topk_flatten_index: torch.Tensor) -> torch.Tensor:
    """match_bbox_preds [B,K,2] of human_detection_net.py:191-192 (bbox_preds [B,2,X,Y])."""
    return ops.gather_bbox(bbox_preds, topk_flatten_index)
