"""JLN post-processing on the fvp kernels.

* :class:`SoftArgmaxLayer` -- drop-in for
  ``models.joint_localization_net.SoftArgmaxLayer`` (joint_localization_net.py:15-56):
  same constructor (``cfg.NETWORK.BETA``), same ``forward(x, grids) -> (x, confs)``.
* :func:`fuse_pose_preds` -- ``JointLocalizationNet.fuse_pose_preds`` (:83-120).
* :func:`fused_jln_forward` -- ``JointLocalizationNet.forward`` (:122-182) for
  every proposal of a batch at once: one per-person planes launch
  (``project_layer.forward_batch``), the P2PNet / WeightNet CNNs on all
  proposals together, the soft-argmax + offsets and the fusion as two fvp
  launches; no per-frame loop and no per-frame host sync.  Eval mode only:
  in training the CNNs' BatchNorm statistics are per frame in the reference,
  so the original per-frame forward is kept.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from .heatmaps import release_shared


class SoftArgmaxLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.beta = cfg.NETWORK.BETA

    def forward(self, x, grids):
        """x [3,B,C,H*W,1] or [3,B,C,H,W] -> (coords [3,B,C,2], confs [B])."""
        ops.forward_only(x)
        pose, maxprob = ops.soft_argmax(x, grids, None, float(self.beta))
        C = x.shape[2]
        confs = maxprob.sum(dim=(0, 2)) / (3 * C)
        return pose, confs


def fuse_pose_preds(pose_preds, weights):
    """pose_preds [3,P,J,2], weights [3P,J,1] -> fused [P,J,3] (joint_localization_net.py:83-120)."""
    P, J = pose_preds.shape[1], pose_preds.shape[2]
    fused, _ = ops.fuse_poses(pose_preds, weights, pose_preds.new_zeros((3, P, J)))
    return fused


def fused_jln_forward(self, meta, heatmaps, proposal_centers, mask, cameras, resize_transform):
    """JointLocalizationNet.forward (joint_localization_net.py:122-182), batched.

    Same inputs and outputs: (all_fused_pose_preds [B,K,J,3],
    all_pose_preds [3,B,K,J,2]); proposal_centers[..., 4] of valid proposals is
    overwritten with the confidences, as in the reference (:180)."""
    if self.training:
        out = self._fvp_original_forward(meta, heatmaps, proposal_centers, mask, cameras, resize_transform)
        release_shared(heatmaps)
        return out
    device = heatmaps.device
    B, K = proposal_centers.shape[:2]
    J = heatmaps.shape[2]
    all_fused = torch.zeros((B, K, J, 3), device=device)
    all_pose = torch.zeros((3, B, K, J, 2), device=device)
    seqs = list(meta["seq"])[:B]
    if len(set(seqs)) != 1:  # frames of several sequences: one batched call per sequence
        for s in dict.fromkeys(seqs):
            sel = torch.tensor([q == s for q in seqs], device=device)
            _jln_batch(self, meta, heatmaps, proposal_centers, mask & sel[:, None], cameras, resize_transform,
                       all_fused, all_pose, first=seqs.index(s))
    else:
        _jln_batch(self, meta, heatmaps, proposal_centers, mask, cameras, resize_transform, all_fused, all_pose,
                   first=0)
    # the HDN's one-forward channels-last copy (fvp.heatmaps.share_channels_last) ends here,
    # with its last consumer: it is not kept alive on the caller's tensor
    release_shared(heatmaps)
    return all_fused, all_pose


def _jln_batch(self, meta, heatmaps, proposal_centers, mask, cameras, resize_transform, all_fused, all_pose, first):
    from . import cnn, integration

    sub_meta = dict(meta)
    sub_meta["seq"] = [meta["seq"][first]] * heatmaps.shape[0]
    # the CNN wrappers' staleness checks (host work) before the sync below, while the
    # GPU still runs the HDN: after it the GPU waits for every host step
    opts = integration.options_of(self)
    use = opts.cnn and not self.conv_net.training
    conv = cnn.cached(self.conv_net, opts.cnn_dtype) if use else self.conv_net
    wnet = cnn.cached(self.weight_net) if use and not self.weight_net.training else self.weight_net
    # mask.nonzero(), its frames and the selected proposal rows in one launch: the batch's one host
    # sync (only views after it); the scatters below index with idx
    sel = None
    if (mask.is_cuda and mask.dim() == 2 and mask.dtype == torch.bool and proposal_centers.dtype == torch.float32
            and proposal_centers.dim() == 3 and proposal_centers.stride(2) == 1):
        sel = ops.mask_select(mask, proposal_centers)
        idx = sel[0]
    else:
        idx = mask.nonzero()
    planes, offset, _ = self.project_layer.forward_batch(heatmaps, sub_meta, proposal_centers, mask, cameras,
                                                         resize_transform, idx=idx, sel=sel)
    P = planes.shape[0] // 3
    if P == 0:
        return
    out = conv(planes)                                                              # [3P,J,S,S]
    # torch.stack(torch.chunk(out, 3)) of joint_localization_net.py: a view for a contiguous
    # [3P, ...] tensor (chunk k, row p = row k*P + p), no copy
    features = out.reshape((3, P) + tuple(out.shape[1:]))                           # [3,P,J,S,S]
    pose, maxprob = ops.soft_argmax(features, self.project_layer.center_grid, offset,
                                    float(self.soft_argmax_layer.beta))
    weights = wnet(features)                                                        # [3P,J,1]
    fused, confs = ops.fuse_poses(pose, weights, maxprob)
    # mask's (frame, proposal) pairs in mask order, as the boolean scatters: one launch
    # (all_fused[fi, ki] = fused; all_pose[:, fi, ki] = pose; proposal_centers[fi, ki, 4] = confs)
    if (proposal_centers.dtype == torch.float32 and proposal_centers.stride(2) == 1 and all_fused.is_contiguous()
            and all_pose.is_contiguous()):
        ops.scatter_poses(idx, fused, pose, confs, all_fused, all_pose, proposal_centers, 4)
    else:
        fi, ki = idx[:, 0], idx[:, 1]
        all_fused[fi, ki] = fused
        all_pose[:, fi, ki] = pose
        proposal_centers[fi, ki, 4] = confs
