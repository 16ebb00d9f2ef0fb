"""Drop the HIP path into a checkout of the reference (ME495/Faster-VoxelPose).

``install()`` rebinds the reference's hot-path names to this package's
implementations, in the modules that import them, BEFORE the model is built
(``models.faster_voxelpose.get(cfg)``, run/validate.py:68):

    models.project_whole.ProjectLayer        -> fvp.project_whole.ProjectLayer
    models.human_detection_net.ProjectLayer  -> fvp.project_whole.ProjectLayer  (imported name, :11)
    models.project_individual.ProjectLayer   -> fvp.project_individual.ProjectLayer
    models.joint_localization_net.ProjectLayer -> fvp.project_individual.ProjectLayer  (:12)
    core.proposal.nms2D / human_detection_net.nms2D -> fvp.proposal.nms2D  (:12)
    models.human_detection_net.ProposalLayer -> fvp.proposal.ProposalLayer  (:14-125)

With ``fused=True`` it also replaces JointLocalizationNet.forward by
:func:`fvp.jln.fused_jln_forward` (every proposal of a batch at once, soft-argmax
and fusion on fvp kernels; eval mode) and HumanDetectionNet.forward
(human_detection_net.py:157-220) by :func:`fused_hdn_forward`, which takes the
cube AND its xy max-plane from one voxelize launch (skipping CenterNet's
``torch.max(x, dim=4)``, cnns_2d.py:291) and uses the fvp gathers for the
bbox and z-column extraction (:191-192, :199-200) and one launch for the z
pick and the test-mode ProposalLayer (:208-220).  Signatures, outputs and
state_dict keys are unchanged, so run/validate.py and existing checkpoints
work as before.
"""
from __future__ import annotations

import sys

import torch

from . import cnn as fvp_cnn
from . import jln, project_individual, project_whole, proposal

USE_FVP_CNN = False  # set by install(cnn=True)
FVP_CNN_DTYPE = torch.float32


def install(fused: bool = True, modules=None, cnn: bool = False) -> dict:
    """Patch the already-importable reference modules.  Returns what was patched.

    cnn=True (with fused=True): in eval mode the fused forwards run CenterNet,
    C2CNet and P2PNet on the fvp MFMA convolutions (fvp/cnn.py) instead of
    torch's, in fp32, and WeightNet as one fused launch; cnn="bf16": bf16
    operands with fp32 accumulation for the MFMA convolutions (opt-in, ~1e-2
    relative)."""
    global USE_FVP_CNN, FVP_CNN_DTYPE
    USE_FVP_CNN = bool(cnn)
    FVP_CNN_DTYPE = torch.bfloat16 if cnn == "bf16" else torch.float32
    mods = modules if modules is not None else sys.modules
    patched = {}

    def setattr_if(modname, attr, value):
        m = mods.get(modname)
        if m is not None and hasattr(m, attr):
            setattr(m, attr, value)
            patched[f"{modname}.{attr}"] = value

    setattr_if("models.project_whole", "ProjectLayer", project_whole.ProjectLayer)
    setattr_if("models.human_detection_net", "ProjectLayer", project_whole.ProjectLayer)
    setattr_if("models.project_individual", "ProjectLayer", project_individual.ProjectLayer)
    setattr_if("models.joint_localization_net", "ProjectLayer", project_individual.ProjectLayer)
    setattr_if("core.proposal", "nms2D", proposal.nms2D)
    setattr_if("models.human_detection_net", "nms2D", proposal.nms2D)
    setattr_if("models.human_detection_net", "ProposalLayer", proposal.ProposalLayer)
    if fused:
        hdn = mods.get("models.human_detection_net")
        if hdn is not None and hasattr(hdn, "HumanDetectionNet"):
            hdn.HumanDetectionNet.forward = fused_hdn_forward
            patched["models.human_detection_net.HumanDetectionNet.forward"] = fused_hdn_forward
        jn = mods.get("models.joint_localization_net")
        if jn is not None and hasattr(jn, "JointLocalizationNet"):
            cls = jn.JointLocalizationNet
            if not hasattr(cls, "_fvp_original_forward"):
                cls._fvp_original_forward = cls.forward
            cls.forward = jln.fused_jln_forward
            patched["models.joint_localization_net.JointLocalizationNet.forward"] = jln.fused_jln_forward
    return patched


def center_net_from_xy(center_net, xy: torch.Tensor):
    """CenterNet.forward (cnns_2d.py:280-295) minus its first line, fed with
    the xy max-plane the voxelize kernel already produced."""
    if USE_FVP_CNN and not center_net.training:
        return fvp_cnn.cached(center_net, FVP_CNN_DTYPE).from_xy(xy)
    x = center_net.front_layers(xy)
    x = center_net.encoder_decoder(x)
    return center_net.output_hm(x), center_net.output_size(x)


def fused_hdn_forward(self, heatmaps, meta, cameras, resize_transform):
    """HumanDetectionNet.forward (human_detection_net.py:157-220) on the fvp ops.

    Same inputs and outputs: (proposal_heatmaps_2d [B,1,X,Y],
    proposal_heatmaps_1d [B,K,Z], proposal_centers [B,K,7], bbox_preds [B,X*Y,2]).
    """
    batch_size = heatmaps.shape[0]
    cubes, xy = self.project_layer.forward_fused(heatmaps, meta, cameras, resize_transform)
    hm2d, bbox_preds = center_net_from_xy(self.center_net, xy)
    confs_2d, index_2d, flat = proposal.nms2D(hm2d.detach(), self.max_people)
    match_bbox = proposal.gather_bbox(bbox_preds, flat)
    columns = proposal.gather_columns(cubes, flat)                        # [B, K, J, Z]
    c2c = self.c2c_net
    if USE_FVP_CNN and not c2c.training:
        c2c = fvp_cnn.cached(c2c, FVP_CNN_DTYPE)
    hm1d = c2c(torch.flatten(columns, 0, 1)).view(batch_size, self.max_people, -1)
    pl = self.proposal_layer
    if pl.training and ("roots_3d" in meta and "num_person" in meta):  # GT matching (training)
        confs_1d, index_1d = hm1d.detach().topk(1)
        topk_index = torch.cat([index_2d, index_1d], dim=2)
        centers = pl(topk_index, confs_2d * confs_1d.squeeze(2), match_bbox, meta)
    else:  # z pick + ProposalLayer test mode in one launch (human_detection_net.py:208-220, :99-124)
        centers = proposal.proposal_centers(pl, index_2d, hm1d.detach(), confs_2d, match_bbox)
    return hm2d, hm1d, centers, torch.flatten(bbox_preds, 2, 3).permute(0, 2, 1)
