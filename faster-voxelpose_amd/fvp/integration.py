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

With ``backbone=True`` the PoseResNet heatmap backbone runs on the fvp MFMA
convolutions (fvp.backbone; resnet.py:98-201) in eval mode:

    models.resnet.ResNet.forward             -> fvp_resnet_forward
    models.faster_voxelpose.FasterVoxelPoseNet.forward -> fused_fvp_forward (fused=True)

the latter runs the backbone once over all views of the batch (instead of the
per-view loop and stack of faster_voxelpose.py:73-75) and hands the HDN and
JLN the channels-last heatmaps the backbone writes, so neither re-lays them
out; ``input_heatmaps`` is still returned in the reference layout.

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

import dataclasses
import os
import sys

import torch

from . import backbone as fvp_backbone
from . import cnn as fvp_cnn
from . import heatmaps as fvp_heatmaps
from . import jln, project_individual, project_whole, proposal


def _env_recompute():
    v = os.environ.get("FVP_RECOMPUTE_COLUMNS")
    return None if v is None else v != "0"


@dataclasses.dataclass(frozen=True)
class FvpOptions:
    """How the fused forwards run, per model (no process-wide switches).

    install() attaches one to the classes it patches; set_options(model, ...)
    gives one model (and every submodule) its own; a forward reads the
    options of the module it runs on (``options_of``), so two models in one
    process can differ.

    cnn / cnn_dtype: in eval mode run CenterNet, C2CNet, P2PNet on the fvp MFMA
      convolutions (fvp/cnn.py) and WeightNet as one fused launch; bf16 =
      bf16 operands with fp32 accumulation (opt-in, ~1e-2 relative).
    backbone / backbone_dtype: the same for the PoseResNet backbone.
    recompute_columns: fused_hdn_forward writes no cube and recomputes the K
      winners' z-columns from the heatmaps (fvp_voxel_columns, bit-identical to
      gathering them from the cube); None = only when the batch's cube would
      exceed recompute_cube_bytes (a memory saving: the TD-bound gather hides
      the cube writes, so below that the one-launch NMS + column gather is as
      fast or faster).  Default from the environment variable
      FVP_RECOMPUTE_COLUMNS (0 / 1) when set.
    c2c_graphs: with cnn, the launch-bound 1-D C2CNet replays from a
      hipGraph per column-batch shape (fvp.cnn.GraphedCNN) when it does not run
      as one launch (fvp.cnn.Net1D).
    share_layout: fused_hdn_forward lays planar fp32 heatmaps out channels-last
      ONCE for the batch (fvp.heatmaps.to_channels_last) and attaches the copy
      to the heatmaps tensor, so its own gather and the JLN's person planes
      (the same tensor object, faster_voxelpose.py:85-93) both read it in
      place -- one layout pass per batch instead of one per consumer."""
    cnn: bool = False
    cnn_dtype: torch.dtype = torch.float32
    backbone: bool = False
    backbone_dtype: torch.dtype = torch.float32
    recompute_columns: bool | None = dataclasses.field(default_factory=_env_recompute)
    recompute_cube_bytes: int = 512 << 20
    c2c_graphs: bool = True
    share_layout: bool = True


DEFAULT_OPTIONS = FvpOptions()


def options_of(module) -> FvpOptions:
    """The FvpOptions a fused forward on `module` uses (its own, its class's, or the defaults)."""
    opts = getattr(module, "fvp_options", None)
    return opts if isinstance(opts, FvpOptions) else DEFAULT_OPTIONS


def set_options(model, **changes) -> FvpOptions:
    """Give `model` and every submodule (an nn.Module's modules(); or just the
    object) its own options: the current ones with `changes` applied.  No
    parameters or buffers are added, so state_dict is unchanged."""
    opts = dataclasses.replace(options_of(model), **changes)
    for m in (model.modules() if hasattr(model, "modules") else [model]):
        object.__setattr__(m, "fvp_options", opts)  # plain attribute (not a submodule / parameter)
    return opts


def install(fused: bool = True, modules=None, cnn: bool = False, backbone: bool = False) -> dict:
    """Patch the already-importable reference modules.  Returns what was patched.

    cnn=True (with fused=True): in eval mode the fused forwards run CenterNet,
    C2CNet and P2PNet on the fvp MFMA convolutions (fvp/cnn.py) instead of
    torch's, in fp32, and WeightNet as one fused launch; cnn="bf16": bf16
    operands with fp32 accumulation for the MFMA convolutions (opt-in, ~1e-2
    relative).  backbone=True / "bf16": the same for the PoseResNet backbone.
    These become the FvpOptions of the patched classes (per-model overrides:
    set_options)."""
    opts = FvpOptions(cnn=bool(cnn), cnn_dtype=torch.bfloat16 if cnn == "bf16" else torch.float32,
                      backbone=bool(backbone), backbone_dtype=torch.bfloat16 if backbone == "bf16" else torch.float32)
    mods = modules if modules is not None else sys.modules
    patched = {}

    def setattr_if(modname, attr, value):
        m = mods.get(modname)
        if m is not None and hasattr(m, attr):
            setattr(m, attr, value)
            patched[f"{modname}.{attr}"] = value

    for modname, cls in (("models.human_detection_net", "HumanDetectionNet"),
                         ("models.joint_localization_net", "JointLocalizationNet"),
                         ("models.resnet", "ResNet"), ("models.faster_voxelpose", "FasterVoxelPoseNet")):
        m = mods.get(modname)
        if m is not None and hasattr(m, cls):
            getattr(m, cls).fvp_options = opts
            patched[f"{modname}.{cls}.fvp_options"] = opts
    setattr_if("models.project_whole", "ProjectLayer", project_whole.ProjectLayer)
    setattr_if("models.human_detection_net", "ProjectLayer", project_whole.ProjectLayer)
    setattr_if("models.project_individual", "ProjectLayer", project_individual.ProjectLayer)
    setattr_if("models.joint_localization_net", "ProjectLayer", project_individual.ProjectLayer)
    setattr_if("core.proposal", "nms2D", proposal.nms2D)
    setattr_if("models.human_detection_net", "nms2D", proposal.nms2D)
    setattr_if("models.human_detection_net", "ProposalLayer", proposal.ProposalLayer)
    if backbone:
        rn = mods.get("models.resnet")
        if rn is not None and hasattr(rn, "ResNet"):
            cls = rn.ResNet
            if not hasattr(cls, "_fvp_original_forward"):
                cls._fvp_original_forward = cls.forward
            cls.forward = fvp_resnet_forward
            patched["models.resnet.ResNet.forward"] = fvp_resnet_forward
        fv = mods.get("models.faster_voxelpose")
        if fused and fv is not None and hasattr(fv, "FasterVoxelPoseNet"):
            cls = fv.FasterVoxelPoseNet
            if not hasattr(cls, "_fvp_original_forward"):
                cls._fvp_original_forward = cls.forward
            cls.forward = fused_fvp_forward
            patched["models.faster_voxelpose.FasterVoxelPoseNet.forward"] = fused_fvp_forward
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


def center_net_from_xy(center_net, xy: torch.Tensor, opts: FvpOptions = DEFAULT_OPTIONS):
    """CenterNet.forward (cnns_2d.py:280-295) minus its first line, fed with
    the xy max-plane the voxelize kernel already produced."""
    if opts.cnn and not center_net.training:
        return fvp_cnn.cached(center_net, opts.cnn_dtype).from_xy(xy)
    x = center_net.front_layers(xy)
    x = center_net.encoder_decoder(x)
    return center_net.output_hm(x), center_net.output_size(x)


def fused_hdn_forward(self, heatmaps, meta, cameras, resize_transform):
    """HumanDetectionNet.forward (human_detection_net.py:157-220) on the fvp ops.

    Same inputs and outputs: (proposal_heatmaps_2d [B,1,X,Y],
    proposal_heatmaps_1d [B,K,Z], proposal_centers [B,K,7], bbox_preds [B,X*Y,2]).
    """
    batch_size = heatmaps.shape[0]
    opts = options_of(self)
    pl_ = self.project_layer
    if opts.share_layout:
        fvp_heatmaps.share_channels_last(heatmaps)
    recompute = opts.recompute_columns
    if recompute is None:
        X, Y, Z = (int(v) for v in pl_.voxels_per_axis)
        recompute = batch_size * heatmaps.shape[2] * X * Y * Z * 4 > opts.recompute_cube_bytes
    if recompute:
        # no cube: the xy plane only, then the winners' columns recomputed (:162-200)
        _, xy = pl_.forward_fused(heatmaps, meta, cameras, resize_transform, want_cube=False, want_xy=True)
        hm2d, bbox_preds = center_net_from_xy(self.center_net, xy, opts)
        confs_2d, index_2d, flat = proposal.nms2D(hm2d, self.max_people)
        columns = pl_.columns(heatmaps, meta, cameras, resize_transform, flat)  # [B,K,J,Z]
    else:
        cubes, xy = pl_.forward_fused(heatmaps, meta, cameras, resize_transform)
        hm2d, bbox_preds = center_net_from_xy(self.center_net, xy, opts)
        # nms2D and the z-column gather of its winners in one launch (:188, :199-200)
        confs_2d, index_2d, flat, columns = proposal.nms2D_columns(hm2d, self.max_people, cubes)
    match_bbox = proposal.gather_bbox(bbox_preds, flat)
    c2c = self.c2c_net
    if opts.cnn and not c2c.training:
        c2c = fvp_cnn.cached(c2c, opts.cnn_dtype, graphs=opts.c2c_graphs)
    hm1d = c2c(torch.flatten(columns, 0, 1)).view(batch_size, self.max_people, -1)
    pl = self.proposal_layer
    if pl.training and ("roots_3d" in meta and "num_person" in meta):  # GT matching (training)
        confs_1d, index_1d = hm1d.detach().topk(1)
        topk_index = torch.cat([index_2d, index_1d], dim=2)
        centers = pl(topk_index, confs_2d * confs_1d.squeeze(2), match_bbox, meta)
    else:  # z pick + ProposalLayer test mode in one launch (human_detection_net.py:208-220, :99-124)
        centers = proposal.proposal_centers(pl, index_2d, hm1d.detach(), confs_2d, match_bbox)
    return hm2d, hm1d, centers, torch.flatten(bbox_preds, 2, 3).permute(0, 2, 1)


def _fvp_backbone_ok(module, x, opts: FvpOptions) -> bool:
    return (opts.backbone and not module.training and isinstance(x, torch.Tensor) and x.is_cuda
            and not (torch.is_grad_enabled() and x.requires_grad))


def fvp_resnet_forward(self, x):
    """ResNet.forward (resnet.py:187-201) on the fvp MFMA convolutions in eval
    mode; the reference's forward in training (BatchNorm batch statistics,
    autograd) and on CPU tensors."""
    opts = options_of(self)
    if _fvp_backbone_ok(self, x, opts):
        return fvp_backbone.cached(self, opts.backbone_dtype)(x)
    return type(self)._fvp_original_forward(self, x)


def fused_fvp_forward(self, backbone=None, views=None, meta=None, targets=None, input_heatmaps=None, cameras=None,
                      resize_transform=None):
    """FasterVoxelPoseNet.forward (faster_voxelpose.py:51-162) with the views
    path on the fvp backbone in eval mode: all B*V views in one pass, heatmaps
    written channels-last once and handed to the HDN / JLN gathers in place
    (fvp.heatmaps.attach); everything after it is the reference's forward."""
    opts = options_of(self)
    attached = None
    if (views is not None and backbone is not None and not self.training and hasattr(backbone, "deconv_layers")
            and _fvp_backbone_ok(backbone, views, opts)):
        cl = fvp_backbone.cached(backbone, opts.backbone_dtype).heatmaps_cl(views)
        input_heatmaps, views = cl.planar(), None  # [B,V,J,H,W], carrying the channels-last copy
        attached = input_heatmaps
    try:
        return type(self)._fvp_original_forward(self, backbone=backbone, views=views, meta=meta, targets=targets,
                                                input_heatmaps=input_heatmaps, cameras=cameras,
                                                resize_transform=resize_transform)
    finally:
        # the caller gets the reference's plain planar heatmaps: the copy does not outlive the forward
        fvp_heatmaps.release(attached)
