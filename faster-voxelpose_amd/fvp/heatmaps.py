"""Channels-last heatmaps: the layout the voxelize and person gathers read.

The reference's heatmaps are ``[B, V, J, H, W]`` (one plane per joint).  The
fvp backbone (fvp.backbone) writes them channels-last, ``[B, V, H, W, Cp]``
with the J joints in channels 0..J-1 -- one 64-B pixel holds every joint of a
bilinear tap -- so the gathers read them in place instead of re-laying them
out first (fvp_voxelize_cl).  A :class:`ChannelsLastHeatmaps` can travel
through the reference's interfaces attached to the planar tensor it equals
(:func:`attach`), because those interfaces take a plain tensor.
"""
from __future__ import annotations

import torch

from . import _lib


class ChannelsLastHeatmaps:
    """Heatmaps [B, V, J, H, W] stored as ``t`` = [B, V, H, W, Cp] fp32 (Cp >= J)."""

    def __init__(self, t: torch.Tensor, num_joints: int):
        if t.dim() != 5 or t.dtype != torch.float32 or not t.is_contiguous() or t.shape[4] < num_joints:
            raise _lib.FvpError(f"fvp: channels-last heatmaps must be contiguous fp32 [B,V,H,W,Cp>=J], got "
                                f"{tuple(t.shape)} {t.dtype}")
        self.t, self.J = t, int(num_joints)

    @property
    def shape(self) -> tuple:
        B, V, H, W, _ = self.t.shape
        return (B, V, self.J, H, W)

    @property
    def device(self):
        return self.t.device

    @property
    def cp(self) -> int:
        return self.t.shape[4]

    def planar(self) -> torch.Tensor:
        """[B, V, J, H, W] fp32 (the reference layout), carrying this object (attach)."""
        B, V, J, H, W = self.shape
        out = torch.empty((B, V, J, H, W), dtype=torch.float32, device=self.t.device)
        if out.numel():
            from .ops import _ptr, _stream
            _lib.call("fvp_nhwc_to_nchw", _ptr(self.t), B * V, J, H, W, self.cp, _ptr(out), _stream(out))
        return attach(out, self)


def attach(planar: torch.Tensor, cl: ChannelsLastHeatmaps) -> torch.Tensor:
    """Mark `planar` (the same values in the reference layout) as also held
    channels-last.  Only this tensor object carries the mark: any op on it
    (view, stack, slice, in-place write) yields a tensor without it, so a
    consumer never reads a stale copy through the mark."""
    if tuple(planar.shape) != cl.shape:
        raise _lib.FvpError(f"fvp: planar {tuple(planar.shape)} and channels-last {cl.shape} heatmaps differ")
    planar._fvp_cl = (cl, planar._version)
    return planar


def channels_last_of(heatmaps) -> ChannelsLastHeatmaps | None:
    """The channels-last copy of `heatmaps`, if it is one or carries one still valid."""
    if isinstance(heatmaps, ChannelsLastHeatmaps):
        return heatmaps
    mark = getattr(heatmaps, "_fvp_cl", None)
    if mark is None or mark[1] != heatmaps._version:  # written in place since: stale
        return None
    return mark[0]
