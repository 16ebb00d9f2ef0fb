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


def attach(planar: torch.Tensor, cl: ChannelsLastHeatmaps, shared: bool = False) -> torch.Tensor:
    """Mark `planar` (the same values in the reference layout) as also held
    channels-last.  Only this tensor object carries the mark: any op on it
    (view, stack, slice, in-place write) yields a tensor without it, so a
    consumer never reads a stale copy through the mark.  `shared`: the mark is
    a fused HDN's one-forward layout (share_channels_last), never reused by a
    later HDN call and dropped by the JLN that consumes it (release)."""
    if tuple(planar.shape) != cl.shape:
        raise _lib.FvpError(f"fvp: planar {tuple(planar.shape)} and channels-last {cl.shape} heatmaps differ")
    planar._fvp_cl = (cl, planar._version, bool(shared))
    return planar


def channels_last_of(heatmaps, reuse_shared: bool = True) -> ChannelsLastHeatmaps | None:
    """The channels-last copy of `heatmaps`, if it is one or carries one still valid
    (reuse_shared=False: not a copy an earlier share_channels_last made)."""
    if isinstance(heatmaps, ChannelsLastHeatmaps):
        return heatmaps
    mark = getattr(heatmaps, "_fvp_cl", None)
    if mark is None or mark[1] != heatmaps._version:  # written in place since: stale
        return None
    if mark[2] and not reuse_shared:
        return None
    return mark[0]


def release(heatmaps) -> None:
    """Drop the channels-last copy `heatmaps` carries (its memory goes with it)."""
    if isinstance(heatmaps, torch.Tensor) and getattr(heatmaps, "_fvp_cl", None) is not None:
        del heatmaps._fvp_cl


def release_shared(heatmaps) -> None:
    """Drop the copy only if share_channels_last made it (the JLN, its last consumer)."""
    mark = getattr(heatmaps, "_fvp_cl", None) if isinstance(heatmaps, torch.Tensor) else None
    if mark is not None and mark[2]:
        del heatmaps._fvp_cl


def to_channels_last(planar: torch.Tensor) -> ChannelsLastHeatmaps:
    """[B, V, J, H, W] fp32 on a HIP device -> its channels-last copy
    [B, V, H, W, 16 * ceil(J / 16)] (J <= 32), one float4 layout launch
    (fvp_nchw_to_nhwc: the voxelize layout pass over the whole batch)."""
    from .ops import _ptr, _stream

    if planar.dim() != 5 or planar.dtype != torch.float32 or planar.device.type != "cuda":
        raise _lib.FvpError(f"fvp: to_channels_last takes fp32 [B,V,J,H,W] on a HIP device, got "
                            f"{tuple(planar.shape)} {planar.dtype} {planar.device}")
    B, V, J, H, W = planar.shape
    if J > 32:
        raise _lib.FvpError(f"fvp: to_channels_last: {J} joints (at most 32 per pixel)")
    cp = 16 * ((J + 15) // 16)
    src = planar.contiguous()
    t = torch.empty((B, V, H, W, cp), dtype=torch.float32, device=planar.device)
    if t.numel():
        _lib.call("fvp_nchw_to_nhwc", _ptr(src), B * V, J, H, W, cp, _ptr(t), _stream(t))
    return ChannelsLastHeatmaps(t, J)


def share_channels_last(heatmaps) -> ChannelsLastHeatmaps | None:
    """Lay `heatmaps` out channels-last once and attach the copy (the fused
    HDN forward does this so that the JLN, handed the same tensor object,
    reads the same copy, then drops it: release_shared): planar fp32 tensors of
    <= 32 joints on a HIP device.  A copy attached by the backbone path is used
    as it is; one left by an earlier call of this function is NOT -- the caller
    may have refilled the same buffer through ``.data``, DLPack or the C ABI,
    which do not move ``_version`` -- so every fused forward lays out anew.
    Returns the copy in use, if any."""
    cl = channels_last_of(heatmaps, reuse_shared=False)
    if cl is not None or not isinstance(heatmaps, torch.Tensor):
        return cl
    release(heatmaps)
    if (heatmaps.dim() != 5 or heatmaps.dtype != torch.float32 or heatmaps.device.type != "cuda"
            or heatmaps.shape[2] > 32 or heatmaps.shape[0] == 0
            or (torch.is_grad_enabled() and heatmaps.requires_grad)):
        return None
    cl = to_channels_last(heatmaps)
    attach(heatmaps, cl, shared=True)
    return cl
