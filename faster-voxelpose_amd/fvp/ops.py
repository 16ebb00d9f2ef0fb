"""torch.ops.fvp.* custom ops over the C ABI (include/fvp.h).

Each op allocates its outputs on the input's device and launches on the
current HIP stream; nothing synchronises.  Only a device ("cuda" = HIP on
ROCm) implementation is registered: a CPU tensor raises, there is no CPU
fallback.  The ops are forward-only -- the reference's projection layers have
no parameters and no gradient flows through them -- so an
input that requires grad under grad mode is rejected instead of being
silently detached.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from ._lib import GridSpec, ImageSpec, PersonSpec


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _f3(v):
    return (ctypes.c_float * 3)(*[float(x) for x in v])


def _i3(v):
    return (ctypes.c_int32 * 3)(*[int(x) for x in v])


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def forward_only(*tensors) -> None:
    """Reject autograd inputs: the ops have no backward (called by the layers
    before dispatch, where requires_grad is still visible)."""
    if torch.is_grad_enabled():
        for t in tensors:
            if isinstance(t, torch.Tensor) and t.requires_grad:
                raise _lib.FvpError("fvp: input requires grad; the projection path is forward-only")


def _dev_f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.device.type != "cuda":
        raise _lib.FvpError(f"fvp: {name} must be on a HIP device, got {t.device}")
    return t.to(torch.float32).contiguous() if t.dtype != torch.float32 else t.contiguous()



# -- eager fast path -------------------------------------------------------------------
# torch.library.custom_op dispatch costs ~17 us of host time per call (measured on this
# image: 20 vs 2.7 us for a no-op with the same signature), more than a one-frame
# voxelize gather takes on the GPU.  The names in this module are therefore wrappers
# that call the op's implementation directly when nothing needs the dispatcher, and the
# registered op (torch.ops.fvp.*, with its fake kernel) otherwise: under torch.compile /
# export, for tensor subclasses (fake, functional), under any TorchDispatchMode or
# functorch transform (vmap, grad), and when grad mode is on and an input requires
# grad (the op then raises its "no autograd formula" error instead of returning
# outputs without a grad_fn).  `wrapper.op` is the registered op, `wrapper.impl` the
# undecorated implementation.
def _needs_dispatcher(args, kwargs) -> bool:
    from torch.utils._python_dispatch import _get_current_dispatch_mode

    if (torch.compiler.is_compiling() or _get_current_dispatch_mode() is not None
            or torch._C._are_functorch_transforms_active()):
        return True
    grad = torch.is_grad_enabled()
    for a in (*args, *kwargs.values()):
        if isinstance(a, torch.Tensor) and (type(a) is not torch.Tensor or (grad and a.requires_grad)):
            return True
    return False


def _custom_op(name: str, **kw):
    def deco(impl):
        op = torch.library.custom_op(name, **kw)(impl)

        def call(*args, **kwargs):
            if _needs_dispatcher(args, kwargs):
                return op(*args, **kwargs)
            return impl(*args, **kwargs)

        call.__name__, call.__qualname__, call.__doc__ = impl.__name__, impl.__qualname__, impl.__doc__
        call.op = op  # the registered custom op
        call.impl = impl  # the implementation the fast path calls
        call.register_fake = op.register_fake
        return call

    return deco

# ---------------------------------------------------------------------------
@_custom_op("fvp::project_grid", mutates_args=(), device_types="cuda")
def project_grid(cams: torch.Tensor, resize_t: torch.Tensor, start: list[float], end: list[float],
                 center: list[float], bins: list[int], ori_max: float, img_w: float, img_h: float,
                 hm_w: int, hm_h: int) -> torch.Tensor:
    cams = _dev_f32(cams, "cams")
    resize_t = _dev_f32(resize_t, "resize_transform")
    V = cams.shape[0]
    N = bins[0] * bins[1] * bins[2]
    out = torch.empty((V, N, 2), dtype=torch.float32, device=cams.device)
    g = GridSpec(_f3(start), _f3(end), _f3(center), _i3(bins))
    im = ImageSpec(ori_max, img_w, img_h, hm_w, hm_h)
    _lib.call("fvp_project_grid", _ptr(cams), V, _ptr(resize_t), g, im, _ptr(out), _stream(cams))
    return out


@project_grid.register_fake
def _(cams, resize_t, start, end, center, bins, ori_max, img_w, img_h, hm_w, hm_h):
    return cams.new_empty((cams.shape[0], bins[0] * bins[1] * bins[2], 2))


# ---------------------------------------------------------------------------
def grid_slots(V: int) -> int:
    """Camera slots per voxel of a packed grid (FVP_GRID_SLOTS: V rounded up to even)."""
    return V + (V & 1)


@_custom_op("fvp::pack_grid", mutates_args=(), device_types="cuda")
def pack_grid(sample_grid: torch.Tensor) -> torch.Tensor:
    """[V,N,2] (the reference's per-camera layout) -> voxel-major [N,GV,2] read by fvp_voxelize."""
    sg = _dev_f32(sample_grid, "sample_grid")
    V, N = sg.shape[0], sg.shape[1]
    out = torch.empty((N, grid_slots(V), 2), dtype=torch.float32, device=sg.device)
    _lib.call("fvp_pack_grid", _ptr(sg), V, N, _ptr(out), _stream(sg))
    return out


@pack_grid.register_fake
def _(sample_grid):
    V, N = sample_grid.shape[0], sample_grid.shape[1]
    return sample_grid.new_empty((N, grid_slots(V), 2))


def packed_as_reference(packed: torch.Tensor, V: int) -> torch.Tensor:
    """View [V,1,N,2] of a packed grid [N,GV,2]: the reference's sample_grid layout, no copy."""
    return packed.permute(1, 0, 2)[:V].unsqueeze(1)


@_custom_op("fvp::voxelize", mutates_args=(), device_types="cuda")
def voxelize(heatmaps: torch.Tensor, packed_grids: torch.Tensor, grid_index: Optional[torch.Tensor],
             X: int, Y: int, Z: int, want_cube: bool, want_xy: bool) -> tuple[torch.Tensor, torch.Tensor]:
    """packed_grids: [S,N,GV,2] (or [N,GV,2]) from pack_grid; grid_index: int [B] sequence of frame b."""
    if heatmaps.device.type != "cuda":
        raise _lib.FvpError(f"fvp: heatmaps must be on a HIP device, got {heatmaps.device}")
    half = heatmaps.dtype == torch.float16
    hm = heatmaps.contiguous() if half else _dev_f32(heatmaps, "heatmaps")
    pg = _dev_f32(packed_grids, "packed_grids")
    B, V, J, H, W = hm.shape
    N = X * Y * Z
    if pg.dim() == 3:
        pg = pg.unsqueeze(0)
    if pg.shape[1:] != (N, grid_slots(V), 2):
        raise _lib.FvpError(f"fvp: packed grid {tuple(pg.shape)} does not match V={V}, N={N} "
                            f"(expected [S,{N},{grid_slots(V)},2] from pack_grid)")
    gi = _grid_index(grid_index, B, pg.shape[0], hm.device)
    cube = torch.empty((B, J, X, Y, Z) if want_cube else (0,), dtype=torch.float32, device=hm.device)
    xy = torch.empty((B, J, X, Y) if want_xy else (0,), dtype=torch.float32, device=hm.device)
    if B == 0:  # an empty batch: the reference's loop over frames yields empty outputs
        return cube, xy
    lib = _lib.load()
    ws_bytes = (lib.fvp_voxelize_f16_workspace_bytes if half else lib.fvp_voxelize_workspace_bytes)(B, V, J, H, W)
    if ws_bytes == 0:
        raise _lib.FvpError(f"fvp: unsupported heatmap shape {tuple(hm.shape)} (J <= 1024)")
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=hm.device)
    _lib.call("fvp_voxelize_f16" if half else "fvp_voxelize", _ptr(hm), B, V, J, H, W, _ptr(pg), _ptr(gi), X, Y, Z,
              _ptr(cube) if want_cube else None, _ptr(xy) if want_xy else None, _ptr(ws), ws_bytes, _stream(hm))
    return cube, xy


@_custom_op("fvp::voxelize_cams", mutates_args=(), device_types="cuda")
def voxelize_cams(heatmaps: torch.Tensor, cams: torch.Tensor, grid_index: Optional[torch.Tensor],
                  resize_t: torch.Tensor, start: list[float], end: list[float], center: list[float], bins: list[int],
                  ori_max: float, img_w: float, img_h: float, want_cube: bool,
                  want_xy: bool, x_begin: int = 0, x_end: int = -1) -> tuple[torch.Tensor, torch.Tensor]:
    """voxelize with the sampling coordinates projected on the fly from packed camera
    records cams [S,V,FVP_CAM_STRIDE] (no cached grid; for grids too large to stay cached).
    x_begin / x_end (-1: bins[0]): only the voxels of x-rows [x_begin, x_end) of the
    grid -- an x-slab of the large-frame mode -- as cube [B,J,x_end-x_begin,Y,Z]."""
    if heatmaps.device.type != "cuda":
        raise _lib.FvpError(f"fvp: heatmaps must be on a HIP device, got {heatmaps.device}")
    half = heatmaps.dtype == torch.float16
    hm = heatmaps.contiguous() if half else _dev_f32(heatmaps, "heatmaps")
    cm = _dev_f32(cams, "cams")
    rt = _dev_f32(resize_t, "resize_transform")
    B, V, J, H, W = hm.shape
    if cm.dim() == 2:
        cm = cm.unsqueeze(0)
    if cm.shape[1] != V:
        raise _lib.FvpError(f"fvp: {cm.shape[1]} camera records for {V} heatmap views")
    x0, x1, X, Y, Z = _x_rows(bins, x_begin, x_end)
    gi = _grid_index(grid_index, B, cm.shape[0], hm.device)
    cube = torch.empty((B, J, X, Y, Z) if want_cube else (0,), dtype=torch.float32, device=hm.device)
    xy = torch.empty((B, J, X, Y) if want_xy else (0,), dtype=torch.float32, device=hm.device)
    if B == 0:  # an empty batch: the reference's loop over frames yields empty outputs
        return cube, xy
    lib = _lib.load()
    ws_bytes = (lib.fvp_voxelize_f16_workspace_bytes if half else lib.fvp_voxelize_workspace_bytes)(B, V, J, H, W)
    if ws_bytes == 0:
        raise _lib.FvpError(f"fvp: unsupported heatmap shape {tuple(hm.shape)} (J <= 1024)")
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=hm.device)
    g = GridSpec(_f3(start), _f3(end), _f3(center), _i3(bins))
    im = ImageSpec(ori_max, img_w, img_h, W, H)
    outs = (_ptr(cube) if want_cube else None, _ptr(xy) if want_xy else None, _ptr(ws), ws_bytes, _stream(hm))
    if X == bins[0]:
        _lib.call("fvp_voxelize_cams", _ptr(hm), int(half), B, V, J, H, W, _ptr(cm), _ptr(gi), _ptr(rt), g, im, *outs)
    else:
        _lib.call("fvp_voxelize_cams_slab", _ptr(hm), int(half), B, V, J, H, W, _ptr(cm), _ptr(gi), _ptr(rt), g, im,
                  x0, x1, *outs)
    return cube, xy


def _x_rows(bins, x_begin: int, x_end: int):
    """(x0, x1, rows, Y, Z) of an x-row range of a grid (x_end = -1: to the end)."""
    X, Y, Z = (int(b) for b in bins)
    x1 = X if x_end < 0 else int(x_end)
    if not 0 <= x_begin < x1 <= X:
        raise ValueError(f"x-slab [{x_begin}, {x1}) outside [0, {X})")
    return int(x_begin), x1, x1 - int(x_begin), Y, Z


@voxelize_cams.register_fake
def _(heatmaps, cams, grid_index, resize_t, start, end, center, bins, ori_max, img_w, img_h, want_cube, want_xy,
      x_begin=0, x_end=-1):
    B, V, J = heatmaps.shape[:3]
    _, _, X, Y, Z = _x_rows(bins, x_begin, x_end)
    return (heatmaps.new_empty((B, J, X, Y, Z) if want_cube else (0,)),
            heatmaps.new_empty((B, J, X, Y) if want_xy else (0,)))


@voxelize.register_fake
def _(heatmaps, packed_grids, grid_index, X, Y, Z, want_cube, want_xy):
    B, V, J = heatmaps.shape[:3]
    return (heatmaps.new_empty((B, J, X, Y, Z) if want_cube else (0,)),
            heatmaps.new_empty((B, J, X, Y) if want_xy else (0,)))


def _grid_index(grid_index: Optional[torch.Tensor], B: int, S: int, device) -> Optional[torch.Tensor]:
    """int32 [B] sequence index of every frame on `device`.  A host tensor is
    range-checked here, before the copy (no device sync); a device tensor's
    values are the caller's precondition (0 <= g < S, include/fvp.h)."""
    if grid_index is None:
        return None
    if grid_index.numel() != B:
        raise _lib.FvpError("fvp: grid_index must have one entry per frame")
    if grid_index.device.type == "cpu" and B and (int(grid_index.min()) < 0 or int(grid_index.max()) >= S):
        raise _lib.FvpError(f"fvp: grid_index values must lie in [0, {S})")
    return grid_index.to(device=device, dtype=torch.int32, non_blocking=True).contiguous()


def _cl_input(heatmaps_cl: torch.Tensor, J: int) -> torch.Tensor:
    if heatmaps_cl.device.type != "cuda":
        raise _lib.FvpError(f"fvp: heatmaps must be on a HIP device, got {heatmaps_cl.device}")
    if heatmaps_cl.dim() != 5 or heatmaps_cl.dtype != torch.float32 or heatmaps_cl.shape[4] < J:
        raise _lib.FvpError(f"fvp: channels-last heatmaps must be fp32 [B,V,H,W,Cp>=J], got "
                            f"{tuple(heatmaps_cl.shape)} {heatmaps_cl.dtype}")
    return heatmaps_cl.contiguous()


@_custom_op("fvp::voxelize_cl", mutates_args=(), device_types="cuda")
def voxelize_cl(heatmaps_cl: torch.Tensor, J: int, packed_grids: torch.Tensor, grid_index: Optional[torch.Tensor],
                X: int, Y: int, Z: int, want_cube: bool, want_xy: bool) -> tuple[torch.Tensor, torch.Tensor]:
    """voxelize on channels-last heatmaps [B,V,H,W,Cp] (joints in channels 0..J-1): no layout pass."""
    hm = _cl_input(heatmaps_cl, J)
    pg = _dev_f32(packed_grids, "packed_grids")
    B, V, H, W, cp = hm.shape
    N = X * Y * Z
    if pg.dim() == 3:
        pg = pg.unsqueeze(0)
    if pg.shape[1:] != (N, grid_slots(V), 2):
        raise _lib.FvpError(f"fvp: packed grid {tuple(pg.shape)} does not match V={V}, N={N}")
    gi = _grid_index(grid_index, B, pg.shape[0], hm.device)
    cube = torch.empty((B, J, X, Y, Z) if want_cube else (0,), dtype=torch.float32, device=hm.device)
    xy = torch.empty((B, J, X, Y) if want_xy else (0,), dtype=torch.float32, device=hm.device)
    if B == 0:
        return cube, xy
    _lib.call("fvp_voxelize_cl", _ptr(hm), cp, B, V, J, H, W, _ptr(pg), _ptr(gi), X, Y, Z,
              _ptr(cube) if want_cube else None, _ptr(xy) if want_xy else None, _stream(hm))
    return cube, xy


@voxelize_cl.register_fake
def _(heatmaps_cl, J, packed_grids, grid_index, X, Y, Z, want_cube, want_xy):
    B = heatmaps_cl.shape[0]
    return (heatmaps_cl.new_empty((B, J, X, Y, Z) if want_cube else (0,)),
            heatmaps_cl.new_empty((B, J, X, Y) if want_xy else (0,)))


@_custom_op("fvp::voxelize_cl_cams", mutates_args=(), device_types="cuda")
def voxelize_cl_cams(heatmaps_cl: torch.Tensor, J: int, cams: torch.Tensor, grid_index: Optional[torch.Tensor],
                     resize_t: torch.Tensor, start: list[float], end: list[float], center: list[float],
                     bins: list[int], ori_max: float, img_w: float, img_h: float, want_cube: bool,
                     want_xy: bool, x_begin: int = 0, x_end: int = -1) -> tuple[torch.Tensor, torch.Tensor]:
    """voxelize_cams on channels-last heatmaps [B,V,H,W,Cp] (x_begin / x_end as there)."""
    hm = _cl_input(heatmaps_cl, J)
    cm = _dev_f32(cams, "cams")
    rt = _dev_f32(resize_t, "resize_transform")
    B, V, H, W, cp = hm.shape
    if cm.dim() == 2:
        cm = cm.unsqueeze(0)
    if cm.shape[1] != V:
        raise _lib.FvpError(f"fvp: {cm.shape[1]} camera records for {V} heatmap views")
    x0, x1, X, Y, Z = _x_rows(bins, x_begin, x_end)
    gi = _grid_index(grid_index, B, cm.shape[0], hm.device)
    cube = torch.empty((B, J, X, Y, Z) if want_cube else (0,), dtype=torch.float32, device=hm.device)
    xy = torch.empty((B, J, X, Y) if want_xy else (0,), dtype=torch.float32, device=hm.device)
    if B == 0:
        return cube, xy
    g = GridSpec(_f3(start), _f3(end), _f3(center), _i3(bins))
    im = ImageSpec(ori_max, img_w, img_h, W, H)
    outs = (_ptr(cube) if want_cube else None, _ptr(xy) if want_xy else None, _stream(hm))
    if X == bins[0]:
        _lib.call("fvp_voxelize_cl_cams", _ptr(hm), cp, B, V, J, H, W, _ptr(cm), _ptr(gi), _ptr(rt), g, im, *outs)
    else:
        _lib.call("fvp_voxelize_cl_cams_slab", _ptr(hm), cp, B, V, J, H, W, _ptr(cm), _ptr(gi), _ptr(rt), g, im,
                  x0, x1, *outs)
    return cube, xy


@voxelize_cl_cams.register_fake
def _(heatmaps_cl, J, cams, grid_index, resize_t, start, end, center, bins, ori_max, img_w, img_h, want_cube,
      want_xy, x_begin=0, x_end=-1):
    B = heatmaps_cl.shape[0]
    _, _, X, Y, Z = _x_rows(bins, x_begin, x_end)
    return (heatmaps_cl.new_empty((B, J, X, Y, Z) if want_cube else (0,)),
            heatmaps_cl.new_empty((B, J, X, Y) if want_xy else (0,)))


# ---------------------------------------------------------------------------
@_custom_op("fvp::nms_topk", mutates_args=(), device_types="cuda")
def nms_topk(prob: torch.Tensor, K: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    if prob.device.type != "cuda":
        raise _lib.FvpError(f"fvp: prob_map must be on a HIP device, got {prob.device}")
    B, X, Y = prob.shape[0], prob.shape[-2], prob.shape[-1]
    if prob.numel() != B * X * Y:
        raise _lib.FvpError("fvp: nms2D expects a [B, 1, X, Y] map")
    p = prob
    # a channel slice of a contiguous [B,C,X,Y] tensor is passed by frame stride, without a copy
    # (a batch stride below X*Y -- e.g. an expand()ed map with stride 0 -- is copied:
    # the kernel reads each frame's X*Y floats at b*stride)
    if not (p.dtype == torch.float32 and p.stride()[-1] == 1 and p.stride()[-2] == Y
            and (B <= 1 or p.stride()[0] >= X * Y)):
        p = p.to(torch.float32).contiguous()
    stride = p.stride()[0] if B > 1 else X * Y
    vals = torch.empty((B, K), dtype=torch.float32, device=p.device)
    flat = torch.empty((B, K), dtype=torch.int64, device=p.device)
    xy = torch.empty((B, K, 2), dtype=torch.int64, device=p.device)
    if B == 0:
        return vals, xy, flat
    _lib.call("fvp_nms_topk", _ptr(p), B, X, Y, stride, K, _ptr(vals), _ptr(flat), _ptr(xy), _stream(p))
    return vals, xy, flat


def proposal_buffers(B: int, K: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    """(vals [B,K] fp32, flat [B,K] int64), both contiguous, back to back in ONE
    buffer (flat's 8BK bytes, then vals' 4BK): the proposals leave a rank as that
    one buffer (fvp.parallel.gather_proposals, no packing kernels)."""
    buf = torch.empty((12 * B * K,), dtype=torch.uint8, device=device)
    flat = buf[: 8 * B * K].view(torch.int64).view(B, K)
    vals = buf[8 * B * K:].view(torch.float32).view(B, K)
    return vals, flat


def _nms_topk_columns_into(prob, K, cube, vals, flat):
    """fvp_nms_topk_columns into the caller's vals [B,K] fp32 / flat [B,K] int64."""
    if prob.device.type != "cuda":
        raise _lib.FvpError(f"fvp: prob_map must be on a HIP device, got {prob.device}")
    c = _dev_f32(cube, "feature_cubes")
    B, X, Y = prob.shape[0], prob.shape[-2], prob.shape[-1]
    if prob.numel() != B * X * Y or c.dim() != 5 or tuple(c.shape[0:1]) + tuple(c.shape[2:4]) != (B, X, Y):
        raise _lib.FvpError("fvp: nms2D expects a [B, 1, X, Y] map over the cube's [B, J, X, Y, Z] grid")
    p = prob
    if not (p.dtype == torch.float32 and p.stride()[-1] == 1 and p.stride()[-2] == Y
            and (B <= 1 or p.stride()[0] >= X * Y)):
        p = p.to(torch.float32).contiguous()
    stride = p.stride()[0] if B > 1 else X * Y
    J, Z = c.shape[1], c.shape[4]
    xy = torch.empty((B, K, 2), dtype=torch.int64, device=p.device)
    cols = torch.empty((B, K, J, Z), dtype=torch.float32, device=p.device)
    if B == 0 or cols.numel() == 0:
        return vals, xy, flat, cols
    _lib.call("fvp_nms_topk_columns", _ptr(p), B, X, Y, stride, K, _ptr(vals), _ptr(flat), _ptr(xy), _ptr(c), J, Z,
              _ptr(cols), _stream(p))
    return vals, xy, flat, cols


@_custom_op("fvp::nms_topk_columns", mutates_args=(), device_types="cuda")
def nms_topk_columns(prob: torch.Tensor, K: int,
                     cube: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """nms_topk + gather_columns in one launch (fvp_nms_topk_columns): the map's
    top-K and the winners' z-columns [B,K,J,Z] of cube [B,J,X,Y,Z]."""
    B = prob.shape[0]
    vals = torch.empty((B, K), dtype=torch.float32, device=prob.device)
    flat = torch.empty((B, K), dtype=torch.int64, device=prob.device)
    return _nms_topk_columns_into(prob, K, cube, vals, flat)


@nms_topk_columns.register_fake
def _(prob, K, cube):
    B = prob.shape[0]
    return (prob.new_empty((B, K)), prob.new_empty((B, K, 2), dtype=torch.int64),
            prob.new_empty((B, K), dtype=torch.int64), prob.new_empty((B, K, cube.shape[1], cube.shape[4])))


@nms_topk.register_fake
def _(prob, K):
    B = prob.shape[0]
    return (prob.new_empty((B, K)), prob.new_empty((B, K, 2), dtype=torch.int64),
            prob.new_empty((B, K), dtype=torch.int64))


# ---------------------------------------------------------------------------
@_custom_op("fvp::gather_columns", mutates_args=(), device_types="cuda")
def gather_columns(cube: torch.Tensor, flat: torch.Tensor) -> torch.Tensor:
    c = _dev_f32(cube, "feature_cubes")
    B, J, X, Y, Z = c.shape
    f = flat.to(device=c.device, dtype=torch.int64).contiguous()
    K = f.shape[1]
    out = torch.empty((B, K, J, Z), dtype=torch.float32, device=c.device)
    if out.numel() == 0:
        return out
    _lib.call("fvp_gather_columns", _ptr(c), B, J, X, Y, Z, _ptr(f), K, _ptr(out), _stream(c))
    return out


@gather_columns.register_fake
def _(cube, flat):
    B, J, X, Y, Z = cube.shape
    return cube.new_empty((B, flat.shape[1], J, Z))


@_custom_op("fvp::voxel_columns", mutates_args=(), device_types="cuda")
def voxel_columns(heatmaps: torch.Tensor, cl_joints: int, packed_grids: Optional[torch.Tensor],
                  cams: Optional[torch.Tensor], grid_index: Optional[torch.Tensor], resize_t: Optional[torch.Tensor],
                  start: list[float], end: list[float], center: list[float], bins: list[int], ori_max: float,
                  img_w: float, img_h: float, flat: torch.Tensor) -> torch.Tensor:
    """columns[b,k,j,:] = cube[b,j,flat[b,k],:] of the cube voxelize (packed_grids)
    or voxelize_cams (cams) would produce, recomputed for the K winners only
    (fvp_voxel_columns; bit-identical).  heatmaps: planar [B,V,J,H,W] fp32/fp16
    (cl_joints = 0) or channels-last [B,V,H,W,cp] fp32 with cl_joints = J."""
    if heatmaps.device.type != "cuda":
        raise _lib.FvpError(f"fvp: heatmaps must be on a HIP device, got {heatmaps.device}")
    if cl_joints:
        hm = _cl_input(heatmaps, cl_joints)
        B, V, H, W, cp = hm.shape
        J, half, strides = cl_joints, False, (H * W * cp, 1, cp)
    else:
        half = heatmaps.dtype == torch.float16
        hm = heatmaps.contiguous() if half else _dev_f32(heatmaps, "heatmaps")
        B, V, J, H, W = hm.shape
        strides = (J * H * W, H * W, 1)
    X, Y, Z = (int(b) for b in bins)
    f = flat.to(device=hm.device, dtype=torch.int64).contiguous()
    if f.dim() != 2 or f.shape[0] != B:
        raise _lib.FvpError(f"fvp: flat must be [B={B}, K], got {tuple(f.shape)}")
    K = f.shape[1]
    g = im = None
    if packed_grids is not None:
        pg = _dev_f32(packed_grids, "packed_grids")
        if pg.dim() == 3:
            pg = pg.unsqueeze(0)
        if pg.shape[1:] != (X * Y * Z, grid_slots(V), 2):
            raise _lib.FvpError(f"fvp: packed grid {tuple(pg.shape)} does not match V={V}, bins={X, Y, Z}")
        S, cm, rt = pg.shape[0], None, None
    else:
        if cams is None or resize_t is None:
            raise _lib.FvpError("fvp: voxel_columns needs packed_grids, or cams and resize_t")
        pg = None
        cm = _dev_f32(cams, "cams")
        if cm.dim() == 2:
            cm = cm.unsqueeze(0)
        if cm.shape[1] != V:
            raise _lib.FvpError(f"fvp: {cm.shape[1]} camera records for {V} heatmap views")
        S, rt = cm.shape[0], _dev_f32(resize_t, "resize_transform")
        g = GridSpec(_f3(start), _f3(end), _f3(center), _i3(bins))
        im = ImageSpec(ori_max, img_w, img_h, W, H)
    gi = _grid_index(grid_index, B, S, hm.device)
    out = torch.empty((B, K, J, Z), dtype=torch.float32, device=hm.device)
    if out.numel() == 0:
        return out
    _lib.call("fvp_voxel_columns", _ptr(hm), int(half), strides[0], strides[1], strides[2], B, V, J, H, W,
              _ptr(pg) if pg is not None else None, _ptr(cm) if cm is not None else None,
              _ptr(rt) if rt is not None else None, g, im, _ptr(gi), X, Y, Z, _ptr(f), K, _ptr(out), _stream(hm))
    return out


@voxel_columns.register_fake
def _(heatmaps, cl_joints, packed_grids, cams, grid_index, resize_t, start, end, center, bins, ori_max, img_w, img_h,
      flat):
    J = cl_joints if cl_joints else heatmaps.shape[2]
    return heatmaps.new_empty((heatmaps.shape[0], flat.shape[1], J, int(bins[2])), dtype=torch.float32)


@_custom_op("fvp::gather_bbox", mutates_args=(), device_types="cuda")
def gather_bbox(size: torch.Tensor, flat: torch.Tensor) -> torch.Tensor:
    s = _dev_f32(size, "bbox_preds")
    B, _, X, Y = s.shape
    f = flat.to(device=s.device, dtype=torch.int64).contiguous()
    K = f.shape[1]
    out = torch.empty((B, K, 2), dtype=torch.float32, device=s.device)
    if out.numel() == 0:
        return out
    _lib.call("fvp_gather_bbox", _ptr(s), B, X, Y, _ptr(f), K, _ptr(out), _stream(s))
    return out


@gather_bbox.register_fake
def _(size, flat):
    return size.new_empty((size.shape[0], flat.shape[1], 2))


@_custom_op("fvp::proposal_centers", mutates_args=(), device_types="cuda")
def proposal_centers(index: torch.Tensor, hm1d: Optional[torch.Tensor], confs: torch.Tensor, match_bbox: torch.Tensor,
                     scale: list[float], bias: list[float], min_score: float) -> torch.Tensor:
    """Test-mode ProposalLayer.forward (fvp_proposal_centers): with hm1d [B,K,Z] the z pick
    is fused (index int64 [B,K,2]); without it index is the full [B,K,3] -> centers [B,K,7]."""
    c = _dev_f32(confs, "topk_confs")
    B, K = c.shape[0], c.shape[1]
    ix = index.to(device=c.device, dtype=torch.int64).contiguous()
    h = None if hm1d is None else _dev_f32(hm1d, "proposal_heatmaps_1d")
    dims = 2 if h is not None else 3
    bb = _dev_f32(match_bbox, "match_bbox_preds")
    if tuple(ix.shape) != (B, K, dims) or bb.numel() != B * K * 2 or (h is not None and h.shape[:2] != (B, K)):
        raise _lib.FvpError(f"fvp: proposal_centers expects index [B,K,{dims}], confs [B,K], bbox [B,K,2]")
    out = torch.empty((B, K, 7), dtype=torch.float32, device=c.device)
    if out.numel() == 0:
        return out
    f3 = ctypes.c_float * 3
    _lib.call("fvp_proposal_centers", _ptr(ix), dims, _ptr(h), _ptr(c), _ptr(bb), B, K,
              h.shape[2] if h is not None else 0, f3(*scale), f3(*bias), float(min_score), _ptr(out), _stream(c))
    return out


@proposal_centers.register_fake
def _(index, hm1d, confs, match_bbox, scale, bias, min_score):
    return confs.new_empty((confs.shape[0], confs.shape[1], 7))


# ---------------------------------------------------------------------------
@_custom_op("fvp::person_planes", mutates_args=(), device_types="cuda")
def person_planes(heatmaps: torch.Tensor, fine_grid: torch.Tensor, proposals: torch.Tensor,
                  frame_of: Optional[torch.Tensor], fine: list[int], scale: list[float], bias: list[float],
                  whole_size: list[float], ind_size: list[float], bins: list[int], want_cubes: bool,
                  want_planes: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    hm = _dev_f32(heatmaps, "heatmaps")
    fg = _dev_f32(fine_grid, "fine sample grid")
    pc = _dev_f32(proposals, "proposal_centers")
    B, V, J, H, W = hm.shape
    P = pc.shape[0]
    if tuple(fg.shape) != (fine[0] * fine[1] * fine[2], grid_slots(V), 2):
        raise _lib.FvpError("fvp: packed fine grid must be [FX*FY*FZ, GV, 2] (pack_grid of the fine sample grid)")
    fo = None
    if frame_of is not None:
        fo = frame_of.to(device=hm.device, dtype=torch.int32).contiguous()
        if fo.numel() != P:
            raise _lib.FvpError("fvp: frame_of must have one entry per proposal")
    SX, SY, SZ = bins
    cubes = torch.empty((P, J, SX, SY, SZ) if want_cubes else (0,), dtype=torch.float32, device=hm.device)
    planes = torch.empty((3 * P, J, SX, SY) if want_planes else (0,), dtype=torch.float32, device=hm.device)
    offset = torch.empty((P, 3), dtype=torch.float32, device=hm.device)
    if P > 0:
        ws_bytes = _lib.load().fvp_person_workspace_bytes(B, V, J, H, W)
        if ws_bytes == 0:
            raise _lib.FvpError(f"fvp: unsupported heatmap shape {tuple(hm.shape)} (J <= 1024)")
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=hm.device)
        spec = PersonSpec(_i3(fine), _f3(scale), _f3(bias), _f3(whole_size), _f3(ind_size), _i3(bins))
        _lib.call("fvp_person_planes", _ptr(hm), B, V, J, H, W, _ptr(fg), spec, _ptr(pc), _ptr(fo), P,
                  _ptr(cubes) if want_cubes else None, _ptr(planes) if want_planes else None, _ptr(offset),
                  _ptr(ws), ws_bytes, _stream(hm))
    return cubes, planes, offset


@_custom_op("fvp::person_planes_cl", mutates_args=(), device_types="cuda")
def person_planes_cl(heatmaps_cl: torch.Tensor, J: int, fine_grid: torch.Tensor, proposals: torch.Tensor,
                     frame_of: Optional[torch.Tensor], fine: list[int], scale: list[float], bias: list[float],
                     whole_size: list[float], ind_size: list[float], bins: list[int], want_cubes: bool,
                     want_planes: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """person_planes on channels-last heatmaps [B,V,H,W,Cp] (fvp_person_planes_cl): no layout pass."""
    hm = _cl_input(heatmaps_cl, J)
    fg = _dev_f32(fine_grid, "fine sample grid")
    pc = _dev_f32(proposals, "proposal_centers")
    B, V, H, W, cp = hm.shape
    P = pc.shape[0]
    if tuple(fg.shape) != (fine[0] * fine[1] * fine[2], grid_slots(V), 2):
        raise _lib.FvpError("fvp: packed fine grid must be [FX*FY*FZ, GV, 2] (pack_grid of the fine sample grid)")
    fo = None
    if frame_of is not None:
        fo = frame_of.to(device=hm.device, dtype=torch.int32).contiguous()
        if fo.numel() != P:
            raise _lib.FvpError("fvp: frame_of must have one entry per proposal")
    SX, SY, SZ = bins
    cubes = torch.empty((P, J, SX, SY, SZ) if want_cubes else (0,), dtype=torch.float32, device=hm.device)
    planes = torch.empty((3 * P, J, SX, SY) if want_planes else (0,), dtype=torch.float32, device=hm.device)
    offset = torch.empty((P, 3), dtype=torch.float32, device=hm.device)
    if P > 0:
        spec = PersonSpec(_i3(fine), _f3(scale), _f3(bias), _f3(whole_size), _f3(ind_size), _i3(bins))
        _lib.call("fvp_person_planes_cl", _ptr(hm), cp, B, V, J, H, W, _ptr(fg), spec, _ptr(pc), _ptr(fo), P,
                  _ptr(cubes) if want_cubes else None, _ptr(planes) if want_planes else None, _ptr(offset),
                  _stream(hm))
    return cubes, planes, offset


@person_planes_cl.register_fake
def _(heatmaps_cl, J, fine_grid, proposals, frame_of, fine, scale, bias, whole_size, ind_size, bins, want_cubes,
      want_planes):
    P = proposals.shape[0]
    return (heatmaps_cl.new_empty((P, J, bins[0], bins[1], bins[2]) if want_cubes else (0,)),
            heatmaps_cl.new_empty((3 * P, J, bins[0], bins[1]) if want_planes else (0,)),
            heatmaps_cl.new_empty((P, 3)))


@_custom_op("fvp::person_planes_cams", mutates_args=(), device_types="cuda")
def person_planes_cams(heatmaps: torch.Tensor, cams: torch.Tensor, resize_t: torch.Tensor, start: list[float],
                       end: list[float], center: list[float], ori_max: float, img_w: float, img_h: float,
                       proposals: torch.Tensor, frame_of: Optional[torch.Tensor], fine: list[int], scale: list[float],
                       bias: list[float], whole_size: list[float], ind_size: list[float], bins: list[int],
                       want_cubes: bool, want_planes: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """person_planes with the fine-grid coordinates projected on the fly from camera
    records [V,FVP_CAM_STRIDE] (fvp_person_planes_cams): no fine sample grid."""
    hm = _dev_f32(heatmaps, "heatmaps")
    cm = _dev_f32(cams, "cams")
    rt = _dev_f32(resize_t, "resize_transform")
    pc = _dev_f32(proposals, "proposal_centers")
    B, V, J, H, W = hm.shape
    P = pc.shape[0]
    if cm.shape[0] != V:
        raise _lib.FvpError(f"fvp: {cm.shape[0]} camera records for {V} heatmap views")
    fo = None
    if frame_of is not None:
        fo = frame_of.to(device=hm.device, dtype=torch.int32).contiguous()
        if fo.numel() != P:
            raise _lib.FvpError("fvp: frame_of must have one entry per proposal")
    SX, SY, SZ = bins
    cubes = torch.empty((P, J, SX, SY, SZ) if want_cubes else (0,), dtype=torch.float32, device=hm.device)
    planes = torch.empty((3 * P, J, SX, SY) if want_planes else (0,), dtype=torch.float32, device=hm.device)
    offset = torch.empty((P, 3), dtype=torch.float32, device=hm.device)
    if P > 0:
        ws_bytes = _lib.load().fvp_person_workspace_bytes(B, V, J, H, W)
        if ws_bytes == 0:
            raise _lib.FvpError(f"fvp: unsupported heatmap shape {tuple(hm.shape)} (J <= 1024)")
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=hm.device)
        spec = PersonSpec(_i3(fine), _f3(scale), _f3(bias), _f3(whole_size), _f3(ind_size), _i3(bins))
        g = GridSpec(_f3(start), _f3(end), _f3(center), _i3(fine))
        im = ImageSpec(ori_max, img_w, img_h, W, H)
        _lib.call("fvp_person_planes_cams", _ptr(hm), B, V, J, H, W, _ptr(cm), _ptr(rt), g, im, spec, _ptr(pc),
                  _ptr(fo), P, _ptr(cubes) if want_cubes else None, _ptr(planes) if want_planes else None,
                  _ptr(offset), _ptr(ws), ws_bytes, _stream(hm))
    return cubes, planes, offset


@person_planes_cams.register_fake
def _(heatmaps, cams, resize_t, start, end, center, ori_max, img_w, img_h, proposals, frame_of, fine, scale, bias,
      whole_size, ind_size, bins, want_cubes, want_planes):
    P, J = proposals.shape[0], heatmaps.shape[2]
    return (heatmaps.new_empty((P, J, bins[0], bins[1], bins[2]) if want_cubes else (0,)),
            heatmaps.new_empty((3 * P, J, bins[0], bins[1]) if want_planes else (0,)),
            heatmaps.new_empty((P, 3)))


@person_planes.register_fake
def _(heatmaps, fine_grid, proposals, frame_of, fine, scale, bias, whole_size, ind_size, bins, want_cubes,
      want_planes):
    P, J = proposals.shape[0], heatmaps.shape[2]
    return (heatmaps.new_empty((P, J, bins[0], bins[1], bins[2]) if want_cubes else (0,)),
            heatmaps.new_empty((3 * P, J, bins[0], bins[1]) if want_planes else (0,)),
            heatmaps.new_empty((P, 3)))


@_custom_op("fvp::max_planes", mutates_args=(), device_types="cuda")
def max_planes(cubes: torch.Tensor) -> torch.Tensor:
    c = _dev_f32(cubes, "cubes")
    P, J, S = c.shape[0], c.shape[1], c.shape[2]
    if not (c.shape[3] == S and c.shape[4] == S):
        raise _lib.FvpError("fvp: max planes need cubic person volumes (X == Y == Z)")
    planes = torch.empty((3 * P, J, S, S), dtype=torch.float32, device=c.device)
    if P > 0:
        _lib.call("fvp_max_planes", _ptr(c), P, J, S, _ptr(planes), _stream(c))
    return planes


@max_planes.register_fake
def _(cubes):
    P, J, S = cubes.shape[:3]
    return cubes.new_empty((3 * P, J, S, S))


# ---------------------------------------------------------------------------
@_custom_op("fvp::soft_argmax", mutates_args=(), device_types="cuda")
def soft_argmax(features: torch.Tensor, center_grid: torch.Tensor, offset: Optional[torch.Tensor],
                beta: float) -> tuple[torch.Tensor, torch.Tensor]:
    """features [3,P,J,S,S] (or [3,P,J,S*S,1]) -> (pose [3,P,J,2] (+offset), maxprob [3,P,J])."""
    f = _dev_f32(features, "features")
    g = _dev_f32(center_grid, "center_grid")
    P, J = f.shape[1], f.shape[2]
    S2 = f[0, 0, 0].numel() if P > 0 else g.shape[1]
    if g.numel() != 3 * S2 * 2:
        raise _lib.FvpError(f"fvp: center_grid {tuple(g.shape)} does not match {S2} cells per plane")
    off = None if offset is None else _dev_f32(offset, "offset")
    pose = torch.empty((3, P, J, 2), dtype=torch.float32, device=f.device)
    maxprob = torch.empty((3, P, J), dtype=torch.float32, device=f.device)
    _lib.call("fvp_soft_argmax", _ptr(f), P, J, S2, _ptr(g), _ptr(off), float(beta), _ptr(pose), _ptr(maxprob),
              _stream(f))
    return pose, maxprob


@soft_argmax.register_fake
def _(features, center_grid, offset, beta):
    P, J = features.shape[1], features.shape[2]
    return features.new_empty((3, P, J, 2)), features.new_empty((3, P, J))


@_custom_op("fvp::fuse_poses", mutates_args=(), device_types="cuda")
def fuse_poses(pose: torch.Tensor, weights: torch.Tensor, maxprob: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """pose [3,P,J,2], weights [3P,J,1] (WeightNet), maxprob [3,P,J] -> (fused [P,J,3], confs [P])."""
    pz = _dev_f32(pose, "pose")
    w = _dev_f32(weights, "weights")
    mp = _dev_f32(maxprob, "maxprob")
    P, J = pz.shape[1], pz.shape[2]
    if w.numel() != 3 * P * J:
        raise _lib.FvpError(f"fvp: weights {tuple(w.shape)} must hold 3*P*J = {3 * P * J} values")
    fused = torch.empty((P, J, 3), dtype=torch.float32, device=pz.device)
    confs = torch.empty((P,), dtype=torch.float32, device=pz.device)
    _lib.call("fvp_fuse_poses", _ptr(pz), _ptr(w), _ptr(mp), P, J, _ptr(fused), _ptr(confs), _stream(pz))
    return fused, confs


@fuse_poses.register_fake
def _(pose, weights, maxprob):
    P, J = pose.shape[1], pose.shape[2]
    return pose.new_empty((P, J, 3)), pose.new_empty((P,))


def mask_nonzero(mask: torch.Tensor) -> torch.Tensor:
    """``mask.nonzero()`` of a 2-D bool mask on the device in one launch (fvp_mask_nonzero): the
    [count, 2] int64 (row, col) pairs in row-major order.  Reading the count is the one host
    sync, as in torch.nonzero.  Eager only (the count sizes the result)."""
    if mask.dim() != 2 or mask.dtype != torch.bool or mask.device.type != "cuda":
        raise _lib.FvpError(f"fvp: mask_nonzero takes a 2-D bool device tensor, got {tuple(mask.shape)} {mask.dtype}")
    m = mask.contiguous()
    rows, cols = m.shape
    idx = torch.empty((rows * cols, 2), dtype=torch.int64, device=m.device)
    count = torch.empty((1,), dtype=torch.int32, device=m.device)
    if rows * cols == 0:
        return idx
    _lib.call("fvp_mask_nonzero", _ptr(m), rows, cols, _ptr(idx), _ptr(count), _stream(m))
    return idx[:int(count.item())]


def mask_select(mask: torch.Tensor, rows: torch.Tensor) -> tuple:
    """(idx, frame_of, selected) for a [B, K] bool mask and rows [B, K, W] float32 (last dim
    contiguous): ``mask.nonzero()``, its frame column as int32 and ``rows[mask]``, all from one
    launch (fvp_mask_select); the count read is the one host sync, the results are views."""
    if mask.dim() != 2 or mask.dtype != torch.bool or mask.device.type != "cuda":
        raise _lib.FvpError(f"fvp: mask_select takes a 2-D bool device tensor, got {tuple(mask.shape)} {mask.dtype}")
    if (rows.dim() != 3 or tuple(rows.shape[:2]) != tuple(mask.shape) or rows.dtype != torch.float32
            or rows.stride(2) != 1 or rows.device != mask.device):
        raise _lib.FvpError(f"fvp: mask_select rows {tuple(rows.shape)} {rows.dtype} for a mask {tuple(mask.shape)}")
    m = mask.contiguous()
    B, K = m.shape
    W = rows.shape[2]
    idx = torch.empty((B * K, 2), dtype=torch.int64, device=m.device)
    frame_of = torch.empty((B * K,), dtype=torch.int32, device=m.device)
    sel = torch.empty((B * K, W), dtype=torch.float32, device=m.device)
    count = torch.empty((1,), dtype=torch.int32, device=m.device)
    if B * K == 0:
        return idx, frame_of, sel
    _lib.call("fvp_mask_select", _ptr(m), B, K, _ptr(idx), _ptr(count), _ptr(frame_of), _ptr(rows), rows.stride(0),
              rows.stride(1), W, _ptr(sel), _stream(m))
    n = int(count.item())
    return idx[:n], frame_of[:n], sel[:n]


def scatter_poses(idx: torch.Tensor, fused: torch.Tensor, pose: torch.Tensor, confs: torch.Tensor,
                  all_fused: torch.Tensor, all_pose: torch.Tensor, centers: torch.Tensor, conf_col: int = 4) -> None:
    """The JLN's result scatters in one launch (fvp_scatter_poses): all_fused[b, k] = fused,
    all_pose[:, b, k] = pose, centers[b, k, conf_col] = confs for (b, k) = idx rows."""
    P = idx.shape[0]
    if P == 0:
        return
    B, K, J = all_fused.shape[:3]
    for t, shape in ((fused, (P, J, 3)), (pose, (3, P, J, 2)), (confs, (P,)), (all_pose, (3, B, K, J, 2))):
        if tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_contiguous():
            raise _lib.FvpError(f"fvp: scatter_poses operand {tuple(t.shape)} {t.dtype} != {shape} float32")
    if (not all_fused.is_contiguous() or centers.dtype != torch.float32 or centers.dim() != 3
            or centers.stride(2) != 1 or idx.dtype != torch.int64 or idx.dim() != 2 or idx.shape[1] != 2):
        raise _lib.FvpError("fvp: scatter_poses layouts")
    idx = idx.contiguous()  # (torch.nonzero's result is a transposed view on the device)
    _lib.call("fvp_scatter_poses", _ptr(idx), P, B, K, J, _ptr(fused), _ptr(pose), _ptr(confs), _ptr(all_fused),
              _ptr(all_pose), _ptr(centers), centers.stride(0), centers.stride(1), conf_col, _stream(all_fused))


def nms_topk_columns_joint(prob: torch.Tensor, K: int, cube: torch.Tensor):
    """nms_topk_columns with vals / flat in one buffer (proposal_buffers), so
    fvp.parallel.gather_proposals sends them as they are -- eager only: a
    custom op's outputs may not alias each other, so under the dispatcher
    (compile, fake or functional tensors, dispatch modes) the registered op runs."""
    if _needs_dispatcher((prob, cube), {}):
        return nms_topk_columns(prob, K, cube)
    vals, flat = proposal_buffers(prob.shape[0], K, prob.device)
    return _nms_topk_columns_into(prob, K, cube, vals, flat)
