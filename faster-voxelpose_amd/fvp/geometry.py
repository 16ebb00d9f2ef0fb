"""Host-side geometry for the voxel-projection path (no GPU work, no torch kernels).

Everything here is one-time setup that the reference performs on the host or in
tiny torch ops before the hot path runs:

* camera dictionaries -> packed fp32 records the HIP kernels read
  (reference: lib/utils/cameras.py:11-18 ``unfold_camera_param``);
* the 2x3 ``resize_transform`` without cv2
  (reference: lib/utils/transforms.py:15-50 ``get_affine_transform``,
  :81-92 ``get_scale``; lib/dataset/JointsDataset.py:68-78);
* the per-person layer constants ``fine_voxels_per_axis``, ``scale``, ``bias``
  (reference: lib/models/project_individual.py:43-85), computed with the same
  fp32 tensor ops so the values are bit-identical.
"""
from __future__ import annotations

import numpy as np

# Packed camera record, fp32, one row per camera (see include/fvp.h FVP_CAM_STRIDE).
#   [0:9]  R (row major)      [9:12] T (camera centre, mm)
#   [12] fx [13] fy [14] cx [15] cy
#   [16:19] k (radial)        [19:21] p (tangential)   [21:24] zero pad
CAM_STRIDE = 24


def _f32(x) -> np.ndarray:
    # torch.as_tensor(x, dtype=torch.float) on float64 input rounds to nearest fp32.
    return np.asarray(x, dtype=np.float64).astype(np.float32)


def camera_list(cameras, seq):
    """Return the camera records of ``seq`` in view order.

    The reference accepts both ``{seq: [cam, ...]}`` (panoptic.py:171-205) and
    ``{seq: {0: cam, 1: cam, ...}}`` (shelf.py:138-153) and indexes them with
    ``cameras[seq][c]`` for c in range(V) (project_whole.py:155).
    """
    cams = cameras[seq]
    return [cams[c] for c in range(len(cams))]


def pack_camera(cam) -> np.ndarray:
    """One camera dict -> fp32[CAM_STRIDE] (cameras.py:11-18 dtype semantics)."""
    out = np.zeros(CAM_STRIDE, dtype=np.float32)
    out[0:9] = _f32(cam["R"]).reshape(9)
    out[9:12] = _f32(cam["T"]).reshape(3)
    out[12:14] = _f32(np.array([cam["fx"], cam["fy"]], dtype=np.float64)).reshape(2)
    out[14:16] = _f32(np.array([cam["cx"], cam["cy"]], dtype=np.float64)).reshape(2)
    out[16:19] = _f32(cam["k"]).reshape(3)
    out[19:21] = _f32(cam["p"]).reshape(2)
    return out


def pack_cameras(cameras, seq) -> np.ndarray:
    return np.stack([pack_camera(c) for c in camera_list(cameras, seq)])


# ---------------------------------------------------------------------------
# resize transform (cv2-free)
# ---------------------------------------------------------------------------

def get_scale(image_size, resized_size) -> np.ndarray:
    """transforms.py:81-92, verbatim semantics."""
    w, h = image_size
    w_resized, h_resized = resized_size
    if w / w_resized < h / h_resized:
        w_pad = h / h_resized * w_resized
        h_pad = h
    else:
        w_pad = w
        h_pad = w / w_resized * h_resized
    return np.array([w_pad / 200.0, h_pad / 200.0], dtype=np.float32)


def _affine_from_3pts(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """Solve dst = A @ [src, 1] for the 2x3 A in float64 (what
    cv2.getAffineTransform computes from three float32 point pairs)."""
    src = src.astype(np.float64)
    dst = dst.astype(np.float64)
    m = np.zeros((6, 6))
    rhs = np.zeros(6)
    for i in range(3):
        m[2 * i, 0:2] = src[i]
        m[2 * i, 2] = 1.0
        m[2 * i + 1, 3:5] = src[i]
        m[2 * i + 1, 5] = 1.0
        rhs[2 * i] = dst[i, 0]
        rhs[2 * i + 1] = dst[i, 1]
    return np.linalg.solve(m, rhs).reshape(2, 3)


def get_affine_transform(center, scale, rot, output_size):
    """transforms.py:15-50 (shift = 0, inv = 0) with the three-point solve done
    in float64 instead of cv2; the point arrays are float32 as in the reference."""
    scale = np.asarray(scale)
    if scale.ndim == 0:
        scale = np.array([scale, scale])
    scale_tmp = scale * 200.0
    src_w, src_h = scale_tmp[0], scale_tmp[1]
    dst_w, dst_h = output_size[0], output_size[1]
    rot_rad = np.pi * rot / 180

    def get_dir(src_point):
        sn, cs = np.sin(rot_rad), np.cos(rot_rad)
        return [src_point[0] * cs - src_point[1] * sn, src_point[0] * sn + src_point[1] * cs]

    def third(a, b):
        direct = a - b
        return np.array(b) + np.array([-direct[1], direct[0]], dtype=np.float32)

    if src_w >= src_h:
        src_dir = get_dir([0, src_w * -0.5])
        dst_dir = np.array([0, dst_w * -0.5], np.float32)
    else:
        src_dir = get_dir([src_h * -0.5, 0])
        dst_dir = np.array([dst_h * -0.5, 0], np.float32)
    src = np.zeros((3, 2), dtype=np.float32)
    dst = np.zeros((3, 2), dtype=np.float32)
    src[0, :] = center
    src[1, :] = center + src_dir
    dst[0, :] = [dst_w * 0.5, dst_h * 0.5]
    dst[1, :] = np.array([dst_w * 0.5, dst_h * 0.5]) + dst_dir
    src[2:, :] = third(src[0, :], src[1, :])
    dst[2:, :] = third(dst[0, :], dst[1, :])
    return _affine_from_3pts(src, dst)


def resize_transform(ori_image_size, image_size) -> np.ndarray:
    """JointsDataset.py:68-78: the 2x3 float64 matrix every dataset exposes;
    callers hand it to the model as ``torch.as_tensor(..., dtype=torch.float)``."""
    c = np.array([ori_image_size[0] / 2.0, ori_image_size[1] / 2.0])
    s = get_scale((ori_image_size[0], ori_image_size[1]), image_size)
    return get_affine_transform(c, s, 0, image_size)


# ---------------------------------------------------------------------------
# voxel-grid constants
# ---------------------------------------------------------------------------

def linspace_endpoints(size: float):
    """(-S/2, S/2) exactly as ``-boxSize[i] / 2`` (project_whole.py:62-64)."""
    return float(np.float32(-size / 2)), float(np.float32(size / 2))


def grid_axes(space_size, space_center, bins):
    """Per-axis (start, end, n, centre) tuples the kernels rebuild the voxel
    centres from: centre_i = linspace(start, end, n)[i] + centre (fp32).
    (project_whole.py:43-79; project_individual.py:113-149)."""
    axes = []
    for a in range(3):
        s, e = linspace_endpoints(float(space_size[a]))
        axes.append((s, e, int(bins[a]), float(np.float32(space_center[a]))))
    return axes


def individual_constants(whole_size, whole_center, ind_size, ind_bins):
    """project_individual.py:43-85 with torch fp32 semantics.

    Returns dict with fine (int32[3]), scale (f32[3]), bias (f32[3]) plus the
    fp32 copies of the sizes.  Uses torch CPU ops so rounding is identical to
    the reference module's own construction.
    """
    import torch

    wc = torch.tensor(list(map(float, whole_center)))
    ws = torch.tensor(list(map(float, whole_size)))
    isz = torch.tensor(list(map(float, ind_size)))
    vpa = torch.tensor(list(map(int, ind_bins)), dtype=torch.int32)
    fine = (ws / isz * (vpa - 1)).int() + 1
    scale = (fine.float() - 1) / ws
    bias = -isz / 2.0 / ws * (fine - 1) - scale * (wc - ws / 2.0)
    return {
        "fine": fine.numpy().astype(np.int32),
        "scale": scale.numpy().astype(np.float32),
        "bias": bias.numpy().astype(np.float32),
        "whole_size": ws.numpy(),
        "whole_center": wc.numpy(),
        "ind_size": isz.numpy(),
        "ind_bins": vpa.numpy(),
    }
