"""Camera dicts from the reference datasets' raw calibration files.

The hot path consumes ``cameras[seq]`` as built by each dataset's ``_get_cam``
(SURVEY.md §8(f) rank 3): a list (Panoptic, custom) or an int-keyed dict
(Shelf) of ``{R, T, fx, fy, cx, cy, k, p}`` with R world->camera, T the camera
centre in mm, k = (k1, k2, k3), p = (p1, p2).  These functions rebuild them
from the parsed calibration JSON with the same float64 numpy arithmetic, so a
service or test can feed :class:`fvp.project_whole.ProjectLayer` without the
reference's dataset classes (which pull in cv2 / json_tricks).  Pinned to the
reference's own ``_get_cam`` output by tests/golden/cams_ref.npz
(tools/gen_camera_golden.py).
"""
from __future__ import annotations

import json

import numpy as np

# Panoptic world frame (y up) -> the project's frame (z up): panoptic.py:173-175
_PANOPTIC_AXES = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, -1.0], [0.0, 1.0, 0.0]])


def panoptic(calib: dict, cam_list) -> list:
    """panoptic.py:171-205 for one sequence: cameras whose (panel, node) is in
    ``cam_list``, in calibration-file order; t is in cm, T comes out in mm."""
    wanted = {tuple(c) for c in cam_list}
    out = []
    for cam in calib["cameras"]:
        if (cam["panel"], cam["node"]) not in wanted:
            continue
        K = np.array(cam["K"])
        dist = np.array(cam["distCoef"])
        R = np.array(cam["R"]).dot(_PANOPTIC_AXES)
        t = np.array(cam["t"]).reshape((3, 1))
        out.append({
            "R": R,
            "T": -np.dot(R.T, t) * 10.0,
            "fx": K[0, 0], "fy": K[1, 1], "cx": K[0, 2], "cy": K[1, 2],
            "k": dist[[0, 1, 4]].reshape(3, 1),
            "p": dist[[2, 3]].reshape(2, 1),
        })
    return out


def custom(calib: dict) -> list:
    """custom.py:111-144: intrinsics k = (fx, fy, cx, cy), distortion d =
    (k1, k2, p1, p2, k3), a 3x4 projection p = K [R | t]; R, t recovered as
    K^-1 p, T = -R^T t (calibration units)."""
    out = []
    for name in calib.keys():
        c = calib[name]
        fx, fy, cx, cy = c["k"][0], c["k"][1], c["k"][2], c["k"][3]
        K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]])
        Rt = np.linalg.inv(K).dot(np.array(c["p"]).reshape(3, 4))
        R, t = Rt[:3, :3], Rt[:3, 3].reshape(3, 1)
        out.append({
            "fx": fx, "fy": fy, "cx": cx, "cy": cy,
            "k": np.array([c["d"][0], c["d"][1], c["d"][4]]).reshape(3, 1),
            "p": np.array([c["d"][2], c["d"][3]]).reshape(2, 1),
            "R": R,
            "T": -np.dot(R.T, t),
        })
    return out


def shelf(calib: dict) -> dict:
    """shelf.py:138-153: the file already holds the project's format; values
    become arrays and the camera ids ints."""
    return {int(i): {k: np.array(v) for k, v in cam.items()} for i, cam in calib.items()}


def load(path: str, kind: str, cam_list=None):
    """Parse ``path`` and convert it: kind "panoptic" (needs ``cam_list``), "custom" or "shelf"."""
    with open(path) as f:
        calib = json.load(f)
    if kind == "panoptic":
        if cam_list is None:
            raise ValueError("panoptic calibration needs the (panel, node) camera list")
        return panoptic(calib, cam_list)
    if kind == "custom":
        return custom(calib)
    if kind == "shelf":
        return shelf(calib)
    raise ValueError(f"unknown calibration kind {kind!r}")
