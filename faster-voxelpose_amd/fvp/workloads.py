"""Named workloads (BASELINE.json ``configs``) and their camera sets.

A workload fixes the capture geometry (calibration, image sizes, capture
space, voxel counts) and the heatmap shape.  The geometry of each one follows
the reference configs it is named after:

* shelf  : configs/shelf/jln64.yaml:22-27,71-85 + data/Shelf/calibration_shelf.json
* panoptic: configs/panoptic/jln64.yaml:22-30,62-76 + demo/calibration.json
* ring31 : 31 generated Panoptic-like cameras on a 4.5 m ring

The heatmap shape is BASELINE.json's (J=15, 128x240) for every measurement
workload; ``shelf_native`` keeps Shelf's own J=17, 152x200.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field

import numpy as np

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GOLDEN_DIR = os.path.join(REPO_ROOT, "tests", "golden")


def load_calibration(name: str):
    """Load a committed calibration fixture as the reference's ``cameras``
    dict: {seq: {int: cam}} with numpy arrays (shelf.py:138-153) or
    {seq: [cam, ...]} (panoptic.py:171-205 / demo notebook)."""
    path = os.path.join(GOLDEN_DIR, name)
    with open(path) as f:
        raw = json.load(f)
    if "customized_sequence" in raw:  # demo/calibration.json: {seq: [cam...]}
        seq = "customized_sequence"
        cams = [{k: np.array(v) for k, v in c.items()} for c in raw[seq]]
        return {seq: cams}, seq
    cams = {int(i): {k: np.array(v) for k, v in c.items()} for i, c in raw.items()}
    seq = os.path.splitext(name)[0].replace("calibration_", "")
    return {seq: cams}, seq


def ring_cameras(n: int = 31, radius: float = 4500.0, center=(0.0, -500.0, 800.0)):
    """C5 camera ring: looking at ``center`` from a circle of ``radius`` mm,
    heights 1.5/2.45/3.4 m cycling; intrinsics + distortion cycled from the 5
    demo Panoptic cameras."""
    demo, seq = load_calibration("calibration_panoptic_demo.json")
    base = demo[seq]
    heights = [1500.0, 2450.0, 3400.0]
    cams = []
    c = np.array(center, dtype=np.float64)
    for i in range(n):
        ang = 2.0 * math.pi * i / n
        pos = np.array([c[0] + radius * math.cos(ang), c[1] + radius * math.sin(ang), heights[i % 3]])
        fwd = c - pos
        fwd /= np.linalg.norm(fwd)
        up = np.array([0.0, 0.0, 1.0])
        right = np.cross(fwd, up)
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        R = np.stack([right, down, fwd])  # world -> camera; camera z looks at centre
        src = base[i % len(base)]
        cams.append({
            "R": R, "T": pos.reshape(3, 1),
            "fx": float(src["fx"]), "fy": float(src["fy"]),
            "cx": float(src["cx"]), "cy": float(src["cy"]),
            "k": np.array(src["k"]).reshape(3, 1), "p": np.array(src["p"]).reshape(2, 1),
        })
    return {"ring31": cams}, "ring31"


@dataclass
class Workload:
    name: str
    calibration: str           # fixture file name or "ring31"
    ori_image_size: tuple      # (W, H)
    image_size: tuple          # (W, H)
    heatmap_size: tuple        # (W, H)
    num_joints: int
    space_size: tuple
    space_center: tuple
    voxels_per_axis: tuple
    batch: int = 1
    max_people: int = 10
    min_score: float = 0.3
    dtype: str = "float32"
    ind_space_size: tuple = (2000.0, 2000.0, 2000.0)
    ind_voxels_per_axis: tuple = (64, 64, 64)
    extra: dict = field(default_factory=dict)

    def cameras(self):
        if self.calibration == "ring31":
            cams, seq = ring_cameras()
        else:
            cams, seq = load_calibration(self.calibration)
        views = self.extra.get("views")
        if views is not None:
            cams = {seq: [cams[seq][c] for c in range(views)]}
        return cams, seq

    @property
    def num_views(self) -> int:
        return len(self.cameras()[0][self.cameras()[1]])

    @property
    def num_voxels(self) -> int:
        x, y, z = self.voxels_per_axis
        return x * y * z

    def cfg(self, device: str = "cuda:0"):
        from .config import make_cfg
        return make_cfg(self, device=device)


PANOPTIC_SPACE = dict(space_size=(8000.0, 8000.0, 2000.0), space_center=(0.0, -500.0, 800.0))
SHELF_SPACE = dict(space_size=(8000.0, 8000.0, 2000.0), space_center=(450.0, -320.0, 800.0))

WORKLOADS = {
    # C1: configs[0] -- 1 camera, 20x20x8, the CPU-runnable plumbing case
    "c1": Workload("c1", "calibration_panoptic_demo.json", (1920, 1080), (960, 512), (240, 128), 15,
                   voxels_per_axis=(20, 20, 8), batch=1, extra={"views": 1}, **PANOPTIC_SPACE),
    # C2: configs[1] -- Shelf geometry, BASELINE shapes, the metric's workload
    "c2": Workload("c2", "calibration_shelf.json", (1032, 776), (800, 608), (240, 128), 15,
                   voxels_per_axis=(80, 80, 20), batch=1, min_score=0.1, **SHELF_SPACE),
    # C3: configs[2] -- Panoptic demo cameras, batch 8 (TEST.BATCH_SIZE)
    "c3": Workload("c3", "calibration_panoptic_demo.json", (1920, 1080), (960, 512), (240, 128), 15,
                   voxels_per_axis=(80, 80, 20), batch=8, **PANOPTIC_SPACE),
    # C4: configs[3] -- 128x128x32 grid, 10 proposals
    "c4": Workload("c4", "calibration_panoptic_demo.json", (1920, 1080), (960, 512), (240, 128), 15,
                   voxels_per_axis=(128, 128, 32), batch=1, **PANOPTIC_SPACE),
    # C5: configs[4] -- 31 ring cameras, 160x160x64, fp16 heatmaps
    "c5": Workload("c5", "ring31", (1920, 1080), (960, 512), (240, 128), 15,
                   voxels_per_axis=(160, 160, 64), batch=1, dtype="float16", **PANOPTIC_SPACE),
    # Shelf at its native shapes (configs/shelf/jln64.yaml:28-31): J=17, 152x200
    "shelf_native": Workload("shelf_native", "calibration_shelf.json", (1032, 776), (800, 608), (200, 152), 17,
                             voxels_per_axis=(80, 80, 20), batch=1, min_score=0.1, **SHELF_SPACE),
}
