"""Deterministic synthetic inputs for parity tests and the benchmark.

The reference synthesises input heatmaps on the CPU from 2-D joint positions
(lib/dataset/JointsDataset.py:368-447: a Gaussian of sigma = NETWORK.SIGMA
per joint, max over people, clipped to [0, 1]).  This module does the same
for skeletons placed at random in the capture space and projected through
the workload's cameras, so every view sees consistent peaks and the proposal
argmax is tie-free.  Augmentation is off (as at test time).

* ``skeletons(w, b)``           -- people of frame ``b`` (seeded by 1000 + b)
* ``gaussian_heatmaps(w, B)``   -- float32 [B, V, J, H, W]
* ``uniform_heatmaps(w, B, s)`` -- torch.rand stress input [B, V, J, H, W]
"""
from __future__ import annotations

import numpy as np

from . import geometry

# 15-joint template in mm relative to the root (mid-hip), Panoptic joint order
# (lib/dataset/panoptic.py:42-58): neck, nose, mid-hip, l-shoulder, l-elbow,
# l-wrist, l-hip, l-knee, l-ankle, r-shoulder, r-elbow, r-wrist, r-hip,
# r-knee, r-ankle.  x = left/right, y = front, z = up.
TEMPLATE15 = np.array([
    [0, 0, 550], [0, 70, 720], [0, 0, 0],
    [-180, 0, 500], [-260, 10, 240], [-290, 60, 10],
    [-100, 0, 0], [-110, 30, -440], [-110, 0, -840],
    [180, 0, 500], [260, 10, 240], [290, 60, 10],
    [100, 0, 0], [110, 30, -440], [110, 0, -840],
], dtype=np.float64)

ROOT_HEIGHT = 900.0
SIGMA = 3.0  # NETWORK.SIGMA (configs/panoptic/jln64.yaml:38)


def joint_template(num_joints: int) -> np.ndarray:
    if num_joints <= 15:
        return TEMPLATE15[:num_joints]
    extra = [TEMPLATE15[i % 15] + np.array([35.0 * (1 + i // 15), -25.0, 40.0]) for i in range(num_joints - 15)]
    return np.concatenate([TEMPLATE15, np.array(extra)], axis=0)


def skeletons(w, frame: int, people: int = 4) -> np.ndarray:
    """[people, J, 3] world joint positions (mm) for frame ``frame``."""
    rng = np.random.default_rng(1000 + frame)
    tpl = joint_template(w.num_joints)
    out = np.zeros((people, w.num_joints, 3))
    for p in range(people):
        cx = w.space_center[0] + rng.uniform(-0.5, 0.5) * (w.space_size[0] - 1200.0)
        cy = w.space_center[1] + rng.uniform(-0.5, 0.5) * (w.space_size[1] - 1200.0)
        yaw = rng.uniform(0.0, 2.0 * np.pi)
        c, s = np.cos(yaw), np.sin(yaw)
        rot = np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])
        out[p] = tpl @ rot.T + np.array([cx, cy, ROOT_HEIGHT])
    return out


def project_cpu(x: np.ndarray, cam) -> tuple[np.ndarray, np.ndarray]:
    """float64 pinhole + distortion (cameras.py:58-84) -> (pixels [N,2], depth [N])."""
    R = np.asarray(cam["R"], dtype=np.float64)
    T = np.asarray(cam["T"], dtype=np.float64).reshape(3, 1)
    k = np.asarray(cam["k"], dtype=np.float64).reshape(3)
    p = np.asarray(cam["p"], dtype=np.float64).reshape(2)
    xcam = R @ (x.T - T)
    y = xcam[:2] / (xcam[2] + 1e-5)
    r = np.sum(y ** 2, axis=0)
    d = 1 + k[0] * r + k[1] * r * r + k[2] * r * r * r
    u = y[0] * d + 2 * p[0] * y[0] * y[1] + p[1] * (r + 2 * y[0] * y[0])
    v = y[1] * d + 2 * p[1] * y[0] * y[1] + p[0] * (r + 2 * y[1] * y[1])
    pix = np.stack([cam["fx"] * u + cam["cx"], cam["fy"] * v + cam["cy"]], axis=1)
    return pix, xcam[2]


def joint_pixels(w, frame: int, people: int = 4):
    """Heatmap-pixel coordinates [V, people, J, 2] and visibility [V, people, J]."""
    cams, seq = w.cameras()
    cam_list = geometry.camera_list(cams, seq)
    trans = geometry.resize_transform(w.ori_image_size, w.image_size)
    sk = skeletons(w, frame, people).reshape(-1, 3)
    hw, hh = w.heatmap_size
    iw, ih = w.image_size
    pix_all, vis_all = [], []
    for cam in cam_list:
        pix, depth = project_cpu(sk, cam)
        homo = np.concatenate([pix, np.ones((pix.shape[0], 1))], axis=1)
        img = homo @ trans.T
        hm = img * np.array([hw / iw, hh / ih])
        pix_all.append(hm.reshape(people, w.num_joints, 2))
        vis_all.append((depth > 100.0).reshape(people, w.num_joints))
    return np.stack(pix_all), np.stack(vis_all)


def render_frame(w, frame: int, out: np.ndarray, people: int = 4, sigma: float = SIGMA) -> None:
    """Render one frame's [V, J, H, W] float32 heatmaps into ``out``."""
    pix, vis = joint_pixels(w, frame, people)
    hw, hh = w.heatmap_size
    rad = int(np.ceil(3 * sigma))
    out[...] = 0.0
    V, P, J = vis.shape
    for v in range(V):
        for p in range(P):
            for j in range(J):
                if not vis[v, p, j]:
                    continue
                mx, my = pix[v, p, j]
                if not (-rad <= mx < hw + rad and -rad <= my < hh + rad):
                    continue
                x0, x1 = max(0, int(np.floor(mx)) - rad), min(hw, int(np.floor(mx)) + rad + 1)
                y0, y1 = max(0, int(np.floor(my)) - rad), min(hh, int(np.floor(my)) + rad + 1)
                if x0 >= x1 or y0 >= y1:
                    continue
                xs = np.arange(x0, x1, dtype=np.float64)[None, :]
                ys = np.arange(y0, y1, dtype=np.float64)[:, None]
                g = np.exp(-((xs - mx) ** 2 + (ys - my) ** 2) / (2 * sigma * sigma)).astype(np.float32)
                win = out[v, j, y0:y1, x0:x1]
                np.maximum(win, g, out=win)
    np.clip(out, 0.0, 1.0, out=out)


def gaussian_heatmaps(w, batch: int, first_frame: int = 0, people: int = 4, views: int | None = None) -> np.ndarray:
    cams, seq = w.cameras()
    V = len(cams[seq]) if views is None else views
    hw, hh = w.heatmap_size
    out = np.zeros((batch, V, w.num_joints, hh, hw), dtype=np.float32)
    for b in range(batch):
        render_frame(w, first_frame + b, out[b], people)
    return out


def uniform_heatmaps(w, batch: int, seed: int = 0):
    import torch

    cams, seq = w.cameras()
    V = len(cams[seq])
    hw, hh = w.heatmap_size
    g = torch.Generator().manual_seed(seed)
    return torch.rand((batch, V, w.num_joints, hh, hw), generator=g)


def proposals_for_frame(w, frame: int, people: int = 4, bbox=(0.45, 0.55)) -> np.ndarray:
    """JLN-style proposal_centers rows [people, 7] (human_detection_net.py:99-124):
    (x, y, z mm, matched-gt, conf, bbox_w, bbox_h) at the synthetic roots."""
    sk = skeletons(w, frame, people)
    root = sk[:, 2, :] if w.num_joints > 2 else sk[:, 0, :]
    out = np.zeros((people, 7), dtype=np.float32)
    out[:, 0:3] = root
    out[:, 3] = 0.0
    out[:, 4] = 0.9
    out[:, 5] = bbox[0]
    out[:, 6] = bbox[1]
    return out


def jln_batch_proposals(w, frame: int, rng: np.random.Generator, n_extra: int) -> np.ndarray:
    """A frame's JLN proposals [4 + n_extra, 7]: the 4 synthetic people plus n_extra
    random centres over the whole space with bbox sizes in [-0.2, 1.2] -- windows
    clipped at either end, skipped (start >= end) and with negative margins
    (project_individual.py:251-263)."""
    base = proposals_for_frame(w, frame, 4)
    extra = np.zeros((n_extra, 7), np.float32)
    extra[:, 0] = rng.uniform(-4600, 4600, n_extra)
    extra[:, 1] = -500 + rng.uniform(-4600, 4600, n_extra)
    extra[:, 2] = rng.uniform(200, 1500, n_extra)
    extra[:, 5:7] = rng.uniform(-0.2, 1.2, (n_extra, 2))
    return np.concatenate([base, extra])


def joint_features(P: int, J: int, S: int = 64, seed: int = 0) -> np.ndarray:
    """Stand-in P2PNet output [3, P, J, S, S] (fp32): one Gaussian peak (height
    0.15, sigma 3 cells) per (plane, proposal, joint) on N(0, 0.02) noise, so that
    softmax(100 x) is peaked like a trained network's maps.  numpy RNG only, so
    the test and the golden generator rebuild identical inputs."""
    rng = np.random.default_rng(seed)
    f = rng.normal(0.0, 0.02, (3, P, J, S, S)).astype(np.float32)
    c = rng.uniform(8.0, S - 8.0, (3, P, J, 2))
    yy, xx = np.mgrid[0:S, 0:S].astype(np.float64)
    d2 = (xx[None, None, None] - c[..., 0, None, None]) ** 2 + (yy[None, None, None] - c[..., 1, None, None]) ** 2
    f += (0.15 * np.exp(-d2 / (2 * 3.0 ** 2))).astype(np.float32)
    return f


def jln_weights(P: int, J: int, seed: int = 0) -> np.ndarray:
    """Stand-in WeightNet output [3P, J, 1] in (0.05, 0.95) (a sigmoid's range)."""
    return np.random.default_rng(seed + 1).uniform(0.05, 0.95, (3 * P, J, 1)).astype(np.float32)


def jln_offsets(P: int, seed: int = 0) -> np.ndarray:
    """Per-proposal cube offsets [P, 3] in mm."""
    return np.random.default_rng(seed + 2).uniform(-3000.0, 3000.0, (P, 3)).astype(np.float32)


def seeded_state_dict(module, seed: int = 0) -> dict:
    """Deterministic weights for any module, keyed by parameter name (zlib.crc32),
    so the reference's classes and a restatement with the same attribute names
    get identical tensors: conv/linear weights N(0, sqrt(2/fan_in)), biases
    N(0, 0.05), BatchNorm gamma U(0.5, 1.5), beta N(0, 0.1), running mean
    N(0, 0.1), running var U(0.5, 1.5).  (The checkpoints are not available
    offline)"""
    import zlib

    import torch

    out = {}
    for name, t in module.state_dict().items():
        rng = np.random.default_rng((seed * 1000003 + zlib.crc32(name.encode())) & 0xFFFFFFFF)
        shape = tuple(t.shape)
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "num_batches_tracked":
            out[name] = t.clone()
            continue
        if leaf == "weight" and len(shape) > 1:
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
            v = rng.normal(0.0, np.sqrt(2.0 / fan_in), shape)
        elif leaf == "weight":      # BatchNorm gamma
            v = rng.uniform(0.5, 1.5, shape)
        elif leaf == "bias":
            v = rng.normal(0.0, 0.05, shape)
        elif leaf == "running_mean":
            v = rng.normal(0.0, 0.1, shape)
        elif leaf == "running_var":
            v = rng.uniform(0.5, 1.5, shape)
        else:
            v = rng.normal(0.0, 0.1, shape)
        out[name] = torch.from_numpy(v.astype(np.float32))
    return out
