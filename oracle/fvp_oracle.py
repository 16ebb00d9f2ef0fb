"""CPU oracle for the Faster-VoxelPose voxel-projection hot path (numpy, fp32).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s cpu_baseline leg as the *checker*; never by the product path
(faster-voxelpose_amd/fvp/*), which fails loudly without its HIP library.

This is an independent restatement of the reference's arithmetic, written from
the reference's semantics (file:line cited per function) and from the
behaviour of the PyTorch CPU kernels it calls, which were probed in this
container (torch 2.10.0 CPU):

* ``torch.mm`` with K = 3 accumulates as fma(a2,b2, fma(a1,b1, a0*b0))
* ``torch.linspace`` (fp32) is fma(step, i, start) below the halfway index and
  fma(-step, n-1-i, end) above it
* ``F.grid_sample`` (bilinear, zeros, align_corners=True) unnormalises with
  (g + 1) * ((size-1)/2), weights nw = (1-n)(1-w) ... and accumulates
  fma(se_val, se, fma(sw_val, sw, fma(ne_val, ne, nw_val*nw)))
* ``torch.mean(dim=0)`` is a sequential fp32 sum divided by V

fp32 FMA is emulated in float64 (exact product, one extra rounding of the
sum -- a double-rounding mismatch needs an exact float32 tie after the first
rounding, which the golden tests would show).

Parity pin: tests/test_oracle_golden.py checks every function here against
vectors produced by the reference itself (tools/gen_golden.py, which imports
/root/reference in the build container only) -> tests/golden/*.npz.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
F64 = np.float64


def fma32(a, b, c):
    """fp32 fused multiply-add, correctly rounded, emulated in float64.

    a*b of two fp32 values is exact in float64; the sum with c is taken
    exactly as hi + lo (TwoSum), and hi is rounded to fp32.  That rounding is
    wrong only when hi sits exactly on a midpoint between two fp32 values and
    lo != 0 (the double-rounding case): then the sign of lo picks the side.
    (Seen in the reference: resize_transform's 8.9e-18 off-diagonal term of
    the Panoptic affine, transforms.py:59-63, breaks the tie of
    0.47407407 * 192 -- project_grid at C5 moves by one ulp.)"""
    a, b, c = np.broadcast_arrays(np.asarray(a, F64), np.asarray(b, F64), np.asarray(c, F64))
    s = a * b
    hi = s + c
    bb = hi - s
    with np.errstate(invalid="ignore", over="ignore"):
        lo = (s - (hi - bb)) + (c - bb)
        r = hi.astype(F32)
        r64 = r.astype(F64)
        diff = hi - r64
        toward = np.where(diff > 0, F32(np.inf), F32(-np.inf)).astype(F32)
        other = np.nextafter(r, toward)
        tie = np.isfinite(hi) & np.isfinite(lo) & (diff != 0) & (hi == (r64 + other.astype(F64)) * 0.5)
        # the exact value is hi + lo: past the midpoint toward `other` when lo has diff's sign
        pick_other = tie & (lo != 0) & (np.sign(lo) == np.sign(diff))
        pick_r = tie & (lo != 0) & (np.sign(lo) != np.sign(diff))
        lower_side = np.where(pick_other, other, r)
    out = np.where(pick_r, r, lower_side).astype(F32)
    return out[()] if out.ndim == 0 else out


def linspace32(start: float, end: float, n: int) -> np.ndarray:
    """torch.linspace(start, end, n) fp32 on CPU (project_whole.py:62-64)."""
    start = F32(start)
    end = F32(end)
    if n == 1:
        return np.array([start], F32)
    step = F32((end - start) / F32(n - 1))
    i = np.arange(n)
    half = n // 2
    lo = fma32(step, i.astype(F32), start)
    hi = fma32(-step, (n - 1 - i).astype(F32), end)
    return np.where(i < half, lo, hi).astype(F32)


def compute_grid(box_size, box_center, n_bins) -> np.ndarray:
    """project_whole.py:43-79: voxel centres [N,3], z fastest ((ix*Y+iy)*Z+iz)."""
    axes = []
    for a in range(3):
        lo = F32(-float(box_size[a]) / 2)
        hi = F32(float(box_size[a]) / 2)
        axes.append(linspace32(lo, hi, int(n_bins[a])) + F32(box_center[a]))
    gx, gy, gz = np.meshgrid(axes[0], axes[1], axes[2], indexing="ij")
    return np.stack([gx.reshape(-1), gy.reshape(-1), gz.reshape(-1)], axis=1).astype(F32)


def unfold_camera(cam):
    """cameras.py:11-18 (fp32 casts)."""
    R = np.asarray(cam["R"], F64).astype(F32).reshape(3, 3)
    T = np.asarray(cam["T"], F64).astype(F32).reshape(3, 1)
    f = np.array([cam["fx"], cam["fy"]], F64).astype(F32).reshape(2, 1)
    c = np.array([cam["cx"], cam["cy"]], F64).astype(F32).reshape(2, 1)
    k = np.asarray(cam["k"], F64).astype(F32).reshape(3)
    p = np.asarray(cam["p"], F64).astype(F32).reshape(2)
    return R, T, f, c, k, p


def mm3(A: np.ndarray, X: np.ndarray) -> np.ndarray:
    """torch.mm(A[m,3], X[3,N]) fp32 CPU accumulation order."""
    out = np.empty((A.shape[0], X.shape[1]), F32)
    for r in range(A.shape[0]):
        acc = A[r, 0] * X[0]
        acc = fma32(A[r, 1], X[1], acc)
        out[r] = fma32(A[r, 2], X[2], acc)
    return out


def project_point(x: np.ndarray, cam) -> np.ndarray:
    """cameras.py:30-56 (+ :87-89): world [N,3] -> pixels [N,2], fp32."""
    R, T, f, c, k, p = unfold_camera(cam)
    xcam = mm3(R, (x.T - T).astype(F32))
    y = (xcam[:2] / (xcam[2] + F32(1e-5))).astype(F32)
    y0, y1 = y[0], y[1]
    r = (y0 * y0 + y1 * y1).astype(F32)
    d = (F32(1) + k[0] * r) + (k[1] * r) * r
    d = (d + ((k[2] * r) * r) * r).astype(F32)
    u = (y0 * d + ((F32(2) * p[0]) * y0) * y1) + p[1] * (r + (F32(2) * y0) * y0)
    v = (y1 * d + ((F32(2) * p[1]) * y0) * y1) + p[0] * (r + (F32(2) * y1) * y1)
    pix = np.stack([f[0, 0] * u + c[0, 0], f[1, 0] * v + c[1, 0]], axis=1)
    return pix.astype(F32)


def affine_pts(pts: np.ndarray, t: np.ndarray) -> np.ndarray:
    """transforms.py:59-63: [x,y,1] @ t.T via mm (fp32)."""
    t = np.asarray(t, F64).astype(F32)
    homo = np.stack([pts[:, 0], pts[:, 1], np.ones(len(pts), F32)])
    return mm3(t, homo).T.copy()


def project_grid(grid: np.ndarray, cam, ori_image_size, image_size, heatmap_size, resize_t) -> np.ndarray:
    """project_whole.py:81-117 (twin project_individual.py:151-187) -> [N,2] in [-1.1,1.1]."""
    w, h = heatmap_size
    xy = project_point(grid, cam)
    xy = np.clip(xy, F32(-1.0), F32(max(ori_image_size[0], ori_image_size[1])))
    xy = affine_pts(xy, resize_t)
    xy = (xy * np.array([w, h], F32)) / np.array(image_size, F32)
    sg = (xy / np.array([w - 1, h - 1], F32)) * F32(2.0) - F32(1.0)
    return np.clip(sg.astype(F32), F32(-1.1), F32(1.1))


def grid_sample(inp: np.ndarray, g: np.ndarray) -> np.ndarray:
    """F.grid_sample(inp[C,H,W][None], g[None,None], bilinear, zeros,
    align_corners=True)[0,:,0] -> [C,N] (ATen CPU arithmetic, see header)."""
    C, H, W = inp.shape
    ix = (g[:, 0] + F32(1)) * F32((W - 1) / 2)
    iy = (g[:, 1] + F32(1)) * F32((H - 1) / 2)
    x0 = np.floor(ix)
    y0 = np.floor(iy)
    wx = (ix - x0).astype(F32)
    ex = F32(1) - wx
    ny = (iy - y0).astype(F32)
    sy = F32(1) - ny
    nw, ne, sw, se = sy * ex, sy * wx, ny * ex, ny * wx
    xi = x0.astype(np.int64)
    yi = y0.astype(np.int64)
    out = np.empty((C, len(g)), F32)
    taps = []
    for dy, dx in ((0, 0), (0, 1), (1, 0), (1, 1)):
        xx, yy = xi + dx, yi + dy
        m = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        taps.append((m, np.where(m, yy * W + xx, 0)))
    flat = inp.reshape(C, H * W)
    for ch in range(C):
        vals = [np.where(m, flat[ch][idx], F32(0)) for m, idx in taps]
        acc = vals[0] * nw
        acc = fma32(vals[1], ne, acc)
        acc = fma32(vals[2], sw, acc)
        out[ch] = fma32(vals[3], se, acc)
    return out


def view_sum(samples) -> np.ndarray:
    """torch.sum / torch.mean over dim 0 of the [V,J,1,N] grid_sample output
    (project_whole.py:162, project_individual.py:283) on the CPU: ATen's
    cascade (SumKernel.cpp multi_row_sum, 4 levels, level step 16) -- views
    accumulate sequentially into level 0 (from zeros); every complete block of
    16 is added into level 1 and level 0 restarts (every 16 level-1 blocks go
    to level 2); the total is ((level0 + level1) + level2) + level3, so a -0
    total comes out +0.  Verified against torch.sum here for V = 1..300
    (tests/test_oracle_golden.py pins it through the C5 golden).  `samples`
    yields the V per-view arrays in view order."""
    acc = None
    i = 0
    for x in samples:
        if acc is None:
            acc = [np.zeros(x.shape, F32) for _ in range(4)]
        acc[0] = (acc[0] + x).astype(F32)
        i += 1
        if i % 16 == 0:
            for lv in (1, 2, 3):
                acc[lv] = (acc[lv] + acc[lv - 1]).astype(F32)
                acc[lv - 1] = np.zeros_like(acc[0])
                if i & (15 << (4 * lv)):
                    break
    total = acc[0]
    for lv in (1, 2, 3):
        total = (total + acc[lv]).astype(F32)
    return total


def voxelize(heatmaps: np.ndarray, sample_grid: np.ndarray) -> np.ndarray:
    """project_whole.py:119-168 for one frame: [V,J,H,W] x [V,N,2] -> cube [J,N],
    mean over all V (off-image samples count in the divisor; view_sum order)
    then clamp(0,1)."""
    V = heatmaps.shape[0]
    acc = view_sum(grid_sample(heatmaps[v], sample_grid[v]) for v in range(V))
    return np.clip((acc / F32(V)).astype(F32), F32(0), F32(1))


def xy_plane(cube: np.ndarray) -> np.ndarray:
    """cnns_2d.py:291: torch.max(cube[...,X,Y,Z], dim=-1)."""
    return cube.max(axis=-1)


def max_planes(cubes: np.ndarray) -> np.ndarray:
    """joint_localization_net.py:158-160: cat([max dim4, max dim3, max dim2])."""
    return np.concatenate([cubes.max(axis=4), cubes.max(axis=3), cubes.max(axis=2)], axis=0)


def nms2d(prob: np.ndarray, K: int):
    """proposal.py:34-76 for prob [B,1,X,Y]: 3x3/s1/p1 peak mask, flattened
    top-K (NaN first, then value desc, flat index asc on ties), then get_index2D with the
    reference's divisor shape[1] == X (proposal.py:27-29,75)."""
    B, _, X, Y = prob.shape
    p = prob[:, 0]
    pad = np.full((B, X + 2, Y + 2), -np.inf, F32)
    pad[:, 1:-1, 1:-1] = p
    mx = np.full((B, X, Y), -np.inf, F32)
    for dx in range(3):
        for dy in range(3):
            mx = np.maximum(mx, pad[:, dx:dx + X, dy:dy + Y])
    keep = (p == mx).astype(F32)
    nmsv = (keep * p).reshape(B, -1)
    vals = np.empty((B, K), F32)
    idx = np.empty((B, K), np.int64)
    for b in range(B):
        isn = np.isnan(nmsv[b])  # torch.topk ranks NaN above every number
        order = np.lexsort((np.arange(X * Y), -np.where(isn, 0, nmsv[b]), ~isn))[:K]
        idx[b] = order
        vals[b] = nmsv[b][order]
    xy = np.stack([idx // X, idx % X], axis=2)
    return vals, xy, idx


def gather_columns(cube: np.ndarray, flat: np.ndarray) -> np.ndarray:
    """human_detection_net.py:199-200: [B,J,X,Y,Z] x flat [B,K] -> [B,K,J,Z]."""
    B, J, X, Y, Z = cube.shape
    c = cube.reshape(B, J, X * Y, Z)
    return np.stack([c[b][:, flat[b], :].transpose(1, 0, 2) for b in range(B)])


def gather_bbox(size: np.ndarray, flat: np.ndarray) -> np.ndarray:
    """human_detection_net.py:191-192: size [B,2,X,Y] -> [B,K,2]."""
    B = size.shape[0]
    s = size.reshape(B, 2, -1)
    return np.stack([s[b][:, flat[b]].T for b in range(B)])


def proposal_mm(idx3: np.ndarray, space_size, space_center, bins) -> np.ndarray:
    """human_detection_net.py:36-37,101: voxel index -> mm."""
    import torch  # same fp32 ops as the reference's tensors

    scale = torch.tensor(list(space_size)) / (torch.tensor(list(bins)) - 1)
    bias = torch.tensor(list(space_center)) - torch.tensor(list(space_size)) / 2.0
    return (torch.from_numpy(idx3).float() * scale + bias).numpy()


# ---------------------------------------------------------------------------
# per-person layer (project_individual.py)
# ---------------------------------------------------------------------------

class Individual:
    """project_individual.py:29-111: constants, fine grid and centre grid."""

    def __init__(self, whole_size, whole_center, ind_size, ind_bins):
        import torch

        self.wc = torch.tensor(list(map(float, whole_center)))
        self.ws = torch.tensor(list(map(float, whole_size)))
        self.isz = torch.tensor(list(map(float, ind_size)))
        self.vpa = torch.tensor(list(map(int, ind_bins)), dtype=torch.int32)
        self.fine = (self.ws / self.isz * (self.vpa - 1)).int() + 1
        self.scale = (self.fine.float() - 1) / self.ws
        self.bias = -self.isz / 2.0 / self.ws * (self.fine - 1) - self.scale * (self.wc - self.ws / 2.0)
        g = compute_grid(self.isz.numpy(), self.wc.numpy(), self.vpa.numpy()).reshape(*self.vpa.tolist(), 3)
        self.center_grid = np.stack([g[:, :, 0, :2].reshape(-1, 2), g[:, 0, :, ::2].reshape(-1, 2),
                                     g[0, :, :, 1:].reshape(-1, 2)])
        self.fine_bins = self.fine.numpy().astype(np.int64)

    def fine_grid(self) -> np.ndarray:
        return compute_grid(self.ws.numpy(), self.wc.numpy(), self.fine_bins)

    def windows(self, proposals: np.ndarray):
        """project_individual.py:255-269 -> (centers_tl, offset, start, end) as numpy."""
        import torch

        pc = torch.from_numpy(np.ascontiguousarray(proposals, F32))
        ctl = torch.round(pc[:, :3].float() * self.scale + self.bias).int()
        offset = ctl.float() / (self.fine - 1) * self.ws - self.ws / 2.0 + self.isz / 2.0
        mask = ((1 - pc[:, 5:7]) / 2 * (self.vpa[0:2] - 1)).int()
        mask[mask < 0] = 0
        mask = torch.cat([mask, torch.zeros((pc.shape[0], 1), dtype=torch.int32)], dim=1)
        start = torch.where(ctl + mask >= 0, ctl + mask, torch.zeros_like(ctl))
        end = torch.where(ctl + self.vpa - mask <= self.fine, ctl + self.vpa - mask, self.fine)
        return ctl.numpy(), offset.numpy(), start.numpy(), end.numpy()

    def person_cubes(self, heatmaps: np.ndarray, fine_sample_grid: np.ndarray, proposals: np.ndarray):
        """project_individual.py:222-293 for one frame's heatmaps [V,J,H,W] and
        its fine sample grid [V,FX,FY,FZ,2] -> (cubes [P,J,sx,sy,sz], offset [P,3])."""
        V, J = heatmaps.shape[:2]
        sx, sy, sz = self.vpa.tolist()
        ctl, offset, start, end = self.windows(proposals)
        cubes = np.zeros((len(proposals), J, sx, sy, sz), F32)
        for i in range(len(proposals)):
            s, e = start[i], end[i]
            if np.any(s >= e):
                continue
            win = fine_sample_grid[:, s[0]:e[0], s[1]:e[1], s[2]:e[2]].reshape(V, -1, 2)
            acc = view_sum(grid_sample(heatmaps[v], win[v]) for v in range(V))
            acc = (acc / F32(V)).reshape(J, *(e - s))
            o0, o1 = s - ctl[i], e - ctl[i]
            cubes[i, :, o0[0]:o1[0], o0[1]:o1[1], o0[2]:o1[2]] = acc
        return np.clip(cubes, F32(0), F32(1)), offset


# ---------------------------------------------------------------------------
# JLN post-processing.  Computed in float64: the
# reference's fp32 softmax / 4096-term sums are matched within a tolerance,
# not bit-for-bit (tests/test_jln_post.py states it).
def soft_argmax(features: np.ndarray, center_grid: np.ndarray, beta: float):
    """SoftArgmaxLayer.forward (joint_localization_net.py:32-56):
    features [3,P,J,S,S] -> (coords [3,P,J,2], confs [P])."""
    x = features.reshape(features.shape[0], features.shape[1], features.shape[2], -1).astype(np.float64)
    y = np.float32(beta) * x
    e = np.exp(y - y.max(axis=3, keepdims=True))
    p = e / e.sum(axis=3, keepdims=True)
    confs = p.max(axis=3).mean(axis=(0, 2))
    g = center_grid.reshape(3, 1, 1, -1, 2).astype(np.float64)
    coords = (p[..., None] * g).sum(axis=3)
    return coords, confs


def add_offsets(coords: np.ndarray, offset: np.ndarray) -> np.ndarray:
    """joint_localization_net.py:170-174: xy += (x,y), xz += (x,z), yz += (y,z)."""
    o = offset.reshape(-1, 1, 3).astype(np.float64)
    out = coords.copy()
    out[0] += o[:, :, :2]
    out[1] += o[:, :, ::2]
    out[2] += o[:, :, 1:]
    return out


def fuse_pose_preds(pose: np.ndarray, weights: np.ndarray) -> np.ndarray:
    """JointLocalizationNet.fuse_pose_preds (joint_localization_net.py:83-120):
    pose [3,P,J,2], weights [3P,J,1] -> [P,J,3]."""
    P = pose.shape[1]
    w = weights.astype(np.float64).reshape(3, P, -1, 1)
    xy_w, xz_w, yz_w = w[0], w[1], w[2]
    xy, xz, yz = pose[0], pose[1], pose[2]
    xw = np.concatenate([xy_w, xz_w], 2)
    yw = np.concatenate([xy_w, yz_w], 2)
    zw = np.concatenate([xz_w, yz_w], 2)
    xw = xw / xw.sum(2, keepdims=True)
    yw = yw / yw.sum(2, keepdims=True)
    zw = zw / zw.sum(2, keepdims=True)
    x = xw[:, :, :1] * xy[:, :, :1] + xw[:, :, 1:] * xz[:, :, :1]
    y = yw[:, :, :1] * xy[:, :, 1:] + yw[:, :, 1:] * yz[:, :, :1]
    z = zw[:, :, :1] * xz[:, :, 1:] + zw[:, :, 1:] * yz[:, :, 1:]
    return np.concatenate([x, y, z], axis=2)


CUBE_SLABS = 8  # per-x-slab digests localise a mismatch


def cube_digests(cube: np.ndarray, slabs: int = CUBE_SLABS) -> np.ndarray:
    """SHA-256 pins of whole fp32 cubes [B,J,X,Y,Z] (project_whole.py:166-167's
    output layout): per frame, the digest of the frame's little-endian fp32
    bytes (C order, so -0.0 vs +0.0 and NaN payloads count) followed by one
    digest per x-slab (``slabs`` contiguous runs of x-rows, [J, x0:x1, Y, Z]).
    Returns uint8 [B, 1 + slabs, 32]."""
    import hashlib

    cube = np.ascontiguousarray(cube, dtype="<f4")
    B, X = cube.shape[0], cube.shape[2]
    bounds = np.linspace(0, X, slabs + 1).round().astype(int)
    out = np.zeros((B, 1 + slabs, 32), np.uint8)
    for b in range(B):
        out[b, 0] = np.frombuffer(hashlib.sha256(cube[b].tobytes()).digest(), np.uint8)
        for s in range(slabs):
            part = np.ascontiguousarray(cube[b, :, bounds[s]:bounds[s + 1]])
            out[b, 1 + s] = np.frombuffer(hashlib.sha256(part.tobytes()).digest(), np.uint8)
    return out
