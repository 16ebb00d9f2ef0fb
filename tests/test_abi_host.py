"""CPU tests: the C-ABI library loads and exports what include/fvp.h declares,
argument validation happens before any launch, and the host-side mirror of
the reference interface (geometry, config, layer construction) is correct."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO
from fvp import geometry, synthetic
from fvp.workloads import WORKLOADS

HEADER = os.path.join(REPO, "include", "fvp.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(fvp_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from fvp import _lib

    lib = _lib.load()
    names = _declared()
    assert len(names) >= 9
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SIGNATURES), "ctypes table out of sync with include/fvp.h"
    assert lib.fvp_abi_version() == _lib.ABI_VERSION == 22
    assert lib.fvp_status_string(0) == b"success"


def test_argument_validation_without_gpu():
    """NULL / bad sizes are rejected on the host, before any HIP call."""
    from fvp import _lib

    lib = _lib.load()
    assert lib.fvp_voxelize(None, 1, 5, 15, 128, 240, None, None, 80, 80, 20, None, None, None, 0, None) == 1001
    assert lib.fvp_voxelize(1, 0, 5, 15, 128, 240, 1, None, 80, 80, 20, 1, None, None, 0, None) == 1002
    assert lib.fvp_voxelize(1, 1, 5, 1025, 128, 240, 1, None, 80, 80, 20, 1, None, None, 0, None) == 1002  # J > 1024
    assert lib.fvp_voxelize(1, 1, 5, 15, 128, 240, 1, None, 80, 80, 20, 1, None, None, 0, None) == 1003  # no workspace
    need = lib.fvp_voxelize_workspace_bytes(256, 5, 15, 128, 240)
    assert need == 12 * 5 * 128 * 240 * 16 * 4  # channels-last chunk of 12 frames (J padded to 16)
    assert lib.fvp_voxelize(1, 1, 5, 15, 128, 240, 1, None, 80, 80, 20, 1, None, 1, 100, None) == 1003
    assert lib.fvp_voxelize_workspace_bytes(4, 5, 40, 128, 240) == 4 * 5 * 128 * 240 * 32 * 4  # one 32-joint slice
    assert lib.fvp_voxelize_workspace_bytes(4, 5, 1025, 128, 240) == 0
    # fp16, J <= 16: pixel-pair table [V][H][W+1] x 64 B, one group of 4 C5 frames per chunk
    # (the size depends on the arguments only: no process environment is read)
    assert lib.fvp_voxelize_f16_workspace_bytes(8, 31, 15, 128, 240) == 4 * 31 * 128 * 241 * 64
    os.environ["FVP_PAIR_FRAMES"] = "2"  # the round-3 A/B knob: gone
    try:
        assert lib.fvp_voxelize_f16_workspace_bytes(8, 31, 15, 128, 240) == 4 * 31 * 128 * 241 * 64
    finally:
        del os.environ["FVP_PAIR_FRAMES"]
    # fp16, J > 16: the fp32 channels-last copy
    assert lib.fvp_voxelize_f16_workspace_bytes(1, 5, 17, 128, 240) == 5 * 128 * 240 * 32 * 4
    assert lib.fvp_pack_grid(None, 5, 100, None, None) == 1001
    assert lib.fvp_pack_grid(1, 0, 100, 1, None) == 1002
    # packed grid of one sequence beyond 32-bit byte offsets
    assert lib.fvp_voxelize(1, 1, 32, 15, 128, 240, 1, None, 1024, 1024, 512, 1, None, 1, 1 << 40, None) == 1002
    assert lib.fvp_nms_topk(None, 1, 80, 80, 0, 10, None, None, None, None) == 1001
    assert lib.fvp_nms_topk(1, 1, 2, 2, 0, 10, 1, 1, None, None) == 1002  # K > X*Y
    assert lib.fvp_nms_topk(1, 2, 8, 8, 10, 5, 1, 1, None, None) == 1002  # frame stride < X*Y
    assert lib.fvp_max_planes(1, 1, 1, 4097, 1, None) == 1002          # S > 4096
    spec = _lib.PersonSpec((253, 253, 64), (0.03, 0.03, 0.03), (0, 0, 0), (8000, 8000, 2000), (2000,) * 3, (64,) * 3)
    assert lib.fvp_person_planes(None, 1, 5, 15, 128, 240, 1, spec, 1, None, 1, None, 1, None, 1, 10, None) == 1001
    assert lib.fvp_person_planes(1, 1, 5, 15, 128, 240, 1, spec, 1, None, 1, None, 1, None, None, 0, None) == 1003
    assert lib.fvp_person_workspace_bytes(2, 5, 15, 128, 240) == 2 * 5 * 128 * 240 * 16 * 4
    bad = _lib.PersonSpec((253, 253, 64), (0.03,) * 3, (0,) * 3, (8000,) * 3, (2000,) * 3, (64, 64, 32))
    assert lib.fvp_person_planes(1, 1, 5, 15, 128, 240, 1, bad, 1, None, 1, None, 1, None, 1, 1 << 30, None) == 1002
    assert lib.fvp_gather_columns(None, 1, 1, 1, 1, 1, None, 1, None, None) == 1001
    vc = lib.fvp_voxel_columns  # (hm, half, strides x3, B, V, J, H, W, grids, cams, rt, grid, img, gi, X, Y, Z, flat, K, cols)
    assert vc(None, 0, 1, 1, 1, 1, 5, 15, 128, 240, 1, None, None, None, None, None, 80, 80, 20, 1, 10, 1, None) == 1001
    assert vc(1, 0, 1, 1, 1, 1, 0, 15, 128, 240, 1, None, None, None, None, None, 80, 80, 20, 1, 10, 1, None) == 1002
    assert vc(1, 0, 1, 1, 1, 1, 5, 15, 128, 240, None, None, None, None, None, None, 80, 80, 20, 1, 10, 1, None) == 1001
    # split-K scratch: CenterNet's 20x20 128->128 level at 8 frames (200 blocks, 72 K-chunks -> 3-way)
    assert lib.fvp_conv2d_workspace_bytes(8, 20, 20, 128, 3, 3, 128, 0, 0) == 3 * 3200 * 128 * 4
    assert lib.fvp_conv2d_workspace_bytes(120, 64, 64, 32, 3, 3, 32, 0, 0) == 0  # enough blocks: no split
    assert lib.fvp_conv2d_workspace_bytes(8, 20, 20, 16, 1, 1, 16, 0, 0) == 0    # short K walk: no split
    assert lib.fvp_weight_net(1, 10, 64, 64, 1, 1, 1, 32, 1, 1, 64, 1, None, 1, None) == 1001
    assert lib.fvp_weight_net(1, 10, 64, 64, 1, 1, 1, 65, 1, 1, 64, 1, 1, 1, None) == 1002   # C > 64
    assert lib.fvp_weight_net(1, 10, 200, 200, 1, 1, 1, 32, 1, 1, 64, 1, 1, 1, None) == 1002  # map beyond LDS
    assert lib.fvp_weight_net(None, 0, 64, 64, None, None, None, 32, None, None, 64, None, None, None, None) == 0
    assert lib.fvp_maxpool_nhwc(1, 1, 1, 20, 16, 2, 2, 1, None) == 1002  # H < KH
    assert lib.fvp_maxpool_nhwc(1, 1, 1, 20, 16, 1, 3, 1, None) == 1002
    assert lib.fvp_conv2d_nhwc(1, 1, 1, 8, 16, 1, 1, 1, 16, 128, 1, 1, None, None, 0, 3, 1, None) == 1002  # upsample2
    with pytest.raises(_lib.FvpError, match="NULL"):
        _lib.check(1001, "fvp_voxelize")


@pytest.mark.parametrize("shape, want", [
    ((240, 64, 64, 64), (4, 8, 2, 1, 7680, 1000)),   # P2PNet 64 px: exact 8 x 16 px tiles, 64 columns a block
    ((240, 64, 64, 32), (4, 8, 1, 1, 7680, 1000)),   # 32 output channels: NB = 1
    ((240, 16, 16, 128), (4, 8, 2, 1, 960, 1000)),   # >= 512 blocks at NB = 2
    ((8, 80, 80, 32), (4, 8, 1, 1, 400, 1000)),      # CenterNet 80 px: > 256 blocks, 4-wave blocks
    ((8, 40, 40, 64), (3, 10, 1, 2, 224, 1120)),     # 20 x 20 tiles: 3 x 10 grids (7 x 2 per image)
    ((8, 20, 20, 128), (5, 5, 1, 2, 128, 1280)),     # 10 x 10 tiles: 5 x 5 grids, 25 of 32 slots
    ((40, 16, 30, 512), (4, 8, 2, 1, 1280, 1066)),   # ResNet-50 stage 4: 8 x 15 tiles
])
def test_wino_plan(shape, want):
    """fvp_conv3x3_wino_plan (host only): tile grid, NB, XS, blocks, slot coverage."""
    from fvp import cnn

    assert cnn.wino_plan(*shape) == want


def test_ops_refuse_cpu_tensors():
    from fvp import ops  # noqa: F401  (registers torch.ops.fvp.*)

    hm = torch.zeros(1, 1, 1, 4, 4)
    sg = torch.zeros(1, 8, 2)
    with pytest.raises(Exception):
        torch.ops.fvp.voxelize(hm, sg, None, 2, 2, 2, True, True)


def test_pack_camera_layout():
    cams, seq = WORKLOADS["c3"].cameras()
    c = cams[seq][0]
    rec = geometry.pack_camera(c)
    assert rec.shape == (geometry.CAM_STRIDE,) and rec.dtype == np.float32
    assert np.array_equal(rec[0:9], np.asarray(c["R"], np.float64).astype(np.float32).reshape(9))
    assert np.array_equal(rec[9:12], np.asarray(c["T"], np.float64).astype(np.float32).reshape(3))
    assert rec[12] == np.float32(c["fx"]) and rec[15] == np.float32(c["cy"])
    assert np.array_equal(rec[16:19], np.asarray(c["k"]).astype(np.float32).reshape(3))
    assert np.array_equal(rec[19:21], np.asarray(c["p"]).astype(np.float32).reshape(2))
    # dict-of-int (shelf) and list (panoptic) camera containers
    shelf, s2 = WORKLOADS["c2"].cameras()
    assert geometry.pack_cameras(shelf, s2).shape == (5, geometry.CAM_STRIDE)


def test_resize_transform_closed_forms():
    """r = 0 closed forms quoted in SURVEY.md §8(a) A3."""
    pan = geometry.resize_transform((1920, 1080), (960, 512))
    np.testing.assert_allclose(pan, [[0.474074, 0, 24.8889], [0, 0.474074, 0]], atol=1e-4)
    shelf = geometry.resize_transform((1032, 776), (800, 608))
    np.testing.assert_allclose(shelf, [[0.775194, 0, 0], [0, 0.775194, 3.22481]], atol=1e-5)


def test_layers_construct_without_state():
    from fvp.project_whole import ProjectLayer as PW
    from fvp.project_individual import ProjectLayer as PI

    cfg = WORKLOADS["c3"].cfg("cpu")
    pw, pi = PW(cfg), PI(cfg)
    assert len(pw.state_dict()) == 0 and len(pi.state_dict()) == 0  # checkpoints load unchanged
    assert pw.grid.shape == (128000, 3)
    assert tuple(pi.fine_voxels_per_axis.tolist()) == (253, 253, 64)
    assert pi.center_grid.shape == (3, 4096, 2)


def test_synthetic_inputs_deterministic_and_peaked():
    w = WORKLOADS["c2"]
    a = synthetic.gaussian_heatmaps(w, 2)
    b = synthetic.gaussian_heatmaps(w, 2)
    assert np.array_equal(a, b)
    assert a.shape == (2, 5, 15, 128, 240)
    assert 0.0 <= a.min() and a.max() <= 1.0 and a.max() > 0.9
    assert 0.001 < (a > 0).mean() < 0.2


def test_eager_fast_path_routes_tracing_to_the_registered_op():
    """fvp.ops names call the op implementations directly in eager mode (the
    custom-op dispatcher costs ~17 us per call); under a dispatch mode -- here
    FakeTensorMode, as torch.compile / export use -- they must go through the
    registered op and its fake kernel instead (no native call on fake tensors)."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode

    from fvp import ops

    assert isinstance(ops.voxelize.op, torch._library.custom_ops.CustomOpDef)  # the registered op behind the name
    with FakeTensorMode():
        hm = torch.empty((2, 5, 15, 16, 24), device="cuda")
        grid = torch.empty((4 * 4 * 3, 6, 2), device="cuda")
        cube, xy = ops.voxelize(hm, grid, None, 4, 4, 3, True, True)
        planes_out = ops.person_planes(hm, torch.empty((8 * 8 * 4, 6, 2), device="cuda"),
                                       torch.empty((3, 7), device="cuda"), None, [8, 8, 4], [1.0] * 3, [0.0] * 3,
                                       [1.0] * 3, [1.0] * 3, [4, 4, 4], False, True)
    assert type(cube).__name__ == "FakeTensor" and tuple(cube.shape) == (2, 15, 4, 4, 3)
    assert tuple(xy.shape) == (2, 15, 4, 4)
    assert tuple(planes_out[1].shape) == (9, 15, 4, 4)


def test_eager_fast_path_sends_autograd_and_vmap_to_the_registered_op():
    """A grad-requiring input (grad mode on) or an active functorch transform
    must reach the registered op -- which has no autograd formula / batching
    rule and raises -- never the ctypes implementation, which would return
    outputs without a grad_fn.  Plain tensors take the fast path."""
    import torch

    from fvp import ops

    t = torch.zeros(3, requires_grad=True)
    assert ops._needs_dispatcher((t,), {})
    with torch.no_grad():
        assert not ops._needs_dispatcher((t,), {})
    assert not ops._needs_dispatcher((torch.zeros(3),), {"x": 1})
    hits = []
    torch.func.vmap(lambda x: hits.append(ops._needs_dispatcher((x,), {})) or x)(torch.zeros(2, 3))
    assert hits == [True]
    assert callable(ops.fuse_poses.impl) and ops.fuse_poses.impl is not ops.fuse_poses
    assert isinstance(ops.fuse_poses.op, torch._library.custom_ops.CustomOpDef)
