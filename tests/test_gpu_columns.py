"""fvp_voxel_columns: the winners' z-columns recomputed from the heatmaps
(human_detection_net.py:199-200 without the cube) must equal, bit for bit,
the columns gathered from the cube fvp_voxelize / fvp_voxelize_cams writes --
planar fp32 / fp16 and channels-last input, cached grid and on-the-fly
projection, 5 cameras and the 31-camera ring (16-camera cascade), batches
mixing sequences, and indices outside the map (NaN, as gather_columns)."""
import dataclasses

import pytest
import torch


def _layer(dev, workload, bins=None, otf=False):
    from fvp import geometry
    from fvp.config import make_cfg
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS[workload]
    if bins is not None:
        w = dataclasses.replace(w, voxels_per_axis=bins)
    layer = ProjectLayer(make_cfg(w, str(dev)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float32, device=dev)
    return w, layer, cams, seq, rt


def _flat(B, K, XY, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(0, XY, (B, K), generator=g)


def _check(layer, hm, meta, cams, rt, flat, src=None):
    from fvp import proposal

    cube, _ = layer.forward_fused(hm, meta, cams, rt, want_cube=True, want_xy=False)
    ref = proposal.gather_columns(cube, flat.to(cube.device))
    got = layer.columns(hm if src is None else src, meta, cams, rt, flat.to(cube.device))
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    assert torch.equal(torch.nan_to_num(got, nan=-7.0), torch.nan_to_num(ref, nan=-7.0))
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("cols_otf", [False, True], ids=["cols-grid", "cols-otf"])
@pytest.mark.parametrize("otf", [False, True], ids=["grid", "otf"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16], ids=["f32", "f16"])
def test_columns_match_cube_c2(gpu_device, otf, dtype, cols_otf):
    """The columns' coordinates from the packed grid or projected on the fly
    (ProjectLayer.columns' default) against the cube of either voxelize path."""
    from fvp import synthetic

    w, layer, cams, seq, rt = _layer(gpu_device, "c2", otf=otf)
    layer.columns_on_the_fly = cols_otf
    B, K = 3, 10
    hm = synthetic.uniform_heatmaps(w, B, seed=5).to(dtype).to(gpu_device)
    X, Y, _ = w.voxels_per_axis
    _check(layer, hm, {"seq": [seq] * B}, cams, rt, _flat(B, K, X * Y, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("otf", [False, True], ids=["grid", "otf"])
def test_columns_match_cube_ring31(gpu_device, otf):
    from fvp import synthetic

    w, layer, cams, seq, rt = _layer(gpu_device, "c5", bins=(24, 20, 12), otf=otf)
    B, K = 2, 16
    hm = synthetic.uniform_heatmaps(w, B, seed=9).half().to(gpu_device)
    _check(layer, hm, {"seq": [seq] * B}, cams, rt, _flat(B, K, 24 * 20, 2))


@pytest.mark.gpu
def test_columns_channels_last_and_mixed_sequences(gpu_device):
    from fvp.heatmaps import ChannelsLastHeatmaps

    w, layer, cams, seq, rt = _layer(gpu_device, "c2")
    cams2 = dict(cams)
    seq2 = seq + "_b"
    cams2[seq2] = {i: dict(c, T=c["T"] + 150.0) for i, c in cams[seq].items()}  # a second sequence
    B, J, cp = 4, w.num_joints, 16
    H, W = w.heatmap_size[1], w.heatmap_size[0]
    g = torch.Generator(device="cpu").manual_seed(3)
    planar = torch.rand((B, 5, J, H, W), generator=g).to(gpu_device)
    cl = torch.zeros((B, 5, H, W, cp), device=gpu_device)
    cl[..., :J] = planar.permute(0, 1, 3, 4, 2)
    meta = {"seq": [seq, seq2, seq, seq2]}
    X, Y, _ = w.voxels_per_axis
    flat = _flat(B, 10, X * Y, 4)
    flat[0, 0], flat[1, 3] = -1, X * Y  # outside the map: NaN columns
    got = _check(layer, planar, meta, cams2, rt, flat, src=ChannelsLastHeatmaps(cl, J))
    assert torch.isnan(got[0, 0]).all() and torch.isnan(got[1, 3]).all()


@pytest.mark.gpu
def test_fused_hdn_without_cube_equals_with_cube(gpu_device):
    """integration.fused_hdn_forward with recompute_columns on and off: identical outputs."""
    import types

    import torch.nn as nn
    from fvp import integration, synthetic
    from test_integration import _CenterNet, _Proposal

    torch.manual_seed(0)
    w, layer, cams, seq, rt = _layer(gpu_device, "c3")
    net = types.SimpleNamespace(project_layer=layer, max_people=w.max_people, proposal_layer=_Proposal(w),
                                center_net=_CenterNet(w.num_joints).to(gpu_device).eval(),
                                c2c_net=nn.Conv1d(w.num_joints, 1, 1).to(gpu_device).eval())
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 3)).to(gpu_device)
    meta = {"seq": [seq] * 3}
    outs = {}
    with torch.no_grad():
        for flag in (False, True):
            integration.set_options(net, recompute_columns=flag)
            outs[flag] = integration.fused_hdn_forward(net, hm, meta, cams, rt)
    torch.cuda.synchronize()
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_fused_hdn_automatic_cube_free_choice_at_c5(gpu_device):
    """FvpOptions.recompute_columns = None (the product default) decides by the
    batch's cube size: with the threshold below one C5 frame's cube the
    automatic choice takes the cube-free path at C5's full geometry (31 ring
    cameras, 160x160x64, fp16, on-the-fly coordinates) and must give exactly
    the outputs of the cube path."""
    import types

    import torch.nn as nn
    from fvp import integration, synthetic
    from test_integration import _CenterNet, _Proposal

    torch.manual_seed(1)
    w, layer, cams, seq, rt = _layer(gpu_device, "c5", otf=None)  # auto: C5 projects on the fly
    net = types.SimpleNamespace(project_layer=layer, max_people=w.max_people, proposal_layer=_Proposal(w),
                                center_net=_CenterNet(w.num_joints).to(gpu_device).eval(),
                                c2c_net=nn.Conv1d(w.num_joints, 1, 1).to(gpu_device).eval())
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 2)).half().to(gpu_device)
    meta = {"seq": [seq] * 2}
    seen = []
    orig = layer.columns

    def spy(*a, **k):
        seen.append(1)
        return orig(*a, **k)

    layer.columns = spy
    with torch.no_grad():
        integration.set_options(net, recompute_columns=False)
        ref = integration.fused_hdn_forward(net, hm, meta, cams, rt)
        assert not seen
        X, Y, Z = w.voxels_per_axis
        integration.set_options(net, recompute_columns=None, recompute_cube_bytes=w.num_joints * X * Y * Z * 4)
        got = integration.fused_hdn_forward(net, hm, meta, cams, rt)  # 2 frames' cube > threshold: cube-free
        assert seen, "the automatic size check did not take the cube-free path"
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(torch.nan_to_num(a, nan=-7.0), torch.nan_to_num(b, nan=-7.0))
