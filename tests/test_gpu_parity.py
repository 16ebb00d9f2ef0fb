"""HIP path vs the reference (golden vectors) and vs the CPU oracle.

Every test here runs the product path -- torch.ops.fvp.* over libfvp.so -- on
an MI355X.  The bar is bit-exact: the kernels reproduce the reference CPU
path's fp32 operation order (faster-voxelpose_amd/csrc/fvp_device.h), so the
comparisons use array_equal; the north-star tolerance (1e-4 on voxel values)
is asserted as well so a failure report shows which bar broke.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import fvp_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north_star: "within 1e-4 on float32 voxel values"


def _layers():
    from fvp import project_whole, project_individual, proposal, ops  # noqa: F401
    return project_whole, project_individual, proposal


def _whole(wname, dev):
    from fvp.workloads import WORKLOADS
    from fvp.project_whole import ProjectLayer

    w = WORKLOADS[wname]
    layer = ProjectLayer(w.cfg(str(dev)))
    layer.verbose = False
    cams, seq = w.cameras()
    return w, layer, cams, seq


def _assert_same(got, ref, what):
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, what
    diff = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    assert np.nanmax(diff) <= TOL, f"{what}: max |diff| {np.nanmax(diff)} > {TOL}"
    assert np.array_equal(got, ref), f"{what}: not bit-exact ({np.count_nonzero(diff)} of {diff.size} differ, " \
                                     f"max {np.nanmax(diff)})"


WHOLE = [("whole_c1", "c1"), ("whole_c2", "c2"), ("whole_c3", "c3"), ("whole_shelf_native", "shelf_native")]


@pytest.mark.parametrize("case,wname", WHOLE)
def test_sample_grid_matches_reference(gpu_device, case, wname):
    d = golden(case + ".npz")
    w, layer, cams, seq = _whole(wname, gpu_device)
    rt = torch.from_numpy(d["resize_f32"]).to(gpu_device)
    sg = layer.build_sample_grid(cams, seq, rt, gpu_device)[:, 0].cpu().numpy()
    _assert_same(sg[:, d["sub"]], d["sample_grid_sub"], "sample grid")
    np.testing.assert_allclose(sg.astype(np.float64).sum(axis=(1, 2)), d["sample_grid_sum"], rtol=1e-12)
    if "sample_grid" in d:
        _assert_same(sg, d["sample_grid"], "full sample grid")


@pytest.mark.parametrize("case,wname", WHOLE)
def test_voxelize_matches_reference(gpu_device, case, wname):
    d = golden(case + ".npz")
    w, layer, cams, seq = _whole(wname, gpu_device)
    rt = torch.from_numpy(d["resize_f32"]).to(gpu_device)
    hm = torch.from_numpy(d["heatmaps"]).to(gpu_device)
    B = hm.shape[0]
    cube, xy = layer.forward_fused(hm, {"seq": [seq] * B}, cams, rt)
    torch.cuda.synchronize()
    J = w.num_joints
    N = w.num_voxels
    c = cube.cpu().numpy()
    _assert_same(c.reshape(B, J, N)[:, :, d["sub"]], d["cube_sub"], "cube (sampled voxels)")
    _assert_same(xy.cpu().numpy(), d["xy"], "xy plane")
    assert np.array_equal(c.astype(np.float64).sum(axis=(2, 3, 4)), d["cube_sum"])  # numpy order both sides
    if "cube" in d:
        _assert_same(c, d["cube"], "full cube")
    # the plain drop-in forward returns the same cube
    c2 = layer(hm, {"seq": [seq] * B}, cams, rt)
    assert torch.equal(c2, cube)


@pytest.mark.parametrize("case,wname", WHOLE[:2])
def test_voxelize_uniform_stress_matches_reference(gpu_device, case, wname):
    from fvp import synthetic

    d = golden(case + ".npz")
    w, layer, cams, seq = _whole(wname, gpu_device)
    rt = torch.from_numpy(d["resize_f32"]).to(gpu_device)
    hu = synthetic.uniform_heatmaps(w, 1, seed=0).to(gpu_device)
    cube, xy = layer.forward_fused(hu, {"seq": [seq]}, cams, rt)
    N = w.num_voxels
    _assert_same(cube.cpu().numpy().reshape(1, w.num_joints, N)[:, :, d["sub"]], d["u_cube_sub"], "uniform cube")
    _assert_same(xy.cpu().numpy(), d["u_xy"], "uniform xy")


def _check_topk(vals, flat, xy, ref_vals, ref_flat, ref_xy):
    """Values identical everywhere; indices identical in every tie-free slot.
    A slot whose value is tied with another slot of the same frame may hold any
    member of the tie group (torch.topk leaves their order unspecified): there
    the set of indices of each tie group that lies wholly inside the top-K must
    match the reference's.  Returns the number of slots not compared one by one."""
    assert np.array_equal(vals, ref_vals)
    tied = 0
    for b in range(vals.shape[0]):
        for k in range(vals.shape[1]):
            group = vals[b] == vals[b, k]
            if np.sum(group) == 1:  # tie-free entries: identical argmax indices
                assert flat[b, k] == ref_flat[b, k]
                assert np.array_equal(xy[b, k], ref_xy[b, k])
                continue
            tied += 1
            if not group[-1]:  # the whole group is inside the top-K: same members
                assert set(flat[b][group]) == set(ref_flat[b][group]), (b, k)
    return tied


@pytest.mark.parametrize("tag", ["sq", "nonsq", "big"])
def test_nms_matches_reference(gpu_device, tag):
    from fvp.proposal import nms2D

    d = golden("nms.npz")
    p = torch.from_numpy(d[f"{tag}_prob"]).to(gpu_device)
    v, xy, fl = nms2D(p, d[f"{tag}_vals"].shape[1])
    tied = _check_topk(v.cpu().numpy(), fl.cpu().numpy(), xy.cpu().numpy(), d[f"{tag}_vals"], d[f"{tag}_flat"],
                       d[f"{tag}_xy"])
    print(f"nms {tag}: {tied} tied slots compared as tie-group sets")
    # ties resolved value-desc / index-asc exactly like the oracle
    ov, oxy, ofl = O.nms2d(d[f"{tag}_prob"], d[f"{tag}_vals"].shape[1])
    assert np.array_equal(fl.cpu().numpy(), ofl)


@pytest.mark.parametrize("case,wname", WHOLE)
def test_proposals_and_columns_match_reference(gpu_device, case, wname):
    from fvp.proposal import nms2D, gather_columns

    d = golden(case + ".npz")
    w, layer, cams, seq = _whole(wname, gpu_device)
    rt = torch.from_numpy(d["resize_f32"]).to(gpu_device)
    hm = torch.from_numpy(d["heatmaps"]).to(gpu_device)
    B = hm.shape[0]
    cube, xy = layer.forward_fused(hm, {"seq": [seq] * B}, cams, rt)
    v, idx, fl = nms2D(xy[:, 2:3].contiguous(), w.max_people)
    _check_topk(v.cpu().numpy(), fl.cpu().numpy(), idx.cpu().numpy(), d["nms_vals"], d["nms_flat"], d["nms_xy"])
    cols = gather_columns(cube, torch.from_numpy(d["nms_flat"]).to(gpu_device))
    _assert_same(cols.cpu().numpy(), d["columns"], "columns")


def test_gather_bbox_matches_torch_gather(gpu_device):
    from fvp.proposal import gather_bbox

    g = torch.Generator().manual_seed(3)
    size = torch.rand((3, 2, 80, 80), generator=g)
    flat = torch.randint(0, 6400, (3, 10), generator=g)
    ref = torch.gather(torch.flatten(size, 2, 3).permute(0, 2, 1), 1, flat.unsqueeze(2).repeat(1, 1, 2))
    got = gather_bbox(size.to(gpu_device), flat.to(gpu_device)).cpu()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("otf", [True, False], ids=["onthefly", "finegrid"])
def test_person_cubes_and_planes_match_reference(gpu_device, otf):
    """Both coordinate sources of the per-person kernel (fine grid projected on
    the fly, or the packed per-sequence fine grid) against the reference's cubes."""
    from fvp.workloads import WORKLOADS
    from fvp.project_individual import ProjectLayer

    d = golden("individual_c3.npz")
    w = WORKLOADS["c3"]
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    assert np.array_equal(layer.center_grid.cpu().numpy(), d["center_grid"])
    assert np.array_equal(layer.fine_voxels_per_axis.cpu().numpy(), d["fine"])
    rt = torch.from_numpy(d["resize_f32"]).to(gpu_device)
    hm = torch.from_numpy(d["heatmaps"]).to(gpu_device)
    props = torch.from_numpy(d["proposals"]).to(gpu_device)
    cubes, offset = layer(hm, 0, {"seq": [seq]}, props, cams, rt)
    planes = torch.ops.fvp.max_planes(cubes)
    fsg = layer.build_sample_grid(cams, seq, rt, gpu_device).cpu().numpy()
    _assert_same(fsg.reshape(fsg.shape[0], -1, 2)[:, d["fine_sub"]], d["fine_sample_grid_sub"], "fine sample grid")
    _assert_same(offset.cpu().numpy(), d["offset"], "offset")
    _assert_same(planes.cpu().numpy(), d["planes"], "planes")
    assert np.array_equal(cubes.cpu().numpy().astype(np.float64).sum(axis=(2, 3, 4)), d["cube_sum"])  # numpy order both sides
    _assert_same(cubes[0].cpu().numpy().reshape(5, -1)[:, ::53], d["cube0_sub"], "cube 0")
    p2, off2 = layer.forward_planes(hm, 0, {"seq": [seq]}, props, cams, rt)
    assert torch.equal(p2, planes) and torch.equal(off2, offset)


# ---------------------------------------------------------------------------
# oracle comparisons on shapes the golden set does not cover (edge cases)
# ---------------------------------------------------------------------------

def _custom_workload(**kw):
    from fvp.workloads import WORKLOADS
    import dataclasses

    return dataclasses.replace(WORKLOADS[kw.pop("base", "c3")], **kw)


@pytest.mark.parametrize("bins,J,hm_size", [((13, 11, 7), 3, (240, 128)), ((8, 8, 1), 32, (64, 48)),
                                            ((24, 16, 5), 17, (200, 152)), ((1, 1, 9), 2, (2, 2)),
                                            ((10, 9, 4), 15, (61, 33)), ((6, 7, 5), 20, (45, 31))])
def test_ragged_shapes_vs_oracle(gpu_device, bins, J, hm_size):
    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer

    w = _custom_workload(voxels_per_axis=bins, num_joints=J, heatmap_size=hm_size)
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    trans = geometry.resize_transform(w.ori_image_size, w.image_size)
    rt = torch.as_tensor(trans, dtype=torch.float)
    hm = synthetic.uniform_heatmaps(w, 2, seed=5)
    cube, xy = layer.forward_fused(hm.to(gpu_device), {"seq": [seq] * 2}, cams, rt.to(gpu_device))
    grid = O.compute_grid(w.space_size, w.space_center, bins)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, hm_size, rt.numpy())
                   for c in geometry.camera_list(cams, seq)])
    for b in range(2):
        ref = O.voxelize(hm[b].numpy(), sg).reshape(J, *bins)
        _assert_same(cube[b].cpu().numpy(), ref, f"cube frame {b}")
        _assert_same(xy[b].cpu().numpy(), O.xy_plane(ref), f"xy frame {b}")


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "onthefly"])
@pytest.mark.parametrize("half", [False, True], ids=["f32", "f16"])
@pytest.mark.parametrize("V,J", [(1, 3), (2, 6), (4, 1), (7, 15), (31, 15), (31, 24), (7, 32), (3, 16)])
def test_camera_and_joint_counts_vs_oracle(gpu_device, V, J, half, otf):
    """Every lane-group size (J -> 1/2/4/8 lanes per voxel), odd/even and
    >2*LPV camera counts (packed-grid groups), the fp16 pixel-pair table
    (J <= 16), the fp16 -> fp32 layout fallback (J > 16), and the cached-grid
    and on-the-fly-projection coordinate sources."""
    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer

    bins, hm_size = (12, 10, 6), (64, 48)
    w = _custom_workload(base="c5", voxels_per_axis=bins, num_joints=J, heatmap_size=hm_size, extra={"views": V})
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float)
    hm = synthetic.uniform_heatmaps(w, 3, seed=V * 100 + J)
    if half:
        hm = hm.half()
    cube, xy = layer.forward_fused(hm.to(gpu_device), {"seq": [seq] * 3}, cams, rt.to(gpu_device))
    grid = O.compute_grid(w.space_size, w.space_center, bins)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, hm_size, rt.numpy())
                   for c in geometry.camera_list(cams, seq)])
    assert sg.shape[0] == V
    for b in range(3):
        ref = O.voxelize(hm[b].float().numpy(), sg).reshape(J, *bins)
        _assert_same(cube[b].cpu().numpy(), ref, f"cube frame {b}")
        _assert_same(xy[b].cpu().numpy(), O.xy_plane(ref), f"xy frame {b}")


def test_sample_grid_is_view_of_packed_grid(gpu_device):
    """sample_grid[seq] keeps the reference's [V,1,N,2] layout as a view of the
    voxel-major packed grid; a grid assigned from outside is packed on use."""
    from fvp import geometry, synthetic, ops
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c3"]
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 2)).to(gpu_device)
    cube, _ = layer.forward_fused(hm, {"seq": [seq] * 2}, cams, rt)
    sg = layer.sample_grid[seq]
    N = 80 * 80 * 20
    assert sg.shape == (5, 1, N, 2)
    packed = layer._packed[seq]
    assert packed.shape == (N, ops.grid_slots(5), 2)
    assert torch.equal(packed[:, :5].permute(1, 0, 2), sg[:, 0])
    assert torch.equal(packed[:, 5:], torch.full_like(packed[:, 5:], -2.0))
    other = ProjectLayer(w.cfg(str(gpu_device)))
    other.verbose = False
    other.sample_grid[seq] = sg.contiguous().clone()  # reference-layout tensor from outside
    cube2, _ = other.forward_fused(hm, {"seq": [seq] * 2}, cams, rt)
    assert torch.equal(cube, cube2)
    # the outside grid modified in place is repacked (its _version moved), not read stale
    other.sample_grid[seq][0].copy_(sg[1])
    cube3, _ = other.forward_fused(hm, {"seq": [seq] * 2}, cams, rt)
    fresh = ProjectLayer(w.cfg(str(gpu_device)))
    fresh.verbose = False
    fresh.sample_grid[seq] = other.sample_grid[seq].clone()
    cube4, _ = fresh.forward_fused(hm, {"seq": [seq] * 2}, cams, rt)
    assert torch.equal(cube3, cube4) and not torch.equal(cube3, cube)


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "onthefly"])
def test_mixed_sequences_in_one_batch(gpu_device, otf):
    """Frames of different sequences (different cameras) in one launch."""
    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c3"]
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    cams2 = {"a": cams[seq], "b": list(reversed(cams[seq]))}
    trans = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 3)).to(gpu_device)
    meta = {"seq": ["a", "b", "a"]}
    cube, xy = layer.forward_fused(hm, meta, cams2, trans.to(gpu_device))
    for b, s in enumerate(meta["seq"]):
        single, sxy = layer.forward_fused(hm[b:b + 1], {"seq": [s]}, cams2, trans.to(gpu_device))
        assert torch.equal(single[0], cube[b]) and torch.equal(sxy[0], xy[b])
    assert not torch.equal(cube[0], cube[1])
    other = ProjectLayer(w.cfg(str(gpu_device)))
    other.verbose = False
    other.on_the_fly = not otf
    c_o, x_o = other.forward_fused(hm, meta, cams2, trans.to(gpu_device))
    assert torch.equal(c_o, cube) and torch.equal(x_o, xy)  # both coordinate sources agree bit-for-bit


def test_batch_invariance_full_size(gpu_device):
    """BASELINE full size (C2 geometry, 64 frames): each frame's result is
    independent of its batch position, xy == max_z(cube), values in [0,1]."""
    from fvp import synthetic
    from fvp.workloads import WORKLOADS

    w, layer, cams, seq = _whole("c2", gpu_device)
    from fvp import geometry
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = synthetic.uniform_heatmaps(w, 64, seed=11).to(gpu_device)
    cube, xy = layer.forward_fused(hm, {"seq": [seq] * 64}, cams, rt)
    assert torch.equal(torch.max(cube, dim=4)[0], xy)
    assert float(cube.min()) >= 0.0 and float(cube.max()) <= 1.0
    for b in (0, 37, 63):
        c1, x1 = layer.forward_fused(hm[b:b + 1].clone(), {"seq": [seq]}, cams, rt)
        assert torch.equal(c1[0], cube[b]) and torch.equal(x1[0], xy[b])
    # one frame against the oracle at full size
    d = golden("whole_c2.npz")
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, d["resize_f32"])
                   for c in geometry.camera_list(cams, seq)])
    ref = O.voxelize(hm[37].cpu().numpy(), sg).reshape(cube.shape[1:])
    _assert_same(cube[37].cpu().numpy(), ref, "frame 37 full cube")


def test_cameras_looking_away_give_zero(gpu_device):
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS
    from fvp import geometry

    w = WORKLOADS["c3"]
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    away = []
    for c in cams[seq]:
        c2 = dict(c)
        c2["T"] = np.array(c["T"]) + np.array([[0.0], [0.0], [1e7]])  # far above: everything projects off-image
        away.append(c2)
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.ones((1, 5, w.num_joints, 128, 240), device=gpu_device)
    cube, xy = layer.forward_fused(hm, {"seq": ["away"]}, {"away": away}, rt)
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt.cpu().numpy())
                   for c in away])
    ref = O.voxelize(hm[0].cpu().numpy(), sg).reshape(cube.shape[1:])
    _assert_same(cube[0].cpu().numpy(), ref, "cameras looking away")


def test_reference_assertions_and_errors(gpu_device):
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS
    from fvp import geometry, _lib

    w = WORKLOADS["c3"]
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.zeros((1, 5, 15, 128, 240), device=gpu_device)
    with pytest.raises(AssertionError, match="missing camera parameters"):
        layer(hm, {"seq": ["nope"]}, cams, rt)
    with pytest.raises(AssertionError, match="inconsistent number of cameras"):
        layer(hm[:, :4], {"seq": [seq]}, cams, rt)
    with pytest.raises(Exception):
        layer(hm.cpu(), {"seq": [seq]}, cams, rt)  # no CPU fallback
    with pytest.raises(_lib.FvpError, match="forward-only"):
        layer(hm.clone().requires_grad_(True), {"seq": [seq]}, cams, rt)


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "onthefly"])
def test_empty_batches_and_proposal_sets(gpu_device, otf):
    """B = 0 frames (the reference's frame loop returns an empty [0,J,X,Y,Z]
    cube) and K = 0 / P = 0 proposals give empty outputs, not errors."""
    from fvp import geometry, ops, proposal
    from fvp.project_individual import ProjectLayer as PersonLayer

    w, layer, cams, seq = _whole("c3", gpu_device)
    layer.on_the_fly = otf
    X, Y, Z = w.voxels_per_axis
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.zeros((0, 5, 15, 128, 240), device=gpu_device)
    cube = layer(hm, {"seq": []}, cams, rt)
    assert cube.shape == (0, 15, X, Y, Z) and cube.dtype == torch.float32
    c2, xy = layer.forward_fused(hm, {"seq": []}, cams, rt)
    assert c2.shape == (0, 15, X, Y, Z) and xy.shape == (0, 15, X, Y)
    vals, idx, flat = proposal.nms2D(xy[:, 2:3], 10)
    assert vals.shape == (0, 10) and idx.shape == (0, 10, 2) and flat.shape == (0, 10)
    assert proposal.gather_columns(c2, flat).shape == (0, 10, 15, Z)
    one = torch.rand((1, 15, X, Y, Z), device=gpu_device)
    assert proposal.gather_columns(one, flat.new_zeros((1, 0))).shape == (1, 0, 15, Z)
    person = PersonLayer(w.cfg(str(gpu_device)))
    person.verbose = False
    hm1 = torch.rand((1, 5, 15, 128, 240), device=gpu_device)
    cubes, offset = person(hm1, 0, {"seq": [seq]}, torch.zeros((0, 7), device=gpu_device), cams, rt)
    assert cubes.shape[0] == 0 and offset.shape == (0, 3)


def test_fp16_heatmaps_computed_in_fp32(gpu_device):
    """C5 input dtype: fp16 heatmaps are upcast exactly and computed in fp32
    (oracle on hm.half().float())."""
    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c3"]
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float)
    hm = synthetic.uniform_heatmaps(w, 2, seed=9).half()
    cube, xy = layer.forward_fused(hm.to(gpu_device), {"seq": [seq] * 2}, cams, rt.to(gpu_device))
    c32, x32 = layer.forward_fused(hm.float().to(gpu_device), {"seq": [seq] * 2}, cams, rt.to(gpu_device))
    assert torch.equal(cube, c32) and torch.equal(xy, x32)
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt.numpy())
                   for c in geometry.camera_list(cams, seq)])
    ref = O.voxelize(hm[1].float().numpy(), sg).reshape(cube.shape[1:])
    _assert_same(cube[1].cpu().numpy(), ref, "fp16 frame")


@pytest.mark.parametrize("B", [2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("otf", [False, True], ids=["grid", "otf"])
def test_fp16_frame_pairs_batch_invariance(gpu_device, B, otf):
    """The fp16 pair table holds four frames per entry, a batch's remainder
    two and / or one: every frame of a batch (2 = a pair, 3 = a pair and a
    single, 4 / 5 = a group of 4 (and a single), 6 = a group and a pair, 7 =
    all three) equals its own single-frame launch and the fp32 layout's
    result; 31 ring cameras (the 16-camera cascade) on a small grid."""
    from fvp import geometry, synthetic
    from fvp.config import make_cfg
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS
    import dataclasses

    w = dataclasses.replace(WORKLOADS["c5"], voxels_per_axis=(24, 20, 12))
    layer = ProjectLayer(make_cfg(w, str(gpu_device)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = synthetic.uniform_heatmaps(w, B, seed=21).half().to(gpu_device)
    cube, xy = layer.forward_fused(hm, {"seq": [seq] * B}, cams, rt)
    c32, x32 = layer.forward_fused(hm.float(), {"seq": [seq] * B}, cams, rt)
    assert torch.equal(cube, c32) and torch.equal(xy, x32)
    for b in range(B):
        c1, x1 = layer.forward_fused(hm[b:b + 1], {"seq": [seq]}, cams, rt)
        assert torch.equal(cube[b:b + 1], c1) and torch.equal(xy[b:b + 1], x1), b
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt.cpu().numpy())
                   for c in geometry.camera_list(cams, seq)])
    ref = O.voxelize(hm[B - 1].float().cpu().numpy(), sg).reshape(cube.shape[1:])
    _assert_same(cube[B - 1].cpu().numpy(), ref, "fp16 ring frame")


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "otf"])
def test_fp16_pair_layouts_agree(gpu_device, otf):
    """pairs_vec8_kernel (16-B-aligned heatmaps, width % 8 == 0: 8 entries a
    thread), pairs_rows_kernel (4-B-aligned: a block per row, through LDS) and
    the per-entry layout kernel (a 2-B-aligned address or an odd width) build
    the same pair table: identical cubes and xy planes for 7 frames (entries of
    4, 2 and 1 frames), 31 ring cameras on a small grid."""
    from fvp import geometry, synthetic
    from fvp.config import make_cfg
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS
    import dataclasses

    w = dataclasses.replace(WORKLOADS["c5"], voxels_per_axis=(24, 20, 12))
    layer = ProjectLayer(make_cfg(w, str(gpu_device)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = synthetic.uniform_heatmaps(w, 7, seed=23).half().to(gpu_device)
    cube, xy = layer.forward_fused(hm, {"seq": [seq] * 7}, cams, rt)
    buf = torch.empty(hm.numel() + 8, dtype=torch.float16, device=gpu_device)
    hm_odd = buf[1:1 + hm.numel()].view(hm.shape)  # contiguous, 2 B past a 4-B boundary: the per-entry kernel
    hm_odd.copy_(hm)
    assert hm_odd.is_contiguous() and hm_odd.data_ptr() % 4 == 2
    c_e, x_e = layer.forward_fused(hm_odd, {"seq": [seq] * 7}, cams, rt)
    assert torch.equal(cube, c_e) and torch.equal(xy, x_e)
    hm_4 = buf[2:2 + hm.numel()].view(hm.shape)  # 4 B past a 16-B boundary: pairs_rows_kernel
    hm_4.copy_(hm)
    assert hm_4.data_ptr() % 16 == 4 and hm.data_ptr() % 16 == 0 and hm.shape[-1] % 8 == 0
    c_r, x_r = layer.forward_fused(hm_4, {"seq": [seq] * 7}, cams, rt)
    assert torch.equal(cube, c_r) and torch.equal(xy, x_r)


def test_nms_on_channel_slice_without_copy(gpu_device):
    from fvp.proposal import nms2D

    g = torch.Generator().manual_seed(21)
    planes = torch.rand((3, 15, 80, 80), generator=g).to(gpu_device)
    v1, i1, f1 = nms2D(planes[:, 2:3], 10)
    v2, i2, f2 = nms2D(planes[:, 2:3].contiguous(), 10)
    assert torch.equal(v1, v2) and torch.equal(f1, f2) and torch.equal(i1, i2)
    ov, oxy, ofl = O.nms2d(planes[:, 2:3].cpu().numpy(), 10)
    assert np.array_equal(v1.cpu().numpy(), ov) and np.array_equal(f1.cpu().numpy(), ofl)


@pytest.mark.parametrize("mode", ["f32", "f16", "cl", "onthefly"])
def test_more_than_32_joints(gpu_device, mode):
    """J = 40 runs as joint slices of 32 + 8 (layout pass + gather per slice; the
    channels-last input read at the slice's channel offset) == the oracle bit for bit."""
    import dataclasses

    from fvp import geometry
    from fvp.heatmaps import ChannelsLastHeatmaps
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    J = 40
    w = dataclasses.replace(WORKLOADS["c3"], num_joints=J, voxels_per_axis=(16, 12, 6))
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    layer.on_the_fly = mode == "onthefly"
    cams, seq = w.cameras()
    rt_np = geometry.resize_transform(w.ori_image_size, w.image_size).astype(np.float32)
    rt = torch.from_numpy(rt_np).to(gpu_device)
    Wh, Hh = w.heatmap_size
    B = 2
    hm = torch.rand((B, 5, J, Hh, Wh), generator=torch.Generator().manual_seed(40))
    if mode == "f16":
        hm = hm.half()
    ref_in = hm.float().numpy()
    hg = hm.to(gpu_device)
    meta = {"seq": [seq] * B}
    if mode == "cl":
        cl = torch.full((B, 5, Hh, Wh, 48), 5.0, device=gpu_device)
        cl[..., :J] = hg.permute(0, 1, 3, 4, 2)
        hg = ChannelsLastHeatmaps(cl, J)
    cube, xy = layer.forward_fused(hg, meta, cams, rt)
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt_np)
                   for c in cams[seq]])
    for b in range(B):
        ref = O.voxelize(ref_in[b], sg).reshape(cube.shape[1:])
        _assert_same(cube[b].cpu().numpy(), ref, f"J=40 cube {mode} frame {b}")
        _assert_same(xy[b].cpu().numpy(), O.xy_plane(ref), f"J=40 xy {mode} frame {b}")


def _person_setup(gpu_device, J, S, space=2000.0):
    """C3 cameras, a 2 m capture space (the fine grid stays small: S^3 x V slots)."""
    import dataclasses

    from fvp import geometry, synthetic
    from fvp.project_individual import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = dataclasses.replace(WORKLOADS["c3"], num_joints=J, space_size=(space, space, space),
                            ind_space_size=(space, space, space), ind_voxels_per_axis=(S, S, S))
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 1)).to(gpu_device)
    c = w.space_center
    props = np.array([[c[0], c[1], c[2], 0, 0.9, 0.5, 0.5], [c[0] + 300, c[1] - 200, c[2] - 100, 0, 0.8, 0.2, 0.9],
                      [c[0] - 700, c[1] + 500, c[2] + 300, 0, 0.7, 1.1, 0.3]], np.float32)
    return w, layer, cams, seq, rt, hm, props


@pytest.mark.parametrize("otf", [False, True], ids=["finegrid", "onthefly"])
@pytest.mark.parametrize("J,S", [(40, 32), (5, 96), (3, 80)])
def test_person_joint_slices_and_deep_cubes(gpu_device, J, S, otf):
    """Person cubes / planes with J > 32 (joint slices) and S > 64 (64-deep z
    chunks; max_planes beyond 64 on the per-cell kernel) == the oracle."""
    w, layer, cams, seq, rt, hm, props = _person_setup(gpu_device, J, S)
    layer.on_the_fly = otf
    pg = torch.from_numpy(props).to(gpu_device)
    meta = {"seq": [seq]}
    planes, offset = layer.forward_planes(hm, 0, meta, pg, cams, rt)
    cubes, off2 = layer(hm, 0, meta, pg, cams, rt)
    ind = O.Individual(w.space_size, w.space_center, w.ind_space_size, w.ind_voxels_per_axis)
    fsg = layer.build_sample_grid(cams, seq, rt, gpu_device).cpu().numpy()
    ref_cubes, ref_off = ind.person_cubes(hm[0].cpu().numpy(), fsg, props)
    _assert_same(cubes.cpu().numpy(), ref_cubes, f"cubes J={J} S={S}")
    _assert_same(planes.cpu().numpy(), O.max_planes(ref_cubes), f"fused planes J={J} S={S}")
    _assert_same(offset.cpu().numpy(), ref_off, "offset")
    mp = torch.ops.fvp.max_planes(cubes)
    _assert_same(mp.cpu().numpy(), O.max_planes(ref_cubes), f"max_planes S={S}")


def test_soft_argmax_long_rows(gpu_device):
    """Soft-argmax of 96 x 96 planes (9216 cells: the two-pass kernel) vs float64."""
    from fvp import ops

    P, J, S = 2, 3, 96
    g = torch.Generator().manual_seed(3)
    feat = torch.rand((3, P, J, S, S), generator=g)
    grid = torch.rand((3, S * S, 2), generator=g) * 1000.0
    off = torch.rand((P, 3), generator=g) * 10.0
    pose, maxprob = ops.soft_argmax(feat.to(gpu_device), grid.to(gpu_device), off.to(gpu_device), 100.0)
    ref_pose, _ = O.soft_argmax(feat.numpy(), grid.numpy(), 100.0)
    ref_pose = O.add_offsets(ref_pose, off.numpy())
    y = 100.0 * feat.numpy().reshape(3, P, J, -1).astype(np.float64)
    ref_mp = 1.0 / np.exp(y - y.max(axis=3, keepdims=True)).sum(axis=3)  # max of the softmax
    assert np.abs(pose.cpu().numpy() - ref_pose).max() <= 0.05
    assert np.abs(maxprob.cpu().numpy() - ref_mp).max() <= 1e-5


def _jln_setup(gpu_device, J=15, frames=3):
    from fvp import geometry, synthetic
    from fvp.project_individual import ProjectLayer
    from fvp.workloads import WORKLOADS
    import dataclasses

    w = dataclasses.replace(WORKLOADS["c3"], num_joints=J)
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, frames)).to(gpu_device)
    return w, layer, cams, seq, rt, hm


def _props(w, f, rng, n_extra):
    from fvp import synthetic

    base = synthetic.proposals_for_frame(w, f, 4)
    extra = np.zeros((n_extra, 7), np.float32)
    extra[:, 0] = rng.uniform(-4600, 4600, n_extra)
    extra[:, 1] = -500 + rng.uniform(-4600, 4600, n_extra)
    extra[:, 2] = rng.uniform(200, 1500, n_extra)
    extra[:, 5:7] = rng.uniform(-0.2, 1.2, (n_extra, 2))
    return np.concatenate([base, extra])


@pytest.mark.parametrize("otf", [True, False], ids=["onthefly", "finegrid"])
@pytest.mark.parametrize("J", [15, 17])
def test_person_planes_fused_vs_oracle(gpu_device, J, otf):
    """Fused planes (no cube) == max-projections of the oracle's cubes, incl.
    clipped, skipped and negative-margin windows; J=17 takes the 8-lane path."""
    from fvp import geometry

    w, layer, cams, seq, rt, hm = _jln_setup(gpu_device, J=J, frames=1)
    layer.on_the_fly = otf
    props = _props(w, 0, np.random.default_rng(1), 6)
    planes, offset = layer.forward_planes(hm, 0, {"seq": [seq]}, torch.from_numpy(props).to(gpu_device), cams, rt)
    ind = O.Individual(w.space_size, w.space_center, w.ind_space_size, w.ind_voxels_per_axis)
    fsg = layer.build_sample_grid(cams, seq, rt, gpu_device).cpu().numpy()
    cubes, off = ind.person_cubes(hm[0].cpu().numpy(), fsg, props)
    _assert_same(planes.cpu().numpy(), O.max_planes(cubes), "fused planes")
    _assert_same(offset.cpu().numpy(), off, "offset")
    c2, _ = layer(hm, 0, {"seq": [seq]}, torch.from_numpy(props).to(gpu_device), cams, rt)
    _assert_same(c2.cpu().numpy(), cubes, "cubes")


@pytest.mark.parametrize("otf", [True, False], ids=["onthefly", "finegrid"])
def test_person_planes_batched_matches_per_frame(gpu_device, otf):
    """forward_batch (one launch, >= 64 proposals -> 4-row blocks) == per-frame calls (1-row blocks)."""
    w, layer, cams, seq, rt, hm = _jln_setup(gpu_device, frames=8)
    layer.on_the_fly = otf
    rng = np.random.default_rng(2)
    props = torch.from_numpy(np.stack([_props(w, f, rng, 6) for f in range(8)])).to(gpu_device)  # [8,10,7]
    mask = torch.rand((8, 10), generator=torch.Generator().manual_seed(3)).to(gpu_device) > 0.15
    meta = {"seq": [seq] * 8}
    planes, offset, frame_of = layer.forward_batch(hm, meta, props, mask, cams, rt)
    P = int(mask.sum())
    assert planes.shape[0] == 3 * P and P >= 64 // 2
    k = 0
    for f in range(8):
        sel = props[f][mask[f]]
        if sel.shape[0] == 0:
            continue
        pf, of = layer.forward_planes(hm, f, meta, sel, cams, rt)
        n = sel.shape[0]
        for part in range(3):
            assert torch.equal(planes[part * P + k: part * P + k + n], pf[part * n:(part + 1) * n])
        assert torch.equal(offset[k:k + n], of)
        k += n
    assert k == P


@pytest.mark.parametrize("otf", [True, False], ids=["onthefly", "finegrid"])
def test_person_planes_batched_match_reference_digests(gpu_device, otf):
    """The JLN's batched launch (forward_batch: 8 C3 frames x 10 proposals, one
    launch, 4-row blocks) against the REFERENCE's per-person ProjectLayer run frame
    by frame (tools/gen_golden.py -> individual_batch_c3.npz): every person's xy /
    xz / yz max-plane hashes to the reference's SHA-256, and the offsets are equal."""
    import digest_cases as dc

    g = golden("individual_batch_c3.npz")
    w, layer, cams, seq, rt, hm = _jln_setup(gpu_device, frames=8)
    assert np.array_equal(dc.input_sha(hm.cpu().numpy()), g["heatmaps_sha256"])
    layer.on_the_fly = otf
    props = torch.from_numpy(g["proposals"]).to(gpu_device)  # [8, 10, 7]
    F_, P_ = props.shape[:2]
    mask = torch.ones((F_, P_), dtype=torch.bool, device=gpu_device)
    planes, offset, frame_of = layer.forward_batch(hm, {"seq": [seq] * F_}, props, mask, cams, rt)
    P = F_ * P_
    assert planes.shape[0] == 3 * P
    pl = planes.cpu().numpy()
    bad = [(f, k, i) for f in range(F_) for k in range(P_) for i in range(3)
           if not np.array_equal(dc.input_sha(pl[i * P + f * P_ + k]), g["plane_sha256"][f, k, i])]
    assert not bad, f"planes differing from the reference's (frame, proposal, plane): {bad[:8]}"
    assert np.array_equal(offset.cpu().numpy().reshape(F_, P_, 3), g["offset"])


@pytest.mark.parametrize("K", [1, 16, 17, 40])
def test_nms_topk_both_paths_vs_oracle(gpu_device, K):
    """K <= 16 takes the register top-K kernel, larger K the rescan kernel; both
    order ties value-desc / index-asc like the oracle (maps with many zeros)."""
    from fvp.proposal import nms2D

    g = torch.Generator().manual_seed(K)
    prob = torch.rand((5, 1, 60, 60), generator=g)
    prob[prob < 0.7] = 0.0  # large tied plateaus
    prob[0, 0, 3, 4] = float("nan")
    v, xy, fl = nms2D(prob.to(gpu_device), K)
    ov, oxy, ofl = O.nms2d(prob.numpy(), K)
    got = v.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ov))
    assert np.array_equal(np.nan_to_num(got, nan=7.0), np.nan_to_num(ov, nan=7.0))
    assert np.array_equal(fl.cpu().numpy()[1:], ofl[1:])  # frame 0 holds a NaN (ordering checked above)
    assert np.array_equal(xy.cpu().numpy()[1:], oxy[1:])


@pytest.mark.parametrize("kind", ["zeros", "nan", "negative", "tiny", "big_noise", "big_smooth", "row", "ragged",
                                  "column", "wide_row", "nan_spots"])
def test_nms_select_degenerate_maps_vs_oracle(gpu_device, kind):
    """The threshold-select top-K on plateaus (all-zero, all-NaN, all-negative
    maps: ties broken by index), maps smaller than K waves, 128x128 maps
    (16 elements per thread), ragged shapes, a 300 x 1 column (one-element
    strips), a 2 x 1500 row (wider than the block: element-per-thread mapping)
    and scattered NaNs (windows that hold one), against the oracle bit for bit."""
    from fvp.proposal import nms2D

    g = torch.Generator().manual_seed(11)
    shape, K = {"zeros": ((3, 1, 80, 80), 10), "nan": ((2, 1, 80, 80), 10), "negative": ((2, 1, 40, 40), 16),
                "tiny": ((4, 1, 4, 4), 16), "big_noise": ((3, 1, 128, 128), 10),
                "big_smooth": ((3, 1, 128, 128), 16), "row": ((2, 1, 1, 300), 5),
                "ragged": ((5, 1, 37, 53), 7), "column": ((2, 1, 300, 1), 5), "wide_row": ((2, 1, 2, 1500), 5),
                "nan_spots": ((3, 1, 80, 80), 10)}[kind]
    if kind == "zeros":
        prob = torch.zeros(shape)
    elif kind == "nan":
        prob = torch.full(shape, float("nan"))
    elif kind == "negative":
        prob = -torch.rand(shape, generator=g)
    elif kind == "big_smooth":
        B, _, X, Y = shape
        prob = torch.nn.functional.avg_pool2d(torch.rand((B, 1, X + 8, Y + 8), generator=g), 9, 1)
    else:
        prob = torch.rand(shape, generator=g)
    if kind == "nan_spots":
        prob.view(-1)[torch.randperm(prob.numel(), generator=g)[:12]] = float("nan")
    v, xy, fl = nms2D(prob.to(gpu_device), K)
    ov, oxy, ofl = O.nms2d(prob.numpy(), K)
    got = v.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ov.view(np.uint32)) or (
        np.array_equal(np.isnan(got), np.isnan(ov)) and np.array_equal(np.nan_to_num(got), np.nan_to_num(ov)))
    assert np.array_equal(fl.cpu().numpy(), ofl)
    assert np.array_equal(xy.cpu().numpy(), oxy)


def test_nms_expanded_map_batch_stride_zero(gpu_device):
    """A batch-expanded map (batch stride 0) gives every frame the one map's top-K."""
    from fvp.proposal import nms2D

    g = torch.Generator().manual_seed(3)
    one = torch.rand((1, 1, 40, 40), generator=g)
    prob = one.to(gpu_device).expand(4, 1, 40, 40)
    assert prob.stride()[0] == 0
    for K in (10, 20):
        v, xy, fl = nms2D(prob, K)
        ov, oxy, ofl = O.nms2d(one.numpy(), K)
        for b in range(4):
            assert np.array_equal(v[b].cpu().numpy(), ov[0])
            assert np.array_equal(fl[b].cpu().numpy(), ofl[0])


@pytest.mark.parametrize("K", [16, 20])
def test_nms_signed_zero_and_nan_payload_pass_through(gpu_device, K):
    """keep = 0 times a negative value is -0.0 and 0 * NaN keeps the NaN's payload:
    the selected values come back bit for bit, as torch.topk returns them."""
    from fvp.proposal import nms2D

    vals = -np.arange(1, 37, dtype=np.float32).reshape(1, 1, 6, 6)
    vals[0, 0, 4, 4] = np.frombuffer(np.uint32(0x7FC01234).tobytes(), np.float32)[0]  # NaN with a payload
    prob = torch.from_numpy(vals).to(gpu_device)
    v, xy, fl = nms2D(prob, K)
    # the masked map computed by torch on the same device (max_pool2d keep mask)
    mp = torch.nn.functional.max_pool2d(prob, 3, 1, 1)
    masked = ((prob == mp).float() * prob).flatten().cpu().numpy().view(np.uint32)
    got = v.cpu().numpy()[0].view(np.uint32)
    assert np.array_equal(got, masked[fl.cpu().numpy()[0]])  # values are the selected elements, bit for bit
    ov, _, ofl = O.nms2d(vals, K)
    assert np.array_equal(fl.cpu().numpy(), ofl)
    assert np.signbit(v.cpu().numpy()[0][1:]).sum() == np.signbit(ov[0][1:]).sum()  # -0.0 entries kept negative
    assert np.isnan(v.cpu().numpy()[0, 0])


def test_captured_graph_step_matches_eager(gpu_device):
    """The hot-path step (voxelize -> NMS -> columns) captured as one hipGraph
    replays to the eager results, and picks up new frames copied into its input."""
    from fvp import geometry, synthetic
    from fvp.graphs import CapturedStep
    from fvp.project_whole import ProjectLayer
    from fvp.proposal import gather_columns, nms2D
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c2"]
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    frames = torch.from_numpy(synthetic.gaussian_heatmaps(w, 3)).to(gpu_device)
    hm = frames[0:1].clone()
    meta = {"seq": [seq]}

    def step():
        cube, xy = layer.forward_fused(hm, meta, cams, rt)
        vals, idx, flat = nms2D(xy[:, 2:3], 10)
        return cube, xy, vals, flat, gather_columns(cube, flat)

    cap = CapturedStep(step)
    for f in (0, 2):
        hm.copy_(frames[f:f + 1])
        got = [t.clone() for t in cap.replay()]
        ref = step()
        for g, r in zip(got, ref):
            assert torch.equal(g, r)


def test_person_planes_on_the_fly_equals_fine_grid(gpu_device):
    """Batched planes and offsets: the on-the-fly projection and the packed fine
    grid give bit-identical results (same fp32 projection sequence)."""
    w, layer, cams, seq, rt, hm = _jln_setup(gpu_device, frames=6)
    rng = np.random.default_rng(4)
    props = torch.from_numpy(np.stack([_props(w, f, rng, 6) for f in range(6)])).to(gpu_device)
    mask = torch.ones((6, props.shape[1]), dtype=torch.bool, device=gpu_device)
    meta = {"seq": [seq] * 6}
    layer.on_the_fly = True
    p1, o1, f1 = layer.forward_batch(hm, meta, props, mask, cams, rt)
    layer.on_the_fly = False
    p2, o2, f2 = layer.forward_batch(hm, meta, props, mask, cams, rt)
    assert torch.equal(p1, p2) and torch.equal(o1, o2) and torch.equal(f1, f2)


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "otf"])
@pytest.mark.parametrize("wname,nslab,half", [("c2", 2, False), ("c4", 3, False), ("c2", 3, True)])
def test_x_slabs_equal_full_grid(gpu_device, wname, nslab, half, otf):
    """Large-frame mode: forward_slab on each rank's x-slab
    (fvp.parallel.shard_slab, uneven at 3 slabs) is bit-identical to the same
    rows of the whole-grid launch, for mixed-sequence batches too, from the
    cached grid's rows and projected on the fly for the slab's rows only
    (channels-last input as well)."""
    from fvp import geometry, parallel, synthetic
    from fvp.heatmaps import ChannelsLastHeatmaps

    w, layer, cams, seq = _whole(wname, gpu_device)
    layer.on_the_fly = otf
    X = w.voxels_per_axis[0]
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 3)).to(gpu_device)
    if half:
        hm = hm.half()
    cl = geometry.camera_list(cams, seq)
    cams2 = {"a": cl, "b": cl[::-1]}
    for meta in ({"seq": ["a"] * 3}, {"seq": ["a", "b", "a"]}):
        cube, xy = layer.forward_fused(hm, meta, cams2, rt)
        for r in range(nslab):
            x0, x1 = parallel.shard_slab(X, nslab, r)
            cs, xs = layer.forward_slab(hm, meta, cams2, rt, x0, x1)
            assert torch.equal(cs, cube[:, :, x0:x1]) and torch.equal(xs, xy[:, :, x0:x1])
            if not half:
                B, V, J, H, W = hm.shape
                cl = torch.zeros((B, V, H, W, 16), device=gpu_device)
                cl[..., :J] = hm.permute(0, 1, 3, 4, 2)
                cs, xs = layer.forward_slab(ChannelsLastHeatmaps(cl, J), meta, cams2, rt, x0, x1)
                assert torch.equal(cs, cube[:, :, x0:x1]) and torch.equal(xs, xy[:, :, x0:x1])
    if otf:
        assert not layer.sample_grid, "the on-the-fly slab path built a sample grid"
    with pytest.raises(ValueError):
        layer.forward_slab(hm, meta, cams2, rt, 4, 4)


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "onthefly"])
@pytest.mark.parametrize("half", [False, True], ids=["f32", "f16"])
def test_nonfinite_heatmaps_vs_torch_grid_sample(gpu_device, otf, half):
    """NaN and +-inf heatmap pixels: the reference's own CPU ops (F.grid_sample,
    mean, clamp -- oracle/torch_cpu.py) give NaN where a NaN pixel or an
    inf*0-weight tap is sampled and +-inf elsewhere, clamp keeps NaN; torch.max
    over z propagates NaN.  The HIP path must give the same pattern and values."""
    from fvp import geometry
    from oracle import torch_cpu

    w, layer, cams, seq = _whole("c3", gpu_device)
    layer.on_the_fly = otf
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float)
    g = torch.Generator().manual_seed(11)
    hm = torch.rand((2, 5, 15, 128, 240), generator=g)
    flat = hm.view(-1)
    idx = torch.randperm(flat.numel(), generator=g)[:3000]
    flat[idx[:1000]] = float("nan")
    flat[idx[1000:2000]] = float("inf")
    flat[idx[2000:]] = float("-inf")
    if half:
        hm = hm.half()
    meta = {"seq": [seq] * 2}
    cube, xy = layer.forward_fused(hm.to(gpu_device), meta, cams, rt.to(gpu_device))
    sg = layer.build_sample_grid(cams, seq, rt.to(gpu_device), gpu_device).cpu().contiguous()
    ref = torch_cpu.voxelize(hm.float(), sg, w.voxels_per_axis)
    got = cube.cpu()
    assert torch.isnan(ref).any() and torch.isinf(ref).sum() == 0  # clamp maps +-inf to 1 / 0
    np.testing.assert_array_equal(got.numpy(), ref.numpy())  # NaN == NaN positions, values bit-equal
    np.testing.assert_array_equal(xy.cpu().numpy(), torch.max(ref, dim=4)[0].numpy())


@pytest.mark.parametrize("otf", [True, False], ids=["onthefly", "finegrid"])
def test_person_planes_nonfinite_heatmaps(gpu_device, otf):
    """NaN / +-inf heatmap pixels through the per-person kernel: the fused planes
    (atomic maxima into pre-zeroed planes) equal torch.max over the cube path's
    cubes (joint_localization_net.py:158-160), NaN positions included.  (The
    whole-space test above pins the per-voxel NaN/inf arithmetic to torch's
    grid_sample; the person kernel shares it, fvp_device.h.)"""
    from fvp.project_individual import ProjectLayer

    d = golden("individual_c3.npz")
    w = _custom_workload()
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    rt = torch.from_numpy(d["resize_f32"]).to(gpu_device)
    hm = torch.from_numpy(d["heatmaps"]).clone()
    g = torch.Generator().manual_seed(12)
    flat = hm.view(-1)
    idx = torch.randperm(flat.numel(), generator=g)[:6000]
    flat[idx[:2000]] = float("nan")
    flat[idx[2000:4000]] = float("inf")
    flat[idx[4000:]] = float("-inf")
    hm = hm.to(gpu_device)
    props = torch.from_numpy(d["proposals"]).to(gpu_device)
    cubes, offset = layer(hm, 0, {"seq": [seq]}, props, cams, rt)
    assert torch.isnan(cubes).any()
    ref = torch.cat([torch.max(cubes, dim=4)[0], torch.max(cubes, dim=3)[0], torch.max(cubes, dim=2)[0]])
    planes, off2 = layer.forward_planes(hm, 0, {"seq": [seq]}, props, cams, rt)
    np.testing.assert_array_equal(planes.cpu().numpy(), ref.cpu().numpy())
    assert torch.equal(off2, offset)


@pytest.mark.parametrize("otf", [False, True], ids=["finegrid", "onthefly"])
def test_person_planes_channels_last_bit_exact(gpu_device, otf):
    """fvp_person_planes_cl (channels-last heatmaps, e.g. the backbone's NHWC
    output, read in place) == the planar path, batched and per frame."""
    from fvp.heatmaps import ChannelsLastHeatmaps, attach

    w, layer, cams, seq, rt, hm = _jln_setup(gpu_device, frames=3)
    layer.on_the_fly = otf
    rng = np.random.default_rng(9)
    props = torch.from_numpy(np.stack([_props(w, f, rng, 3) for f in range(3)])).to(gpu_device)
    mask = torch.ones(props.shape[:2], dtype=torch.bool, device=gpu_device)
    mask[1, 2] = False
    meta = {"seq": [seq] * 3}
    cl = torch.full(hm.shape[:2] + hm.shape[3:] + (32,), 9.0, device=gpu_device)  # pitch 32 > JP, junk after J
    cl[..., :15] = hm.permute(0, 1, 3, 4, 2)
    clh = ChannelsLastHeatmaps(cl, 15)
    p1, o1, f1 = layer.forward_batch(hm, meta, props, mask, cams, rt)
    p2, o2, f2 = layer.forward_batch(clh, meta, props, mask, cams, rt)
    assert torch.equal(p1, p2) and torch.equal(o1, o2) and torch.equal(f1, f2)
    a = layer.forward_planes(hm, 1, meta, props[1], cams, rt)
    b = layer.forward_planes(attach(hm.clone(), clh), 1, meta, props[1], cams, rt)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_forward_batch_mixed_sequences(gpu_device):
    """forward_batch over frames of two sequences (one launch per sequence,
    scattered back into (frame, proposal) order) == per-frame forward_planes."""
    w, layer, cams, seq, rt, hm = _jln_setup(gpu_device, frames=3)
    cams = dict(cams)
    cams["other"] = list(reversed(list(cams[seq])))  # another sequence: same cameras, another order
    rng = np.random.default_rng(10)
    props = torch.from_numpy(np.stack([_props(w, f, rng, 2) for f in range(3)])).to(gpu_device)
    mask = torch.ones(props.shape[:2], dtype=torch.bool, device=gpu_device)
    mask[0, 1] = False
    meta = {"seq": [seq, "other", seq]}
    planes, offset, frame_of = layer.forward_batch(hm, meta, props, mask, cams, rt)
    P = planes.shape[0] // 3
    rows, offs = [], []
    for b in range(3):
        pl, off = layer.forward_planes(hm, b, meta, props[b][mask[b]], cams, rt)
        rows.append(pl.view(3, -1, *pl.shape[1:]))
        offs.append(off)
    ref = torch.cat(rows, dim=1).reshape(3 * P, *planes.shape[1:])
    assert torch.equal(planes, ref) and torch.equal(offset, torch.cat(offs))
    assert frame_of.tolist() == mask.nonzero()[:, 0].tolist()


def test_out_of_range_indices(gpu_device):
    """Gathers at an index outside the map read nothing and return NaN (the
    reference's torch.gather raises); a host grid_index out of range is rejected."""
    from fvp import _lib
    from fvp.proposal import gather_bbox, gather_columns

    cube = torch.rand((2, 3, 4, 5, 6), device=gpu_device)
    flat = torch.tensor([[0, 19, 20], [-1, 3, 7]], device=gpu_device)
    cols = gather_columns(cube, flat)
    assert torch.isnan(cols[0, 2]).all() and torch.isnan(cols[1, 0]).all()
    assert torch.equal(cols[0, 1], cube[0, :, 3, 4]) and torch.equal(cols[1, 2], cube[1, :, 1, 2])
    bb = gather_bbox(torch.rand((2, 2, 4, 5), device=gpu_device), flat)
    assert torch.isnan(bb[0, 2]).all() and not torch.isnan(bb[0, 1]).any()
    hm = torch.zeros((2, 1, 2, 8, 8), device=gpu_device)
    pg = torch.zeros((1, 8, 2, 2), device=gpu_device)
    with pytest.raises(_lib.FvpError, match="grid_index"):
        torch.ops.fvp.voxelize(hm, pg, torch.tensor([0, 1], dtype=torch.int32), 2, 2, 2, True, True)


@pytest.mark.parametrize("K", [10, 17])
def test_nms_topk_columns_fused(gpu_device, K):
    """fvp_nms_topk_columns == fvp_nms_topk then fvp_gather_columns (K <= 16 one
    launch; K = 17 the two-launch path), on the C2 golden cube's root-joint plane."""
    from fvp.proposal import gather_columns, nms2D, nms2D_columns

    g = torch.Generator().manual_seed(K)
    cube = torch.rand((3, 15, 80, 80, 20), generator=g).to(gpu_device)
    xy = cube.max(dim=4)[0]
    prob = xy[:, 2:3]
    v1, i1, f1 = nms2D(prob, K)
    c1 = gather_columns(cube, f1)
    v2, i2, f2, c2 = nms2D_columns(prob, K, cube)
    assert torch.equal(v1, v2) and torch.equal(i1, i2) and torch.equal(f1, f2) and torch.equal(c1, c2)
    ov, _, ofl = O.nms2d(prob.cpu().numpy(), K)
    assert np.array_equal(v2.cpu().numpy(), ov)
    assert np.array_equal(c2.cpu().numpy(), O.gather_columns(cube.cpu().numpy(), f2.cpu().numpy()))


@pytest.mark.parametrize("side", [160, 180, 190])
def test_nms_large_maps_vs_oracle(gpu_device, side):
    """C5-sized detection maps: 160^2 and 180^2 through the select kernel (32
    elements per thread), 190^2 through the K-round kernel; ties included (a
    quantised map has plateaus)."""
    from fvp.proposal import nms2D

    g = torch.Generator().manual_seed(side)
    p = (torch.rand((2, 1, side, side), generator=g) * 64).floor() / 64
    v, xy, fl = nms2D(p.to(gpu_device), 10)
    ov, oxy, ofl = O.nms2d(p.numpy(), 10)
    assert np.array_equal(v.cpu().numpy(), ov) and np.array_equal(fl.cpu().numpy(), ofl)
    assert np.array_equal(xy.cpu().numpy(), oxy)


@pytest.mark.parametrize("wname", ["c2", "c4"])
def test_cube_pointer_not_16b_aligned(gpu_device, wname):
    """The C ABI takes any float* for the cube: the gather's float4 epilogue
    runs only when the caller's pointer is 16-B aligned (checked on the host),
    so a cube 4 B past a 16-B boundary gets the scalar stores -- same values
    (fvp_voxelize.hip vec epilogue)."""
    from fvp import _lib, geometry, synthetic

    w, layer, cams, seq = _whole(wname, gpu_device)
    layer.on_the_fly = False
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 2)).to(gpu_device)
    meta = {"seq": [seq] * 2}
    cube, xy = layer.forward_fused(hm, meta, cams, rt)
    grids, _ = layer._grids_for_batch(hm, meta, cams, rt)
    B, V, J, H, W = hm.shape
    X, Y, Z = w.voxels_per_axis
    L = _lib.load()
    nws = L.fvp_voxelize_workspace_bytes(B, V, J, H, W)
    ws = torch.empty((nws + 3) // 4, device=gpu_device)
    buf = torch.full((cube.numel() + 4,), -7.0, device=gpu_device)
    xy2 = torch.empty_like(xy)
    st = torch.cuda.current_stream(gpu_device).cuda_stream
    for off in (1, 2, 3):
        buf.fill_(-7.0)
        assert (buf.data_ptr() + 4 * off) % 16 != 0
        _lib.check(L.fvp_voxelize(hm.data_ptr(), B, V, J, H, W, grids.data_ptr(), None, X, Y, Z,
                                  buf.data_ptr() + 4 * off, xy2.data_ptr(), ws.data_ptr(), nws, st), "fvp_voxelize")
        torch.cuda.synchronize()
        assert torch.equal(buf[off:off + cube.numel()].view(cube.shape), cube), off
        assert bool((buf[:off] == -7.0).all()) and bool((buf[off + cube.numel():] == -7.0).all()), off
        assert torch.equal(xy2, xy)


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "otf"])
@pytest.mark.parametrize("image_size,hm_size", [((800.5, 608.0), (240, 128)), ((960.0, 512.0), (65537, 2)),
                                                ((70000.0, 512.0), (240, 128))])
def test_divisors_outside_div_const_sweep_take_ieee_division(gpu_device, otf, image_size, hm_size):
    """pixel_to_sample's four divisions (IMAGE_SIZE w / h, HEATMAP_SIZE - 1)
    take the reciprocal form div_const only for integer divisors in
    [1, 65535], the range tools/div_const_sweep.c proves exact; a fractional
    image size, a heatmap 65537 wide and an image 70000 wide take the IEEE
    division -- the sample grid equals the oracle's (numpy fp32 division)
    bit for bit, and so does the on-the-fly projection's cube."""
    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer

    bins = (6, 5, 4)
    w = _custom_workload(voxels_per_axis=bins, num_joints=3, heatmap_size=hm_size, image_size=image_size)
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float)
    grid = O.compute_grid(w.space_size, w.space_center, bins)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, hm_size, rt.numpy())
                   for c in geometry.camera_list(cams, seq)])
    got = layer.build_sample_grid(cams, seq, rt.to(gpu_device), gpu_device)[:, 0].cpu().numpy()
    _assert_same(got, sg, "sample grid")
    if hm_size[0] * hm_size[1] <= 1 << 20:
        hm = synthetic.uniform_heatmaps(w, 1, seed=3)
        cube, _ = layer.forward_fused(hm.to(gpu_device), {"seq": [seq]}, cams, rt.to(gpu_device))
        _assert_same(cube[0].cpu().numpy(), O.voxelize(hm[0].numpy(), sg).reshape(3, *bins), "cube")


@pytest.mark.parametrize("kind", ["plateau", "plateau_k16", "smooth_b8", "c5_size", "single"])
def test_nms_plateaus_and_columns_vs_oracle(gpu_device, kind):
    """nms2D and the fused column gather on a few peaks over exact zeros (the
    candidate list then holds hundreds of tied zeros, ranked by index), on C3-like
    smooth maps at B = 8, a 160 x 160 map and K = X*Y: bit for bit against the
    oracle, columns against torch indexing."""
    from fvp.proposal import nms2D, nms2D_columns

    g = torch.Generator().manual_seed(len(kind))
    shape, K = {"plateau": ((8, 1, 80, 80), 10), "plateau_k16": ((3, 1, 80, 80), 16),
                "smooth_b8": ((8, 1, 80, 80), 10), "c5_size": ((2, 1, 160, 160), 10),
                "single": ((3, 1, 3, 3), 9)}[kind]
    B, _, X, Y = shape
    if kind.startswith("plateau"):
        prob = torch.rand(shape, generator=g)
        prob[prob < 0.999] = 0.0
    elif kind == "smooth_b8":
        prob = torch.nn.functional.avg_pool2d(torch.rand((B, 1, X + 6, Y + 6), generator=g), 7, 1)
    else:
        prob = torch.rand(shape, generator=g)
    J, Z = 3, 6
    cube = torch.rand((B, J, X, Y, Z), generator=g).to(gpu_device)
    pd = prob.to(gpu_device)
    ov, oxy, ofl = O.nms2d(prob.numpy(), K)
    v, xy, fl = nms2D(pd, K)
    v2, xy2, fl2, cols = nms2D_columns(pd, K, cube)
    assert np.array_equal(v.cpu().numpy(), ov) and np.array_equal(v2.cpu().numpy(), ov)
    assert np.array_equal(fl.cpu().numpy(), ofl) and np.array_equal(fl2.cpu().numpy(), ofl)
    assert np.array_equal(xy.cpu().numpy(), oxy) and np.array_equal(xy2.cpu().numpy(), oxy)
    ref_cols = torch.stack([cube[b].reshape(J, X * Y, Z)[:, fl[b]].permute(1, 0, 2) for b in range(B)])
    assert torch.equal(cols, ref_cols)
