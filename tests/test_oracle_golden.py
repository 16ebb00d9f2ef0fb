"""Pin the CPU oracle (oracle/fvp_oracle.py) to vectors the reference itself
produced (tools/gen_golden.py -> tests/golden/*.npz).  CPU only."""
import numpy as np
import pytest

from conftest import golden
from oracle import fvp_oracle as O
from fvp import geometry
from fvp.workloads import WORKLOADS

WHOLE = [("whole_c1", "c1"), ("whole_c2", "c2"), ("whole_c3", "c3"), ("whole_shelf_native", "shelf_native")]


def _sample_grid(w, resize_f32):
    cams, seq = w.cameras()
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    return grid, np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, resize_f32)
                           for c in geometry.camera_list(cams, seq)])


@pytest.mark.parametrize("case,wname", WHOLE)
def test_resize_transform_matches_reference_dataset(case, wname):
    d = golden(case + ".npz")
    w = WORKLOADS[wname]
    np.testing.assert_allclose(geometry.resize_transform(w.ori_image_size, w.image_size), d["trans"], rtol=0, atol=1e-12)
    assert np.array_equal(np.asarray(d["trans"], np.float32), d["resize_f32"])


@pytest.mark.parametrize("case,wname", WHOLE)
def test_voxel_grid_and_sample_grid_bit_exact(case, wname):
    d = golden(case + ".npz")
    w = WORKLOADS[wname]
    grid, sg = _sample_grid(w, d["resize_f32"])
    assert np.array_equal(grid[d["sub"]], d["grid_ref"])
    assert np.array_equal(sg[:, d["sub"]], d["sample_grid_sub"])
    np.testing.assert_allclose(sg.astype(np.float64).sum(axis=(1, 2)), d["sample_grid_sum"], rtol=1e-12)
    if "sample_grid" in d:
        assert np.array_equal(sg, d["sample_grid"])


@pytest.mark.parametrize("case,wname", WHOLE)
def test_voxelize_and_xy_bit_exact(case, wname):
    d = golden(case + ".npz")
    w = WORKLOADS[wname]
    _, sg = _sample_grid(w, d["resize_f32"])
    J = w.num_joints
    X, Y, Z = w.voxels_per_axis
    for b in range(d["heatmaps"].shape[0]):
        cube = O.voxelize(d["heatmaps"][b], sg)
        assert np.array_equal(cube[:, d["sub"]], d["cube_sub"][b])
        assert np.array_equal(O.xy_plane(cube.reshape(J, X, Y, Z)), d["xy"][b])
        if "cube" in d:
            assert np.array_equal(cube.reshape(J, X, Y, Z), d["cube"][b])


def test_voxelize_uniform_stress_bit_exact():
    from fvp import synthetic

    for case, wname in WHOLE[:2]:
        d = golden(case + ".npz")
        w = WORKLOADS[wname]
        _, sg = _sample_grid(w, d["resize_f32"])
        hu = synthetic.uniform_heatmaps(w, 1, seed=0).numpy()
        cube = O.voxelize(hu[0], sg)
        assert np.array_equal(cube[:, d["sub"]], d["u_cube_sub"][0])


def _check_topk(vals, flat, xy, ref_vals, ref_flat, ref_xy):
    """Values identical; indices identical wherever the value is not tied."""
    assert np.array_equal(vals, ref_vals)
    for b in range(vals.shape[0]):
        for k in range(vals.shape[1]):
            if np.sum(vals[b] == vals[b, k]) == 1:
                assert flat[b, k] == ref_flat[b, k]
                assert np.array_equal(xy[b, k], ref_xy[b, k])


@pytest.mark.parametrize("tag", ["sq", "nonsq", "big"])
def test_nms_random_maps(tag):
    d = golden("nms.npz")
    v, xy, fl = O.nms2d(d[f"{tag}_prob"], d[f"{tag}_vals"].shape[1])
    _check_topk(v, fl, xy, d[f"{tag}_vals"], d[f"{tag}_flat"], d[f"{tag}_xy"])


@pytest.mark.parametrize("case,wname", WHOLE)
def test_nms_and_columns_on_root_plane(case, wname):
    d = golden(case + ".npz")
    w = WORKLOADS[wname]
    prob = d["xy"][:, 2:3]
    v, xy, fl = O.nms2d(prob, w.max_people)
    _check_topk(v, fl, xy, d["nms_vals"], d["nms_flat"], d["nms_xy"])
    if "cube" in d:
        cols = O.gather_columns(d["cube"], d["nms_flat"])
        assert np.array_equal(cols, d["columns"])


def test_project_pose_bit_exact():
    d = golden("project_pose.npz")
    w = WORKLOADS["c3"]
    cams, seq = w.cameras()
    pp = np.stack([O.project_point(d["pts"], c) for c in cams[seq]])
    assert np.array_equal(pp, d["proj"])


def test_individual_layer_bit_exact():
    d = golden("individual_c3.npz")
    w = WORKLOADS["c3"]
    cams, seq = w.cameras()
    ind = O.Individual(w.space_size, w.space_center, w.ind_space_size, w.ind_voxels_per_axis)
    assert np.array_equal(ind.fine.numpy(), d["fine"])
    assert np.array_equal(ind.scale.numpy(), d["scale"])
    assert np.array_equal(ind.bias.numpy(), d["bias"])
    assert np.array_equal(ind.center_grid, d["center_grid"])
    fg = ind.fine_grid()
    assert np.array_equal(fg[d["fine_sub"]], d["fine_grid_sub"])
    cl = geometry.camera_list(cams, seq)
    fsg = np.stack([O.project_grid(fg, c, w.ori_image_size, w.image_size, w.heatmap_size, d["resize_f32"]) for c in cl])
    assert np.array_equal(fsg[:, d["fine_sub"]], d["fine_sample_grid_sub"])
    F = ind.fine_bins
    cubes, off = ind.person_cubes(d["heatmaps"][0], fsg.reshape(len(cl), F[0], F[1], F[2], 2), d["proposals"])
    assert np.array_equal(O.max_planes(cubes), d["planes"])
    assert np.array_equal(off, d["offset"])
    # the fixture exercises clipped windows and one skipped proposal
    _, _, start, end = ind.windows(d["proposals"])
    assert np.any(start == 0) and np.any(end == F)
    assert np.any(np.any(start >= end, axis=1))


def test_individual_constants_host_mirror():
    d = golden("individual_c3.npz")
    w = WORKLOADS["c3"]
    c = geometry.individual_constants(w.space_size, w.space_center, w.ind_space_size, w.ind_voxels_per_axis)
    assert np.array_equal(c["fine"], d["fine"])
    assert np.array_equal(c["scale"], d["scale"])
    assert np.array_equal(c["bias"], d["bias"])


def _c5_heatmaps(d):
    """C5 heatmaps are regenerated (28.6 MB fp16), pinned by the digest the generator stored."""
    import hashlib

    from fvp import synthetic

    w = WORKLOADS["c5"]
    hm = synthetic.gaussian_heatmaps(w, 1).astype(np.float16).astype(np.float32)
    assert hashlib.sha256(np.ascontiguousarray(hm).tobytes()).digest() == d["heatmaps_sha256"].tobytes(), \
        "fvp.synthetic no longer reproduces the C5 heatmaps the reference was run on"
    return hm


def test_c4_full_size_bit_exact():
    """BASELINE configs[3] (128x128x32, demo cameras) at full size: sample grid,
    every voxel of the sampled set, the full xy plane, NMS and columns, and the
    uniform-random stress frame."""
    from fvp import synthetic

    d = golden("whole_c4.npz")
    w = WORKLOADS["c4"]
    grid, sg = _sample_grid(w, d["resize_f32"])
    assert np.array_equal(grid[d["sub"]], d["grid_ref"])
    assert np.array_equal(sg[:, d["sub"]], d["sample_grid_sub"])
    J, (X, Y, Z) = w.num_joints, w.voxels_per_axis
    cube = O.voxelize(d["heatmaps"][0], sg)
    assert np.array_equal(cube[:, d["sub"]], d["cube_sub"][0])
    c4 = cube.reshape(J, X, Y, Z)
    assert np.array_equal(O.xy_plane(c4), d["xy"][0])
    assert np.array_equal(c4.max(axis=(1, 2, 3)), d["cube_max"][0])
    v, xy, fl = O.nms2d(d["xy"][:, 2:3], w.max_people)
    _check_topk(v, fl, xy, d["nms_vals"], d["nms_flat"], d["nms_xy"])
    assert np.array_equal(O.gather_columns(c4[None], d["nms_flat"]), d["columns"])
    hu = synthetic.uniform_heatmaps(w, 1, seed=0).numpy()
    assert np.array_equal(O.voxelize(hu[0], sg[:, d["sub"]]), d["u_cube_sub"][0])


def test_c5_ring_cameras_bit_exact_on_sampled_voxels():
    """BASELINE configs[4] (31 ring cameras, some voxels behind a camera,
    160x160x64, fp16-rounded heatmaps): the sample grid and the cube on the
    sampled voxels (the oracle's full 1.6 M-voxel cube is left to the GPU test)."""
    d = golden("whole_c5.npz")
    w = WORKLOADS["c5"]
    cams, seq = w.cameras()
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    assert np.array_equal(grid[d["sub"]], d["grid_ref"])
    sg = np.stack([O.project_grid(grid[d["sub"]], c, w.ori_image_size, w.image_size, w.heatmap_size, d["resize_f32"])
                   for c in geometry.camera_list(cams, seq)])
    assert np.array_equal(sg, d["sample_grid_sub"])
    hm = _c5_heatmaps(d)
    assert np.array_equal(O.voxelize(hm[0], sg), d["cube_sub"][0])
    # voxels behind a camera are part of the fixture (no masking in project_point)
    behind = 0
    for c in geometry.camera_list(cams, seq):
        R, T = np.asarray(c["R"], np.float64), np.asarray(c["T"], np.float64).reshape(3, 1)
        behind += int(((R @ (grid[d["sub"]].T.astype(np.float64) - T))[2] < 0).sum())
    assert behind > 0


# whole-cube SHA-256 pins written by the reference's ProjectLayer (tests/digest_cases.py);
# the oracle must reproduce every byte of every frame (C5's 31-camera cubes are
# left to the GPU tests: minutes of numpy)
@pytest.mark.parametrize("key", ["c1_g", "c1_u", "c2_g", "c2_u", "c3_g", "c3_u", "shelf_native_g", "c4_g", "c4_u", "c5_g", "c5_u"])
def test_oracle_full_cube_digests(key):
    import os

    import digest_cases as dc

    if key.startswith("c5") and os.environ.get("FVP_SLOW_ORACLE", "0") == "0":
        pytest.skip("C5 oracle cube takes ~4 min of numpy: FVP_SLOW_ORACLE=1 (its sample grid is pinned below)")

    d = golden("cube_digests.npz")
    wname, _, frames = dc.CASES[key]
    w = WORKLOADS[wname]
    hm, _ = dc.inputs(key)
    assert np.array_equal(dc.input_sha(hm), d[f"{key}_input_sha256"]), "regenerated input differs"
    rt = np.asarray(geometry.resize_transform(w.ori_image_size, w.image_size), np.float32)
    _, sg = _sample_grid(w, rt)
    X, Y, Z = w.voxels_per_axis
    cube = np.stack([O.voxelize(hm[b], sg).reshape(w.num_joints, X, Y, Z) for b in range(frames)])
    got = O.cube_digests(cube)
    bad = [(b, s) for b in range(frames) for s in range(got.shape[1]) if not np.array_equal(got[b, s], d[f"{key}_digests"][b, s])]
    assert not bad, f"{key}: (frame, digest slot) mismatches {bad} (slot 0 = whole frame, 1.. = x-slabs)"
    assert np.array_equal(cube.astype(np.float64).sum(axis=(1, 2, 3, 4)), d[f"{key}_sum64"])


@pytest.mark.parametrize("wname", ["c1", "c2", "c3", "shelf_native", "c4", "c5"])
def test_oracle_full_sample_grid_digests(wname):
    """Every camera's whole per-sequence sample grid (project_whole.py:81-117,
    cached at :151-156) against the SHA-256 of the reference's own cache --
    at C5 this is where a one-ulp fp32 fma tie (resize_transform's 8.9e-18
    off-diagonal term) used to slip past the strided samples."""
    import digest_cases as dc

    d = golden("cube_digests.npz")
    w = WORKLOADS[wname]
    rt = np.asarray(geometry.resize_transform(w.ori_image_size, w.image_size), np.float32)
    _, sg = _sample_grid(w, rt)
    ref = d[f"grid_{wname}_sha256"]
    bad = [v for v in range(sg.shape[0]) if not np.array_equal(dc.input_sha(np.ascontiguousarray(sg[v], "<f4")), ref[v])]
    assert not bad, f"{wname}: sample grid of cameras {bad} differs from the reference's"
