"""Every voxel of every config, bit for bit: the HIP cube's SHA-256 against the
digest of the reference's own ProjectLayer cube (project_whole.py:119-168),
written by tools/gen_golden.py into tests/golden/cube_digests.npz for the
cases of tests/digest_cases.py (C1-C5 and native Shelf; Gaussian-blob and
uniform-random inputs).  A mismatch names the x-slabs that differ.

Each case runs through the cached-grid gather and the on-the-fly projection
gather, fp32 cases also through the channels-last input path
(fvp_voxelize_cl, the backbone's layout), and the per-sequence sample grid the
GPU builds is hashed against the reference's cache."""
import numpy as np
import pytest
import torch

import digest_cases as dc
from conftest import golden
from oracle import fvp_oracle as O

pytestmark = pytest.mark.gpu


def _layer(wname, dev, otf):
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS[wname]
    layer = ProjectLayer(w.cfg(str(dev)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    return w, layer, cams, seq


def _compare(cube, key, tag):
    d = golden("cube_digests.npz")
    c = cube.cpu().numpy()
    got = O.cube_digests(c)
    ref = d[f"{key}_digests"]
    assert got.shape == ref.shape, (got.shape, ref.shape)
    bad = {b: [s - 1 for s in range(1, got.shape[1]) if not np.array_equal(got[b, s], ref[b, s])]
           for b in range(got.shape[0]) if not np.array_equal(got[b, 0], ref[b, 0])}
    assert not bad, f"{tag}: cube differs from the reference's (frame: differing x-slabs of 8) {bad}"
    assert np.array_equal(c.astype(np.float64).sum(axis=(1, 2, 3, 4)), d[f"{key}_sum64"])
    print(f"{tag}: {c.shape[0]} frame(s) x {c[0].size} voxel values identical to the reference (SHA-256)")


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "otf"])
@pytest.mark.parametrize("key", list(dc.CASES))
def test_full_cube_digest(gpu_device, key, otf):
    from fvp import geometry

    wname, _, frames = dc.CASES[key]
    hm, half = dc.inputs(key)
    assert np.array_equal(dc.input_sha(hm), golden("cube_digests.npz")[f"{key}_input_sha256"])
    w, layer, cams, seq = _layer(wname, gpu_device, otf)
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    x = torch.from_numpy(hm)
    x = (x.half() if half else x).to(gpu_device)
    meta = {"seq": [seq] * frames}
    cube, xy = layer.forward_fused(x, meta, cams, rt)
    torch.cuda.synchronize()
    _compare(cube, key, f"{key} {'otf' if otf else 'grid'}")
    assert torch.equal(xy, cube.amax(dim=4))
    if not half:  # the same frames held channels-last, read in place
        from fvp.heatmaps import ChannelsLastHeatmaps

        B, V, J, H, W = x.shape
        cp = 16 * ((J + 15) // 16)
        cl = torch.full((B, V, H, W, cp), 3.0, device=gpu_device)  # junk in the padding channels
        cl[..., :J] = x.permute(0, 1, 3, 4, 2)
        cube_cl, _ = layer.forward_fused(ChannelsLastHeatmaps(cl.contiguous(), J), meta, cams, rt)
        assert torch.equal(cube_cl, cube), f"{key}: channels-last input gives another cube"


@pytest.mark.parametrize("wname", ["c1", "c2", "c3", "shelf_native", "c4", "c5"])
def test_sample_grid_digest(gpu_device, wname):
    """project_grid_kernel's per-sequence cache, every coordinate of every
    camera, against the SHA-256 of the reference's own (project_whole.py:81-117)."""
    from fvp import geometry

    w, layer, cams, seq = _layer(wname, gpu_device, False)
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    sg = layer.build_sample_grid(cams, seq, rt, gpu_device)[:, 0].cpu().numpy()
    ref = golden("cube_digests.npz")[f"grid_{wname}_sha256"]
    bad = [v for v in range(sg.shape[0]) if not np.array_equal(dc.input_sha(np.ascontiguousarray(sg[v], "<f4")), ref[v])]
    assert not bad, f"{wname}: sample grid of cameras {bad} differs from the reference's"


@pytest.mark.parametrize("key", ["c5_g4", "c5_g8", "c5_u"])
def test_c5_x_slabs_on_the_fly_match_reference(gpu_device, key):
    """Large-frame mode at full C5 geometry (31 ring cameras,
    fp16 heatmaps, the 16-camera cascade, 4 frames per pair-table entry): each
    of k = 8 ranks' x-slab of 20 rows, projected on the fly from the camera
    records (fvp_voxelize_cams_slab: no rank builds the 406 MB sample grid),
    hashes to the reference's own per-slab digest of the same rows; the xy
    slabs assemble the whole xy plane, and the columns each slab owns sum to
    the whole cube's columns at the top-K proposals."""
    import hashlib

    from fvp import geometry, parallel
    from fvp.proposal import gather_columns, nms2D

    wname, _, frames = dc.CASES[key]
    hm, half = dc.inputs(key)
    assert half and np.array_equal(dc.input_sha(hm), golden("cube_digests.npz")[f"{key}_input_sha256"])
    ref = golden("cube_digests.npz")[f"{key}_digests"]
    w, layer, cams, seq = _layer(wname, gpu_device, None)  # automatic choice: on the fly at C5
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    x = torch.from_numpy(hm).half().to(gpu_device)
    meta = {"seq": [seq] * frames}
    X, Y, Z = w.voxels_per_axis
    k = ref.shape[1] - 1
    assert layer._project_on_the_fly(x.shape[1]) and k == 8
    xy_rows, slabs = [], []
    for r in range(k):
        x0, x1 = parallel.shard_slab(X, k, r)
        cs, xs = layer.forward_slab(x, meta, cams, rt, x0, x1)
        assert cs.shape == (frames, w.num_joints, x1 - x0, Y, Z)
        c = cs.cpu().numpy()
        for b in range(frames):
            got = np.frombuffer(hashlib.sha256(np.ascontiguousarray(c[b], "<f4").tobytes()).digest(), np.uint8)
            assert np.array_equal(got, ref[b, 1 + r]), f"{key}: frame {b} x-slab {r} [{x0},{x1}) differs"
        assert torch.equal(xs, cs.amax(dim=4))
        xy_rows.append(xs)
        slabs.append((x0, cs))
    assert not layer.sample_grid, "the slab path built a sample grid"
    xy = torch.cat(xy_rows, dim=2)
    _, _, flat = nms2D(xy[:, 2:3].contiguous(), w.max_people)
    cols = sum(parallel.owned_columns(cs, flat, x0) for x0, cs in slabs)
    cube, xy_full = layer.forward_fused(x, meta, cams, rt)
    assert torch.equal(xy, xy_full)
    assert torch.equal(cols, gather_columns(cube, flat))
    print(f"{key}: {frames} frame(s) x {k} on-the-fly x-slabs identical to the reference's slab digests; "
          f"columns from the slabs == whole-cube columns")
