"""N > 1 path on CPU: frame sharding + the one proposal all-gather, world_size 2
over gloo (the GPU run uses the same code over RCCL).  The per-frame compute
is the CPU oracle here, standing in for the HIP ops."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fvp import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frames_result(first, count):
    """Oracle voxelise -> root xy plane -> nms2d for frames [first, first+count) of C1."""
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "faster-voxelpose_amd"))
    from fvp import geometry, synthetic
    from fvp.workloads import WORKLOADS
    from oracle import fvp_oracle as O

    w = WORKLOADS["c1"]
    cams, seq = w.cameras()
    rt = geometry.resize_transform(w.ori_image_size, w.image_size).astype(np.float32)
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt)
                   for c in geometry.camera_list(cams, seq)])
    hm = synthetic.gaussian_heatmaps(w, count, first_frame=first)
    xy = np.stack([O.xy_plane(O.voxelize(hm[b], sg).reshape(w.num_joints, *w.voxels_per_axis)) for b in range(count)])
    vals, _, flat = O.nms2d(xy[:, 2:3], 5)
    return torch.from_numpy(vals), torch.from_numpy(flat)


def _worker(rank, world, port, total, q, joint=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = parallel.shard_frames(total, world, rank)
        vals, flat = _frames_result(s, e - s)
        if joint:  # as the HIP NMS writes them: one buffer, sent without packing
            from fvp import ops
            jv, jf = ops.proposal_buffers(vals.shape[0], vals.shape[1], "cpu")
            jv.copy_(vals)
            jf.copy_(flat)
            assert parallel._joint_buffer(jv, jf) is not None
            vals, flat = jv, jf
        gv, gf = parallel.gather_proposals(vals, flat)
        if rank == 0:
            q.put((gv.numpy(), gf.numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_frames_partitions_exactly():
    for n in (0, 1, 7, 256, 257):
        for world in (1, 2, 3, 8):
            spans = [parallel.shard_frames(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(e - s for s, e in spans) - min(e - s for s, e in spans) <= 1
    with pytest.raises(ValueError):
        parallel.shard_frames(4, 2, 2)


def test_joint_buffer_is_recognised_only_when_exact():
    from fvp import ops

    v, f = ops.proposal_buffers(2, 5, "cpu")
    assert parallel._joint_buffer(v, f) is not None
    assert parallel._joint_buffer(v.clone(), f) is None
    assert parallel._joint_buffer(v, f.clone()) is None
    assert parallel._joint_buffer(v[:1], f[:1]) is None


def test_pack_roundtrip_is_lossless():
    g = torch.Generator().manual_seed(0)
    v = torch.randn(5, 10, generator=g)
    v[0, 0] = float("nan")
    v[1, 1] = -0.0
    f = torch.randint(0, 6400, (5, 10), generator=g)
    v2, f2 = parallel.unpack_proposals(parallel.pack_proposals(v, f), 10)
    assert torch.equal(f2, f)
    assert torch.equal(v2.view(torch.int32), v.view(torch.int32))


@pytest.mark.parametrize("world,joint", [(2, False), (2, True), (3, True)])
def test_two_rank_gloo_sharded_proposals_match_single_process(world, joint):
    total = 2 * world
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q, joint)) for r in range(world)]
    for p in procs:
        p.start()
    gv, gf = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rv, rf = _frames_result(0, total)
    assert np.array_equal(gv, rv.numpy())
    assert np.array_equal(gf, rf.numpy())


def _golden_worker(rank, world, port, q):
    """bench.py's N > 1 step on CPU: rank r takes shard_frames(4, world, r) of
    the golden C2 frames (tests/digest_cases.py "c2_g"), voxelises them (oracle
    standing in for the HIP op; each frame's cube checked against the
    reference's SHA-256), NMS on the root plane, then gather_proposals."""
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "faster-voxelpose_amd"), os.path.join(repo, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import digest_cases as dc
        from fvp import geometry
        from fvp.workloads import WORKLOADS
        from oracle import fvp_oracle as O

        w = WORKLOADS["c2"]
        hm, _ = dc.inputs("c2_g")
        s, e = parallel.shard_frames(hm.shape[0], world, rank)
        cams, seq = w.cameras()
        rt = geometry.resize_transform(w.ori_image_size, w.image_size).astype(np.float32)
        grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
        sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt)
                       for c in geometry.camera_list(cams, seq)])
        cube = np.stack([O.voxelize(hm[b], sg).reshape(w.num_joints, *w.voxels_per_axis) for b in range(s, e)])
        ref = np.load(os.path.join(repo, "tests", "golden", "cube_digests.npz"))["c2_g_digests"][s:e]
        assert np.array_equal(O.cube_digests(cube)[:, 0], ref[:, 0]), f"rank {rank}: frames {s}..{e} differ"
        vals, _, flat = O.nms2d(cube.max(axis=4)[:, 2:3], w.max_people)
        gv, gf = parallel.gather_proposals(torch.from_numpy(vals), torch.from_numpy(flat))
        q.put((rank, s, e, vals, flat, gv.numpy(), gf.numpy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_golden_frames_gathered_in_rank_order():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_golden_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    own_v = np.concatenate([g[3] for g in got])
    own_f = np.concatenate([g[4] for g in got])
    assert [g[1:3] for g in got] == [(0, 2), (2, 4)]
    for g in got:  # every rank holds all frames' proposals, rank 0's frames first
        assert np.array_equal(g[5], own_v) and np.array_equal(g[6], own_f)


def _slab_setup(world):
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "faster-voxelpose_amd"))
    from fvp import geometry, synthetic
    from fvp.workloads import WORKLOADS
    from oracle import fvp_oracle as O

    w = WORKLOADS["c1"]
    cams, seq = w.cameras()
    rt = geometry.resize_transform(w.ori_image_size, w.image_size).astype(np.float32)
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt)
                   for c in geometry.camera_list(cams, seq)])
    hm = synthetic.gaussian_heatmaps(w, 2, first_frame=7)
    return w, O, sg, hm


def _cpu_columns(cube, flat):
    """human_detection_net.py:199-200 on CPU: out[b,k,j,:] = cube[b,j,x,y,:] at flat = x*Y + y."""
    B, J, X, Y, Z = cube.shape
    c = cube.reshape(B, J, X * Y, Z).permute(0, 2, 1, 3)
    return c[torch.arange(B)[:, None], flat]


def _slab_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, O, sg, hm = _slab_setup(world)
        X, Y, Z = w.voxels_per_axis
        x0, x1 = parallel.shard_slab(X, world, rank)
        n0, n1 = x0 * Y * Z, x1 * Y * Z
        cube = np.stack([O.voxelize(hm[b], sg[:, n0:n1]).reshape(w.num_joints, x1 - x0, Y, Z)
                         for b in range(hm.shape[0])])
        xy = parallel.gather_xy_slabs(torch.from_numpy(cube.max(axis=4)), X)
        vals, _, flat = O.nms2d(xy[:, 2:3].numpy(), 5)
        cols = parallel.columns_from_slab(torch.from_numpy(cube), torch.from_numpy(flat), x0, gather=_cpu_columns)
        if rank == 0:
            q.put((xy.numpy(), vals, flat, cols.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_x_slab_large_frame_mode_matches_single_process(world):
    """§8(e) large-frame mode: x-slabs per rank (uneven at world 3: 7/7/6 of 20
    rows), xy all-gather, column all-reduce == the unsplit computation."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_slab_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    xy, vals, flat, cols = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    w, O, sg, hm = _slab_setup(world)
    cube = np.stack([O.voxelize(hm[b], sg).reshape(w.num_joints, *w.voxels_per_axis) for b in range(hm.shape[0])])
    ref_xy = cube.max(axis=4)
    rv, _, rf = O.nms2d(ref_xy[:, 2:3], 5)
    assert np.array_equal(xy, ref_xy)
    assert np.array_equal(vals, rv) and np.array_equal(flat, rf)
    assert np.array_equal(cols, _cpu_columns(torch.from_numpy(cube), torch.from_numpy(rf)).numpy())
    assert np.count_nonzero(cols) > 0


def test_shard_slab_rejects_more_ranks_than_rows():
    assert parallel.shard_slab(20, 3, 2) == (14, 20)
    with pytest.raises(ValueError):
        parallel.shard_slab(2, 3, 0)
