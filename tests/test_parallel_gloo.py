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


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = parallel.shard_frames(total, world, rank)
        vals, flat = _frames_result(s, e - s)
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


def test_pack_roundtrip_is_lossless():
    g = torch.Generator().manual_seed(0)
    v = torch.randn(5, 10, generator=g)
    v[0, 0] = float("nan")
    v[1, 1] = -0.0
    f = torch.randint(0, 6400, (5, 10), generator=g)
    v2, f2 = parallel.unpack_proposals(parallel.pack_proposals(v, f), 10)
    assert torch.equal(f2, f)
    assert torch.equal(v2.view(torch.int32), v.view(torch.int32))


def test_two_rank_gloo_sharded_proposals_match_single_process():
    world, total = 2, 4
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    gv, gf = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rv, rf = _frames_result(0, total)
    assert np.array_equal(gv, rv.numpy())
    assert np.array_equal(gf, rf.numpy())
