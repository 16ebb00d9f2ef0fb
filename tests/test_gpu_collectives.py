"""The multi-GPU collectives of fvp/parallel.py on real HIP tensors over RCCL.

A one-rank "nccl" (RCCL) process group is created in-process from a FileStore
(no launcher, no re-exec); the frame-sharded all-gather of proposals
(gather_proposals) and the large-frame mode's xy-slab all-gather and column
all-reduce (gather_xy_slabs, columns_from_slab) then run on the outputs of the
HIP ops and must reproduce the unsharded results bit for bit.  Ranks > 1 are
covered on CPU by tests/test_parallel_gloo.py (gloo, world 2 and 3); the
8-GPU scaling run is the driver's.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_group(gpu_device):
    if dist.is_initialized():
        pytest.skip("a process group already exists")
    fd, path = tempfile.mkstemp(prefix="fvp_rccl_")
    os.close(fd)
    dist.init_process_group("nccl", store=dist.FileStore(path, 1), rank=0, world_size=1, device_id=gpu_device)
    try:
        assert dist.get_backend() == "nccl"
        yield dist.group.WORLD
    finally:
        dist.destroy_process_group()
        os.unlink(path)


def test_rccl_collectives_on_hip_outputs(gpu_device, rccl_group):
    from fvp import parallel
    from fvp.project_whole import ProjectLayer
    from fvp.proposal import gather_columns, nms2D
    from fvp.workloads import WORKLOADS

    d = golden("whole_c3.npz")
    w = WORKLOADS["c3"]
    layer = ProjectLayer(w.cfg(str(gpu_device)))
    layer.verbose = False
    cams, seq = w.cameras()
    hm = torch.from_numpy(d["heatmaps"]).to(gpu_device)
    rt = torch.from_numpy(d["resize_f32"]).to(gpu_device)
    meta = {"seq": [seq] * hm.shape[0]}
    cube, xy = layer.forward_fused(hm, meta, cams, rt)
    vals, _, flat = nms2D(xy[:, 2:3], w.max_people)

    # frame sharding: the one all-gather of compact proposals
    gv, gf = parallel.gather_proposals(vals, flat, group=rccl_group)
    assert torch.equal(gv, vals) and torch.equal(gf, flat)
    assert np.array_equal(gv.cpu().numpy(), d["nms_vals"])

    # large-frame mode: this rank owns every x-row (world 1): the slab path end to end
    X = w.voxels_per_axis[0]
    x0, x1 = parallel.shard_slab(X, 1, 0)
    cube_s, xy_s = layer.forward_slab(hm, meta, cams, rt, x0, x1)
    full_xy = parallel.gather_xy_slabs(xy_s, X, group=rccl_group)
    assert torch.equal(full_xy, xy)
    v2, _, f2 = nms2D(full_xy[:, 2:3], w.max_people)
    cols = parallel.columns_from_slab(cube_s, f2, x0, group=rccl_group)
    assert torch.equal(cols, gather_columns(cube, flat))
    torch.cuda.synchronize()


def test_rccl_gather_many_frames(gpu_device, rccl_group):
    """The bench's shape: 256 frames x K=10 packed proposals through RCCL."""
    from fvp import parallel

    g = torch.Generator().manual_seed(0)
    vals = torch.rand((256, 10), generator=g).to(gpu_device)
    vals[0, 0] = -0.0
    flat = torch.randint(0, 6400, (256, 10), generator=g).to(gpu_device)
    gv, gf = parallel.gather_proposals(vals, flat, group=rccl_group)
    assert torch.equal(gv.view(torch.int32), vals.view(torch.int32))  # lossless, -0.0 included
    assert torch.equal(gf, flat)
