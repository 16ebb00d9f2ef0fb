"""bench.py's own N > 1 step on CPU: the sharding
(bench.shard_plan), the step's parts (bench.step_functions: vox / post /
collect) and their order (bench.run_step) -- the exact code the driver's
multi-GPU SCALE run executes over RCCL -- run here at world 2 and 3 over gloo
for the default weak-scaling mode, --strong and --slabs, with the CPU oracle
standing in for the HIP ops.  Every mode's result equals the unsharded
computation bit for bit, and the unsharded cubes of the first four frames are
the reference's own (tests/golden/cube_digests.npz "c2_g")."""
import functools
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOAD = "c2"  # BASELINE configs[1], the bench default


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _paths():
    import sys

    for p in (REPO, os.path.join(REPO, "faster-voxelpose_amd"), os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)


@functools.lru_cache(maxsize=None)
def _setup():
    _paths()
    from fvp import geometry
    from fvp.workloads import WORKLOADS
    from oracle import fvp_oracle as O

    w = WORKLOADS[WORKLOAD]
    cams, seq = w.cameras()
    rt = geometry.resize_transform(w.ori_image_size, w.image_size).astype(np.float32)
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    sg = np.stack([O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt)
                   for c in geometry.camera_list(cams, seq)])
    return w, seq, sg


class OracleCompute:
    """bench.HipCompute's interface on the CPU oracle (oracle/fvp_oracle.py)."""

    def __init__(self):
        self.w, _, self.sg = _setup()

    def voxelize(self, hm, meta, x0=None, x1=None):
        from oracle import fvp_oracle as O

        X, Y, Z = self.w.voxels_per_axis
        x0, x1 = (0, X) if x0 is None else (x0, x1)
        sg = self.sg[:, x0 * Y * Z:x1 * Y * Z]
        h = hm.numpy()
        cube = np.stack([O.voxelize(h[b], sg).reshape(self.w.num_joints, x1 - x0, Y, Z) for b in range(h.shape[0])])
        return torch.from_numpy(cube), torch.from_numpy(cube.max(axis=4))

    @staticmethod
    def nms2D(prob, K):
        from oracle import fvp_oracle as O

        vals, idx, flat = O.nms2d(prob.numpy(), K)
        return torch.from_numpy(vals), torch.from_numpy(idx), torch.from_numpy(flat)

    def nms2D_columns(self, prob, K, cube):
        vals, idx, flat = self.nms2D(prob, K)
        return vals, idx, flat, self.gather_columns(cube, flat)

    @staticmethod
    def gather_columns(cube, flat):
        from oracle import fvp_oracle as O

        return torch.from_numpy(O.gather_columns(cube.numpy(), flat.numpy()))


def _worker(rank, world, port, mode, batch, q):
    _paths()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from fvp import synthetic

        w, seq, _ = _setup()
        X = w.voxels_per_axis[0]
        B, first, x0, x1 = bench.shard_plan(world, rank, batch, X, mode == "slabs", mode == "strong")
        hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, B, first_frame=first))  # as bench.main
        root = 2 if w.num_joints > 2 else 0
        vox, post, collect = bench.step_functions(OracleCompute(), hm, {"seq": [seq] * B}, x0, x1, X, world, True,
                                                  mode == "slabs", root, w.max_people)
        vals, flat, cols, gathered = bench.run_step(vox, post, collect)
        gathered = None if gathered is None else (gathered[0].numpy(), gathered[1].numpy())
        q.put((rank, first, B, x0, x1, vals.numpy(), flat.numpy(), cols.numpy(), gathered))
    finally:
        dist.destroy_process_group()


@functools.lru_cache(maxsize=None)
def _unsharded(frames):
    """The job's frames in one process: cube -> root xy plane -> top-K -> columns."""
    _paths()
    from fvp import synthetic
    from oracle import fvp_oracle as O

    w, _, sg = _setup()
    hm = synthetic.gaussian_heatmaps(w, frames)
    cube = np.stack([O.voxelize(hm[b], sg).reshape(w.num_joints, *w.voxels_per_axis) for b in range(frames)])
    ref = np.load(os.path.join(REPO, "tests", "golden", "cube_digests.npz"))["c2_g_digests"]
    n = min(frames, ref.shape[0])
    assert np.array_equal(O.cube_digests(cube[:n])[:, 0], ref[:n, 0]), "unsharded oracle cubes differ from the reference's"
    root = 2 if w.num_joints > 2 else 0
    vals, _, flat = O.nms2d(cube.max(axis=4)[:, root:root + 1], w.max_people)
    return vals, flat, O.gather_columns(cube, flat)


@pytest.mark.parametrize("mode,world,batch", [("weak", 2, 2), ("weak", 3, 1), ("strong", 2, 4), ("strong", 3, 3),
                                              ("slabs", 2, 2), ("slabs", 3, 2)])
def test_bench_step_at_world_2_and_3_equals_unsharded(mode, world, batch):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    frames = world * batch if mode == "weak" else batch
    rv, rf, rc = _unsharded(frames)
    if mode == "slabs":
        spans = [(g[3], g[4]) for g in got]
        assert spans[0][0] == 0 and spans[-1][1] == 80 and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        for g in got:  # every rank: the whole job's proposals and columns (after the xy gather / column reduce)
            assert g[1] == 0 and g[2] == batch and g[8] is None
            assert np.array_equal(g[5], rv) and np.array_equal(g[6], rf) and np.array_equal(g[7], rc)
    else:
        assert [g[1] for g in got] == [r * got[0][2] for r in range(world)] and sum(g[2] for g in got) == frames
        for g in got:
            s, e = g[1], g[1] + g[2]
            # the rank's own frames, then every rank's proposals in rank order (the one all-gather)
            assert np.array_equal(g[5], rv[s:e]) and np.array_equal(g[6], rf[s:e]) and np.array_equal(g[7], rc[s:e])
            assert np.array_equal(g[8][0], rv) and np.array_equal(g[8][1], rf)
    assert np.count_nonzero(rc) > 0


def test_shard_plan_modes():
    _paths()
    import bench

    assert bench.shard_plan(1, 0, 256, 80) == (256, 0, 0, 80)
    assert [bench.shard_plan(4, r, 8, 80) for r in range(4)] == [(8, 8 * r, 0, 80) for r in range(4)]
    assert [bench.shard_plan(4, r, 8, 80, strong=True) for r in range(4)] == [(2, 2 * r, 0, 80) for r in range(4)]
    assert [bench.shard_plan(3, r, 8, 160, slabs=True) for r in range(3)] == [(8, 0, 0, 54), (8, 0, 54, 107),
                                                                              (8, 0, 107, 160)]
    assert [bench.shard_plan(8, r, 8, 160, slabs=True, strong=True)[2:] for r in range(8)] == \
        [(20 * r, 20 * r + 20) for r in range(8)]
    with pytest.raises(ValueError):
        bench.shard_plan(3, 0, 8, 80, strong=True)


def _line_worker(rank, world, port, q):
    _paths()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench

        # each rank's (wall time, op time): rank 1 is the slowest GPU
        el, ms = 0.5 + 0.1 * rank, [2.40, 2.75, 2.50][rank]
        per_rank = bench.rank_stats([el, ms], "cpu")
        line = None
        if rank == 0:
            ceiling = bench.tap_floor_ceiling(128000, 5, 15, 128, 240, 4, True, 6200.0, 17_280_000)
            traffic = {"traffic": 1.0e10, "traffic_upper": 1.3e10, "layout": 5.0e9, "gather": 5.0e9}
            line = bench.roofline_fields("op", 256 * 17_280_000, [r[1] for r in per_rank], 5, traffic, 6200.0,
                                         38_400_000 * 256, 4, ceiling)
        q.put((rank, per_rank, line))
    finally:
        dist.destroy_process_group()


def test_bench_line_reports_the_slowest_rank_over_gloo():
    """At world > 1 the line's kernel_ms / achieved / frac come from the slowest
    rank's op time (the all-reduced per-rank table), and every rank's time is
    listed."""
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_line_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    table = [[0.5 + 0.1 * r, [2.40, 2.75, 2.50][r]] for r in range(world)]
    for _, per_rank, _ in got:  # every rank holds the same table
        assert np.allclose(per_rank, table)
    line = got[0][2]
    assert line["kernel_ms"] == 2.75 and line["slowest_rank"] == 1 and line["kernel_ms_rank0"] == 2.40
    assert line["kernel_ms_per_rank"] == [2.40, 2.75, 2.50]
    alg = 256 * 17_280_000
    assert line["achieved"] == round(alg / 2.75e-3 / 1e9, 1)
    assert line["frac"] == round(alg / 2.75e-3 / 1e9 / 8000.0, 4)
    assert 0.28 < line["ceiling"]["frac"] < 0.31 and line["frac_of_ceiling"] == round(line["frac"] / line["ceiling"]["frac"], 4)
    assert line["traffic"] == 10_000_000_000 and line["traffic_upper"] == 13_000_000_000


def test_traffic_split_per_kernel(tmp_path):
    """bench.traffic_from_csvs: the layout pass's FETCH doubled (the guide's
    calibrated coalesced stream), the gather's raw with its doubled value as the
    upper bound."""
    _paths()
    import bench

    hdr = '"Kernel_Name","Counter_Name","Counter_Value"\n'
    f = tmp_path / "f.csv"
    f.write_text(hdr + '"fvp::heatmaps_to_cl_kernel<4>","FETCH_SIZE",100\n"fvp::voxelize_kernel<4>","FETCH_SIZE",300\n'
                 '"other_kernel","FETCH_SIZE",999\n')
    w = tmp_path / "w.csv"
    w.write_text(hdr + '"fvp::heatmaps_to_cl_kernel<4>","WRITE_SIZE",50\n"fvp::voxelize_kernel<4>","WRITE_SIZE",20\n')
    t = bench.traffic_from_csvs([str(f)], [str(w)], 2)
    k = 1024.0 / 2
    assert t["layout"] == (2 * 100 + 50) * k and t["gather"] == (300 + 20) * k
    assert t["traffic"] == (2 * 100 + 50 + 300 + 20) * k and t["traffic_upper"] == (2 * 100 + 50 + 600 + 20) * k
