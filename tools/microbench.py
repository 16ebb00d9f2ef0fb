#!/usr/bin/env python3
"""A/B timing of voxelize variants (tools/vox_variants.hip) against the product
kernel, interleaved in one process (cdna_hip_programming.md §5.4 rule 24).

    python tools/microbench.py [--batch 256] [--rounds 5] [--workload c2]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))

VARIANTS = [1, 11, 10, 201, 211, 210, 311, 411, 410]


def build_variants():
    src = os.path.join(REPO, "tools", "vox_variants.hip")
    out = os.path.join(REPO, "tools", "libvoxvar.so")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        import torch

        tl = os.path.join(os.path.dirname(torch.__file__), "lib")
        obj = out + ".o"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-c", src, "-o", obj],
                       check=True)
        subprocess.run(["g++", "-shared", "-o", out, obj, f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"],
                       check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--variants", default=",".join(map(str, VARIANTS)))
    args = ap.parse_args()

    path = build_variants()
    import numpy as np
    import torch

    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    lib = ctypes.CDLL(path)
    lib.voxvar_launch.argtypes = [ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    lib.voxvar_launch.restype = ctypes.c_int

    dev = torch.device("cuda:0")
    w = WORKLOADS[args.workload]
    B = args.batch
    layer = ProjectLayer(w.cfg("cuda:0"))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, B)).to(dev)
    meta = {"seq": [seq] * B}
    ref_cube, ref_xy = layer.forward_fused(hm, meta, cams, rt)
    grids = layer.sample_grid[seq].contiguous()
    B_, V, J, H, W = hm.shape
    X, Y, Z = w.voxels_per_axis
    stream = torch.cuda.current_stream().cuda_stream
    variants = [int(v) for v in args.variants.split(",")]
    cube = torch.empty_like(ref_cube)
    xy = torch.empty_like(ref_xy)
    ok = {}
    for var in variants:
        cube.fill_(-7.0)
        xy.fill_(-7.0)
        rc = lib.voxvar_launch(var, hm.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                               xy.data_ptr(), stream)
        torch.cuda.synchronize()
        assert rc == 0, (var, rc)
        good_xy = torch.equal(xy, ref_xy)
        good_cube = torch.equal(cube, ref_cube) if var % 10 == 1 else True
        ok[var] = good_xy and good_cube
        print(f"variant {var:3d}: xy {'ok' if good_xy else 'MISMATCH'} cube {'ok' if good_cube else 'MISMATCH'}",
              flush=True)

    def run(var):
        if var == 0:
            torch.ops.fvp.voxelize(hm, grids[:, 0].unsqueeze(0), None, X, Y, Z, True, True)
        else:
            lib.voxvar_launch(var, hm.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                              xy.data_ptr(), stream)

    # ---- channels-last experiment
    lib.voxvar_to_cl.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.voxvar_cl.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    cl = torch.empty((B, V, H, W, 16), device=dev)
    assert lib.voxvar_to_cl(hm.data_ptr(), B, V, J, H, W, cl.data_ptr(), 4, stream) == 0
    torch.cuda.synchronize()
    ref_cl = torch.nn.functional.pad(hm.permute(0, 1, 3, 4, 2), (0, 16 - J))
    print("to_cl exact:", torch.equal(cl, ref_cl), flush=True)
    for cols, cub in ((16, 1), (16, 0), (32, 1), (8, 1)):
        cube.fill_(-7.0)
        xy.fill_(-7.0)
        rc = lib.voxvar_cl(cols, cub, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                           xy.data_ptr(), stream)
        torch.cuda.synchronize()
        print(f"cl cols={cols} cube={cub}: rc={rc} xy {'ok' if torch.equal(xy, ref_xy) else 'MISMATCH'} cube "
              f"{'ok' if (not cub or torch.equal(cube, ref_cube)) else 'MISMATCH'}", flush=True)

    def run_cl(tag):
        if tag == "to_cl":
            lib.voxvar_to_cl(hm.data_ptr(), B, V, J, H, W, cl.data_ptr(), 4, stream)
        else:
            cols, cub = tag
            lib.voxvar_cl(cols, cub, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                          xy.data_ptr(), stream)

    # chunked: transpose + gather per chunk of frames with a reused (cache-resident) scratch
    def run_chunked(chunk):
        fb = V * J * H * W
        for c0 in range(0, B, chunk):
            nb = min(chunk, B - c0)
            lib.voxvar_to_cl(hm.data_ptr() + c0 * fb * 4, nb, V, J, H, W, cl.data_ptr(), 4, stream)
            lib.voxvar_cl(16, 1, cl.data_ptr(), nb, V, J, H, W, grids.data_ptr(), X, Y, Z,
                          cube.data_ptr() + c0 * J * X * Y * Z * 4, xy.data_ptr() + c0 * J * X * Y * 4, stream)
    for chunk in (1, 2, 4, 8, 16, 32, 256):
        cube.fill_(-7.0)
        run_chunked(chunk)
        torch.cuda.synchronize()
        assert torch.equal(cube, ref_cube) and torch.equal(xy, ref_xy), chunk
        ts = []
        for r in range(args.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run_chunked(chunk)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / args.iters)
        t = float(np.median(ts))
        print(f"chunked to_cl+gather chunk={chunk:3d}: {t:8.3f} ms {B / (t * 1e-3):10.0f} FPS", flush=True)

    lib.voxvar_cl2.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    for vc, cols in ((5, 16), (3, 16), (1, 16), (5, 8), (5, 4)):
        cube.fill_(-7.0)
        xy.fill_(-7.0)
        rc = lib.voxvar_cl2(vc, cols, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                            xy.data_ptr(), stream)
        torch.cuda.synchronize()
        good = torch.equal(xy, ref_xy) and torch.equal(cube, ref_cube)
        ts = []
        for r in range(args.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                lib.voxvar_cl2(vc, cols, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                               xy.data_ptr(), stream)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / args.iters)
        t = float(np.median(ts))
        print(f"cl2 vc={vc} cols={cols}: rc={rc} {'ok' if good else 'MISMATCH'} {t:8.3f} ms {B / (t * 1e-3):10.0f} FPS-eq",
              flush=True)

    lib.voxvar_cl3.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    for region, rx, ry in ((0, 1, 1), (1, 2, 4), (1, 4, 2), (1, 8, 1), (1, 1, 4 * 2)):
        cube.fill_(-7.0)
        xy.fill_(-7.0)
        rc = lib.voxvar_cl3(region, rx, ry, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                            xy.data_ptr(), stream)
        torch.cuda.synchronize()
        good = torch.equal(xy, ref_xy) and torch.equal(cube, ref_cube)
        ts = []
        for r in range(args.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                lib.voxvar_cl3(region, rx, ry, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z,
                               cube.data_ptr(), xy.data_ptr(), stream)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / args.iters)
        t = float(np.median(ts))
        print(f"cl3 region={region} {rx}x{ry}: rc={rc} {'ok' if good else 'MISMATCH'} {t:8.3f} ms "
              f"{B / (t * 1e-3):10.0f} FPS-eq", flush=True)

    lib.voxvar_cl4.argtypes = [ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    lib.voxvar_cl5.argtypes = lib.voxvar_cl4.argtypes
    for cols in (8, 16):
        cube.fill_(-7.0)
        xy.fill_(-7.0)
        rc = lib.voxvar_cl5(cols, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                            xy.data_ptr(), stream)
        torch.cuda.synchronize()
        good = torch.equal(xy, ref_xy) and torch.equal(cube, ref_cube)
        ts = []
        for r in range(args.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                lib.voxvar_cl5(cols, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                               xy.data_ptr(), stream)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / args.iters)
        t = float(np.median(ts))
        print(f"cl5 prefetch cols={cols}: rc={rc} {'ok' if good else 'MISMATCH'} {t:8.3f} ms "
              f"{B / (t * 1e-3):10.0f} FPS-eq", flush=True)
    for cols in (8, 16, 32):
        cube.fill_(-7.0)
        xy.fill_(-7.0)
        rc = lib.voxvar_cl4(cols, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                            xy.data_ptr(), stream)
        torch.cuda.synchronize()
        good = torch.equal(xy, ref_xy) and torch.equal(cube, ref_cube)
        ts = []
        for r in range(args.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                lib.voxvar_cl4(cols, cl.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                               xy.data_ptr(), stream)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / args.iters)
        t = float(np.median(ts))
        print(f"cl4 cam-outer cols={cols}: rc={rc} {'ok' if good else 'MISMATCH'} {t:8.3f} ms "
              f"{B / (t * 1e-3):10.0f} FPS-eq", flush=True)

    cl_tags = ["to_cl", (16, 1), (16, 0), (32, 1), (8, 1)]
    cl_times = {str(t): [] for t in cl_tags}
    for r in range(args.rounds):
        for tg in cl_tags:
            run_cl(tg)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run_cl(tg)
            e1.record()
            torch.cuda.synchronize()
            cl_times[str(tg)].append(e0.elapsed_time(e1) / args.iters)
    for tg in cl_tags:
        t = float(np.median(cl_times[str(tg)]))
        print(f"cl {str(tg):10s}: {t:8.3f} ms  {B / (t * 1e-3):10.0f} FPS-equivalent", flush=True)

    times = {v: [] for v in [0] + variants}
    for r in range(args.rounds):
        for var in [0] + variants:
            run(var)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run(var)
            e1.record()
            torch.cuda.synchronize()
            times[var].append(e0.elapsed_time(e1) / args.iters)
    per_frame = V * J * H * W * 4 + J * X * Y * Z * 4 + J * X * Y * 4
    for var in [0] + variants:
        t = float(np.median(times[var]))
        fps = B / (t * 1e-3)
        gbs = B * per_frame / (t * 1e-3) / 1e9
        print(f"variant {var:3d}: {t:8.3f} ms  {fps:10.0f} FPS  {gbs:7.1f} GB/s ({gbs / 80:.1f}% of 8 TB/s)"
              f"  min {min(times[var]):.3f}  {'' if var == 0 or ok[var] else 'WRONG'}", flush=True)


if __name__ == "__main__":
    main()
