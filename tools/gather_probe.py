#!/usr/bin/env python3
"""Replay probe of the C2 voxelize gather (tools/gather_probe.hip).

One 8-frame C2 chunk (Shelf cameras, 80x80x20, J=15) in the channels-last
layout the gather reads, the product's packed grid and launch shape; each
probe mode is timed with HIP events on the launch stream (mean of --iters
launches after warm-up), next to the product's fvp_voxelize_cl on the same
inputs.  Prints one JSON line per mode.

    python tools/gather_probe.py [--frames 8] [--iters 50] [--workload c2]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]

MODES = {"FULL": 0, "TAPS": 1, "TAPS_L1": 2, "TAPS_SKIP_OOB": 3, "TAPS_ALL_OOB": 4, "NO_TAPS": 5, "TAPS_2ROW": 6,
         "CAM_OUTER": 7, "NOSTORE": 8, "FULL2": 9, "STORES_ONLY": 10, "TAPS_L2": 11,
         "TAPS_HALF": 12, "TAPS_L1_HALF": 13}
EXACT = ("FULL", "CAM_OUTER", "FULL2")  # modes that must reproduce the product's cube and xy


def build():
    import torch

    src = os.path.join(REPO, "tools", "gather_probe.hip")
    out = os.path.join(REPO, "tools", "bin", "libgprobe.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    deps = [src, os.path.join(REPO, "faster-voxelpose_amd", "csrc", "fvp_layout.h"),
            os.path.join(REPO, "faster-voxelpose_amd", "csrc", "fvp_device.h")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        tl = os.path.join(os.path.dirname(torch.__file__), "lib")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-c", src, "-o", out + ".o"],
                       check=True)
        subprocess.run(["g++", "-shared", "-o", out, out + ".o", f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"],
                       check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--modes", default=",".join(MODES))
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--lds-tiles", default="8x8,4x8,8x4,4x4,8x10,10x8", help="LDS prototype tiles (TXxTY columns)")
    args = ap.parse_args()
    path = build()
    if args.build_only:
        return
    import torch

    from fvp import geometry, ops, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    lib = ctypes.CDLL(path)
    lib.gather_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int] * 10 + [ctypes.c_void_p]
    lib.lds_gather_probe.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 10 + [ctypes.c_void_p]
    lib.layout_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int] * 5 + [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    w = WORKLOADS[args.workload]
    cams, seq = w.cameras()
    V, J = len(cams[seq]), w.num_joints
    X, Y, Z = w.voxels_per_axis
    Wd, Hd = w.heatmap_size
    B = args.frames
    layer = ProjectLayer(w.cfg("cuda:0"))
    layer.verbose = False
    layer.on_the_fly = False
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, B)).to(dev)
    meta = {"seq": [seq] * B}
    grids, _ = layer._grids_for_batch(hm, meta, cams, rt)
    hcl = torch.zeros((B, V, Hd, Wd, 16), device=dev)
    hcl[..., :J] = hm.permute(0, 1, 3, 4, 2)
    cube = torch.empty((B, J, X, Y, Z), device=dev)
    xy = torch.empty((B, J, X, Y), device=dev)
    sink = torch.zeros(64 << 20, device=dev)
    stream = torch.cuda.current_stream(dev)
    cols, band = 16, 16  # the launch at C2 / C3 when the probe was written (the product now takes 8: gather_cfg)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.iters):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.iters

    def probe(mode):
        rc = lib.gather_probe(mode, hcl.data_ptr(), grids.data_ptr(), cube.data_ptr(), xy.data_ptr(), sink.data_ptr(),
                              B, V, J, Hd, Wd, X, Y, Z, cols, band, stream.cuda_stream)
        assert rc == 0, rc

    ref_cube, ref_xy = ops.voxelize_cl(hcl, J, grids, None, X, Y, Z, True, True)
    probe(MODES["FULL"])
    torch.cuda.synchronize()
    assert torch.equal(cube, ref_cube) and torch.equal(xy, ref_xy), "FULL probe differs from fvp_voxelize_cl"
    us = timed(lambda: ops.voxelize_cl(hcl, J, grids, None, X, Y, Z, True, True))
    taps = B * X * Y * Z * V
    print(json.dumps({"mode": "product fvp_voxelize_cl", "us": round(us, 2), "frames": B, "workload": w.name}),
          flush=True)
    # layout-pass candidates (tools/gather_probe.hip layout_probe): same output bytes
    outs = {}
    for lm, lname in ((0, "LAYOUT_T shipped"), (1, "LAYOUT_C via LDS"), (2, "LAYOUT_S strided store")):
        dst = torch.full((B, V, Hd * Wd, 16), 7.0, device=dev)

        def lay():
            rc = lib.layout_probe(lm, hm.data_ptr(), dst.data_ptr(), B, V, J, Hd, Wd, stream.cuda_stream)
            assert rc == 0, rc
        lay()
        torch.cuda.synchronize()
        outs[lm] = dst.clone()
        us = timed(lay)
        print(json.dumps({"mode": lname, "us": round(us, 2), "frames": B,
                          "same_as_shipped": bool(torch.equal(outs[lm], outs[0]))}), flush=True)
    del outs
    # the headline op on the same frames: planar heatmaps, layout pass + gather
    us = timed(lambda: ops.voxelize(hm, grids, None, X, Y, Z, True, True))
    print(json.dumps({"mode": "product fvp_voxelize (planar: layout + gather)", "us": round(us, 2), "frames": B}),
          flush=True)
    for tile in [t for t in args.lds_tiles.split(",") if t]:
        TX, TY = map(int, tile.split("x"))

        def lds():
            rc = lib.lds_gather_probe(hm.data_ptr(), grids.data_ptr(), cube.data_ptr(), xy.data_ptr(), B, V, J, Hd,
                                      Wd, X, Y, Z, TX, TY, stream.cuda_stream)
            assert rc == 0, (tile, rc)
        cube.zero_()
        xy.zero_()
        lds()
        torch.cuda.synchronize()
        same = torch.equal(cube, ref_cube) and torch.equal(xy, ref_xy)
        ndiff = int((cube != ref_cube).sum())
        us = timed(lds)
        print(json.dumps({"mode": f"LDS planar {tile}", "us": round(us, 2), "frames": B, "bit_exact": same,
                          "cube_values_differing": ndiff}), flush=True)
    for name in args.modes.split(","):
        if name in EXACT:
            cube.zero_()
            probe(MODES[name])
            torch.cuda.synchronize()
            assert torch.equal(cube, ref_cube) and torch.equal(xy, ref_xy), f"{name} differs from fvp_voxelize_cl"
        us = timed(lambda: probe(MODES[name]))
        print(json.dumps({"mode": name, "us": round(us, 2), "frames": B,
                          "ns_per_voxel_camera": round(us * 1e3 / taps, 5),
                          "tap_GBps_fp32_256B": round(taps * 256 / (us * 1e-6) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
