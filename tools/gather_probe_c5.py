#!/usr/bin/env python3
"""Replay probe of the C5 gather (tools/gather_probe.hip probe_c5_kernel;
VERDICT r2 item 3): one 2-frame chunk of the 31-camera ring, 160x160x64,
fp16 heatmaps, on-the-fly projection, the frame-interleaved fp16 pixel-pair
table the product's layout pass leaves in the workspace.  Each mode is timed
with HIP events on the launch stream (mean of --iters launches after warm-up)
next to the product's gather.  Prints one JSON line per mode.

    python tools/gather_probe_c5.py [--iters 10]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd"), os.path.join(REPO, "tools")]

MODES = {"FULL": 0, "TAPS": 1, "TAPS_ALL_OOB": 4, "NO_TAPS": 5, "NOSTORE": 8, "TAPS_HALF": 12, "PROJ": 14,
         "STORE_PLAIN": 16, "STORE_SMALL": 17, "FULL_PASS": 18}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--modes", default=",".join(MODES))
    args = ap.parse_args()
    import gather_probe
    path = gather_probe.build()
    import torch

    from fvp import _lib, geometry, synthetic
    from fvp.ops import _f3, _i3
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    lib = ctypes.CDLL(path)
    lib.gather_probe_c5.argtypes = ([ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.POINTER(_lib.GridSpec),
                                    ctypes.POINTER(_lib.ImageSpec)] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 10
                                    + [ctypes.c_void_p])
    dev = torch.device("cuda:0")
    w = WORKLOADS["c5"]
    cams, seq = w.cameras()
    V, J = len(cams[seq]), w.num_joints
    X, Y, Z = w.voxels_per_axis
    Wd, Hd = w.heatmap_size
    B = 2
    layer = ProjectLayer(w.cfg("cuda:0"))
    layer.verbose = False
    layer.on_the_fly = True
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, B)).to(dev).half()
    meta = {"seq": [seq] * B}
    cam_t, _ = layer._cams_for_batch(hm, meta, cams)
    start, end, center, nb = layer.grid_spec()
    gs = _lib.GridSpec(_f3(start), _f3(end), _f3(center), _i3(nb))
    im = _lib.ImageSpec(float(max(w.ori_image_size)), float(w.image_size[0]), float(w.image_size[1]), Wd, Hd)
    L = _lib.load()
    ws_bytes = L.fvp_voxelize_f16_workspace_bytes(B, V, J, Hd, Wd)
    ws = torch.zeros((ws_bytes + 3) // 4, device=dev)
    ref_cube = torch.empty((B, J, X, Y, Z), device=dev)
    ref_xy = torch.empty((B, J, X, Y), device=dev)
    cube = torch.empty_like(ref_cube)
    xy = torch.empty_like(ref_xy)
    sink = torch.zeros(64 << 20, device=dev)
    stream = torch.cuda.current_stream(dev)

    def product():
        _lib.call("fvp_voxelize_cams", hm.data_ptr(), 1, B, V, J, Hd, Wd, cam_t.data_ptr(), None, rt.data_ptr(), gs,
                  im, ref_cube.data_ptr(), ref_xy.data_ptr(), ws.data_ptr(), ws_bytes, stream.cuda_stream)

    cols, band = 4, 16  # the product's C5 launch (fvp_voxelize.hip gather_cfg: 256-voxel blocks)

    def probe(mode):
        rc = lib.gather_probe_c5(mode, ws.data_ptr(), cam_t.data_ptr(), rt.data_ptr(), ctypes.byref(gs),
                                 ctypes.byref(im), cube.data_ptr(), xy.data_ptr(), sink.data_ptr(), B, V, J, Hd, Wd,
                                 X, Y, Z, cols, band, stream.cuda_stream)
        assert rc == 0, rc

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.iters):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.iters

    product()  # leaves the chunk's pair table in ws
    torch.cuda.synchronize()
    print(json.dumps({"mode": "product fvp_voxelize_cams (layout + gather)", "us": round(timed(product), 1),
                      "frames": B, "workload": "c5"}), flush=True)
    taps = B * X * Y * Z * V
    for name in args.modes.split(","):
        if name in ("FULL", "STORE_PLAIN", "FULL_PASS"):
            cube.zero_()
            probe(MODES[name])
            torch.cuda.synchronize()
            assert torch.equal(cube, ref_cube) and torch.equal(xy, ref_xy), "FULL differs from fvp_voxelize_cams"
        us = timed(lambda: probe(MODES[name]))
        print(json.dumps({"mode": name, "us": round(us, 1), "frames": B,
                          "ns_per_voxel_camera_frame": round(us * 1e3 / taps, 5)}), flush=True)


if __name__ == "__main__":
    main()
