#!/usr/bin/env python3
"""Can the layout pass of frame chunk k+1 run under the gather of chunk k?
(tools/gather_probe.hip: layout_probe mode 0 = the shipped heatmaps_to_cl
kernel, gather_probe FULL2 = the shipped gather with its vector epilogue.)

256 C2 frames (2.36 GB of planar heatmaps, so the layout reads HBM as in
bench.py) in chunks of C frames, timed with HIP events around the whole
batch: (a) sequential on one stream, as fvp_voxelize runs; (b) two streams,
layout into a double-buffered channels-last workspace one chunk ahead,
events for both dependencies.  Prints one JSON line per (C, schedule).

    python tools/overlap_probe.py [--chunks 4,8] [--reps 3]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd"), os.path.join(REPO, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="4,8")
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--layout-blocks", default="0", help="0 = the shipped launch; n = grid-stride over n blocks")
    ap.add_argument("--cols", default="16", help="gather columns per block (the product: 16 at C2)")
    ap.add_argument("--schedules", default="sequential,overlapped")
    args = ap.parse_args()
    import gather_probe
    path = gather_probe.build()
    import torch

    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    lib = ctypes.CDLL(path)
    lib.gather_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int] * 10 + [ctypes.c_void_p]
    lib.layout_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int] * 5 + [ctypes.c_void_p]
    lib.layout_stride_probe.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 6 + [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    w = WORKLOADS["c2"]
    cams, seq = w.cameras()
    V, J = len(cams[seq]), w.num_joints
    X, Y, Z = w.voxels_per_axis
    Wd, Hd = w.heatmap_size
    F = args.frames
    layer = ProjectLayer(w.cfg("cuda:0"))
    layer.verbose = False
    layer.on_the_fly = False
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, F)).to(dev)
    grids, _ = layer._grids_for_batch(hm[:1], {"seq": [seq]}, cams, rt)
    frame_elems = V * J * Hd * Wd
    s_main = torch.cuda.current_stream(dev)
    s_lay = torch.cuda.Stream(dev)
    sink = torch.zeros(64 << 20, device=dev)

    lay_blocks = [0]
    cols = [16]

    def layout(k, C, buf, stream):
        src = hm.data_ptr() + k * C * frame_elems * 4
        if lay_blocks[0]:
            rc = lib.layout_stride_probe(src, buf.data_ptr(), C, V, J, Hd, Wd, lay_blocks[0], stream.cuda_stream)
        else:
            rc = lib.layout_probe(0, src, buf.data_ptr(), C, V, J, Hd, Wd, stream.cuda_stream)
        assert rc == 0, rc

    def gather(C, buf, cube, xy, stream):
        rc = lib.gather_probe(9, buf.data_ptr(), grids.data_ptr(), cube.data_ptr(), xy.data_ptr(), sink.data_ptr(),
                              C, V, J, Hd, Wd, X, Y, Z, cols[0], 16, stream.cuda_stream)
        assert rc == 0, rc

    for C, lb, nc in [(int(c), int(b), int(k)) for c in args.chunks.split(",") for b in args.layout_blocks.split(",")
                      for k in args.cols.split(",")]:
        lay_blocks[0], cols[0] = lb, nc
        n = F // C
        bufs = [torch.empty((C, V, Hd * Wd, 16), device=dev) for _ in range(2)]
        cube = torch.empty((F, J, X, Y, Z), device=dev)
        xy = torch.empty((F, J, X, Y), device=dev)
        csz, xsz = J * X * Y * Z, J * X * Y

        def cube_k(k):
            return cube.view(-1)[k * C * csz:(k + 1) * C * csz], xy.view(-1)[k * C * xsz:(k + 1) * C * xsz]

        def sequential():
            for k in range(n):
                layout(k, C, bufs[0], s_main)
                cb, xb = cube_k(k)
                gather(C, bufs[0], cb, xb, s_main)

        ready = [torch.cuda.Event() for _ in range(n)]
        free = [torch.cuda.Event() for _ in range(n)]

        def overlapped():
            s_lay.wait_stream(s_main)
            for k in range(n):
                with torch.cuda.stream(s_lay):
                    if k >= 2:
                        s_lay.wait_event(free[k - 2])  # the gather of chunk k-2 has read this buffer
                    layout(k, C, bufs[k % 2], s_lay)
                    ready[k].record(s_lay)
                s_main.wait_event(ready[k])
                cb, xb = cube_k(k)
                gather(C, bufs[k % 2], cb, xb, s_main)
                free[k].record(s_main)
            s_main.wait_stream(s_lay)

        ref = None
        scheds = [(n_, {"sequential": sequential, "overlapped": overlapped}[n_]) for n_ in args.schedules.split(",")]
        for name, fn in scheds + scheds:
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = cube.clone()
            else:
                assert torch.equal(cube, ref), name
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s_main)
            for _ in range(args.reps):
                fn()
            e1.record(s_main)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            print(json.dumps({"chunk_frames": C, "cols": nc, "layout_blocks": lb or "shipped", "schedule": name, "ms_per_256_frames": round(ms * 256 / F, 4),
                              "frames_per_s": round(F / (ms * 1e-3), 1)}), flush=True)
        del bufs, cube, xy, ref


if __name__ == "__main__":
    main()
