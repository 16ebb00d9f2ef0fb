#!/usr/bin/env python3
"""Layout of chunk k+1 under the gather of chunk k, on the product kernels
(round 5).  The layout pass is fvp_nchw_to_nhwc into a [C][V][H][W][16]
buffer (the fp32 channels-last table, heatmaps_to_cl_kernel),
the gather is fvp_voxelize_cl on that buffer (the chunked gather's kernel).
256 C2 frames read from HBM in chunks of C: (a) sequential on one stream;
(b) two streams, double-buffered, events both ways (optionally the layout
stream at high priority).  Cubes are checked against the product op.

    [FVP_LIB=ab_libs/<lib>.so] python3 tools/overlap_probe2.py [--chunks 4,8,12] [--reps 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="4,8,12")
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--schedules", default="sequential,overlapped,overlapped_hi")
    args = ap.parse_args()
    import torch

    from fvp import _lib, geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    L = _lib.load()
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
    ref_cube, ref_xy = layer.forward_fused(hm, {"seq": [seq] * F}, cams, rt)
    frame_elems = V * J * Hd * Wd
    s_main = torch.cuda.current_stream(dev)
    s_lay = torch.cuda.Stream(dev)
    s_lay_hi = torch.cuda.Stream(dev, priority=-1)
    cube = torch.empty_like(ref_cube)
    xy = torch.empty_like(ref_xy)
    csz, xsz = J * X * Y * Z, J * X * Y

    for C in [int(c) for c in args.chunks.split(",")]:
        n = (F + C - 1) // C  # (the last chunk may be short)
        bufs = [torch.empty((C, V, Hd, Wd, 16), device=dev) for _ in range(2)]

        def nb(k):
            return min(C, F - k * C)

        def layout(k, buf, stream):
            _lib.check(L.fvp_nchw_to_nhwc(hm.data_ptr() + k * C * frame_elems * 4, nb(k) * V, J, Hd, Wd, 16,
                                          buf.data_ptr(), stream.cuda_stream), "layout")

        def gather(k, buf, stream):
            _lib.check(L.fvp_voxelize_cl(buf.data_ptr(), 16, nb(k), V, J, Hd, Wd, grids.data_ptr(), None, X, Y, Z,
                                         cube.data_ptr() + k * C * csz * 4, xy.data_ptr() + k * C * xsz * 4,
                                         stream.cuda_stream), "gather")

        def sequential():
            for k in range(n):
                layout(k, bufs[0], s_main)
                gather(k, bufs[0], s_main)

        ready = [torch.cuda.Event() for _ in range(n)]
        free = [torch.cuda.Event() for _ in range(n)]

        def overlapped_on(sl):
            def run():
                sl.wait_stream(s_main)
                for k in range(n):
                    with torch.cuda.stream(sl):
                        if k >= 2:
                            sl.wait_event(free[k - 2])  # the gather of chunk k-2 has read this buffer
                        layout(k, bufs[k % 2], sl)
                        ready[k].record(sl)
                    s_main.wait_event(ready[k])
                    gather(k, bufs[k % 2], s_main)
                    free[k].record(s_main)
                s_main.wait_stream(sl)
            return run

        table = {"sequential": sequential, "overlapped": overlapped_on(s_lay), "overlapped_hi": overlapped_on(s_lay_hi)}
        for name in args.schedules.split(","):
            fn = table[name]
            cube.zero_()
            fn()
            torch.cuda.synchronize()
            assert torch.equal(cube, ref_cube) and torch.equal(xy, ref_xy), name
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s_main)
            for _ in range(args.reps):
                fn()
            e1.record(s_main)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            print(json.dumps({"lib": os.environ.get("FVP_LIB", "libfvp.so"), "chunk_frames": C, "schedule": name,
                              "ms_per_256_frames": round(ms * 256 / F, 4), "frames_per_s": round(F / (ms * 1e-3), 1),
                              "hbm_frac_equiv": round(F * 17.28e6 / (ms * 1e-3) / 8e12, 4)}), flush=True)
        del bufs


if __name__ == "__main__":
    main()
