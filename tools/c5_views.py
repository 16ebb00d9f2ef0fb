#!/usr/bin/env python3
"""C5 geometry with the first V ring cameras: voxelize time per voxel-camera
as V grows (does the per-camera cost rise with the number of camera tables
live at once?).

    python tools/c5_views.py [--views 4,8,16,31] [--batch 8]
"""
from __future__ import annotations

import argparse
import dataclasses
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", default="4,8,16,31")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--workload", default="c5")
    ap.add_argument("--otf", choices=["auto", "1", "0"], default="auto")
    args = ap.parse_args()

    import torch

    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    base = WORKLOADS[args.workload]
    for V in map(int, args.views.split(",")):
        w = dataclasses.replace(base, extra={**base.extra, "views": V})
        cams, seq = w.cameras()
        layer = ProjectLayer(w.cfg(str(dev)))
        layer.verbose = False
        if args.otf != "auto":
            layer.on_the_fly = args.otf == "1"
        rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
        hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, args.batch)).to(dev)
        if w.dtype == "float16":
            hm = hm.half()
        meta = {"seq": [seq] * args.batch}
        layer.prepare(hm, meta, cams, rt)
        for _ in range(2):
            layer.forward_fused(hm, meta, cams, rt, want_cube=True, want_xy=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.iters):
            layer.forward_fused(hm, meta, cams, rt, want_cube=True, want_xy=True)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        vc = args.batch * w.num_voxels * V
        print(f"V={V:3d} otf={layer._project_on_the_fly(V)} {ms:8.3f} ms / {args.batch} frames  "
              f"{ms * 1e6 / vc:.4f} ns per voxel-camera", flush=True)
        del layer, hm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
