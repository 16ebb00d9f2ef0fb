#!/usr/bin/env python3
"""One-frame step latency (C2 geometry): voxelize (cube + xy) -> NMS top-K +
z-columns, eager and replayed from a hipGraph; run under rocprofv3
--kernel-trace --stats for the per-kernel split.

    python tools/latency_b1.py [--workload c2] [--layout planar|channels-last] [--iters 200]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--layout", choices=["planar", "channels-last"], default="planar")
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch

    from fvp import geometry, synthetic
    from fvp.graphs import CapturedStep
    from fvp.heatmaps import ChannelsLastHeatmaps
    from fvp.project_whole import ProjectLayer
    from fvp.proposal import nms2D_columns
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    w = WORKLOADS[args.workload]
    layer = ProjectLayer(w.cfg(str(dev)))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float32, device=dev)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 1)).to(dev)
    if w.dtype == "float16":  # C5: fp16 heatmaps, as bench.py
        hm = hm.half()
    J = w.num_joints
    if args.layout == "channels-last":
        t = torch.zeros(hm.shape[:2] + hm.shape[3:] + (16 * ((J + 15) // 16),), device=dev)
        t[..., :J] = hm.permute(0, 1, 3, 4, 2)
        hm = ChannelsLastHeatmaps(t, J)
    meta = {"seq": [seq]}
    root = 2 if J > 2 else 0

    def step():
        cube, xy = layer.forward_fused(hm, meta, cams, rt)
        return nms2D_columns(xy[:, root:root + 1], w.max_people, cube)

    step()
    torch.cuda.synchronize()
    out = {}
    for name, fn in (("eager", step), ("graph", CapturedStep(step).replay)):
        fn()
        torch.cuda.synchronize()
        lat = []
        for _ in range(args.iters):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t0) * 1e3)
        out[f"{name}_ms_median"] = round(float(np.median(lat)), 4)
        out[f"{name}_ms_p10"] = round(float(np.percentile(lat, 10)), 4)
    print(json.dumps({"workload": args.workload, "layout": args.layout, **out}))


if __name__ == "__main__":
    main()
