#!/usr/bin/env python3
"""Host time of ProjectLayer.forward_batch's pieces on bench_jln.py's C3 setup
(32 frames x 10 proposals): each piece timed with perf_counter on an idle GPU
(synchronised before every iteration), mean over --iters, in microseconds."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch

    from fvp import _lib, geometry, ops, synthetic
    from fvp.project_individual import ProjectLayer
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    w = WORKLOADS["c3"]
    cams, seq = w.cameras()
    layer = ProjectLayer(w.cfg("cuda:0"))
    layer.verbose = False
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    F, P = 32, 10
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, F)).to(dev)
    allp = torch.stack([torch.from_numpy(np.resize(synthetic.proposals_for_frame(w, f, 4), (P, 7))) for f in range(F)]).to(dev)
    mask = torch.ones((F, P), dtype=torch.bool, device=dev)
    meta = {"seq": [seq] * F}
    layer.forward_batch(hm, meta, allp, mask, cams, rt)
    torch.cuda.synchronize()
    idx = mask.nonzero()
    frame_of = idx[:, 0].to(torch.int32)
    props = allp[idx[:, 0], idx[:, 1]]
    grid = layer._seq_grid(hm, 0, meta, cams, rt)
    a = layer._args()
    ws_bytes = _lib.load().fvp_person_workspace_bytes(*hm.shape)
    sel = ops.mask_select(mask, allp)
    from fvp.heatmaps import channels_last_of
    pieces = {
        "forward_batch (launch, after the sync)": lambda: layer.forward_batch(hm, meta, allp, mask, cams, rt),
        "forward_batch(sel=mask_select(...)) (the JLN's path)":
            lambda: layer.forward_batch(hm, meta, allp, mask, cams, rt, idx=sel[0], sel=sel),
        "ops.mask_select (incl. its sync)": lambda: ops.mask_select(mask, allp),
        "ops.forward_only": lambda: ops.forward_only(hm, allp),
        "channels_last_of": lambda: channels_last_of(hm),
        "layer._otf": lambda: layer._otf(hm.shape[1]),
        "mask.nonzero()": lambda: mask.nonzero(),
        "frame_of = idx[:,0].to(int32)": lambda: idx[:, 0].to(torch.int32),
        "props = allp[idx[:,0], idx[:,1]]": lambda: allp[idx[:, 0], idx[:, 1]],
        "layer._run": lambda: layer._run(hm, 0, meta, cams, rt, props, frame_of, False, True),
        "layer._seq_grid": lambda: layer._seq_grid(hm, 0, meta, cams, rt),
        "layer._args": lambda: layer._args(),
        "ops.person_planes (fast path)": lambda: ops.person_planes(hm, grid, props, frame_of, *a, False, True),
        "ops.person_planes.op (dispatcher)": lambda: ops.person_planes.op(hm, grid, props, frame_of, *a, False, True),
        "workspace_bytes query": lambda: _lib.load().fvp_person_workspace_bytes(*hm.shape),
        "PersonSpec(...)": lambda: _lib.PersonSpec(ops._i3(a[0]), ops._f3(a[1]), ops._f3(a[2]), ops._f3(a[3]),
                                                   ops._f3(a[4]), ops._i3(a[5])),
        "4 x torch.empty": lambda: [torch.empty((3 * 320, 15, 64, 64), device=dev), torch.empty((0,), device=dev),
                                    torch.empty((320, 3), device=dev), torch.empty(((ws_bytes + 3) // 4,), device=dev)],
    }
    for name, fn in pieces.items():
        tot = 0.0
        for _ in range(args.iters):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            tot += time.perf_counter() - t0
        torch.cuda.synchronize()
        print(json.dumps({"piece": name, "host_us": round(tot / args.iters * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
