#!/usr/bin/env python3
"""One-frame (B=1) latency of the C2 hot-path step (voxelize -> xy -> NMS
top-K with the fused column gather, as bench.py's latency_b1 lines) under
several ways of waiting for the result: device-wide synchronize (bench.py's
line), the launch stream's synchronize, an event synchronize, and a spin on
event.query().  Median of --iters host wall times each.

    python tools/b1_latency.py [--workload c2] [--iters 200]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch

    from fvp import geometry, synthetic
    from fvp.graphs import CapturedStep
    from fvp.project_whole import ProjectLayer
    from fvp.proposal import nms2D_columns
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    w = WORKLOADS[args.workload]
    cams, seq = w.cameras()
    K, root = w.max_people, 2
    layer = ProjectLayer(w.cfg(str(dev)))
    layer.verbose = False
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    hm1 = torch.from_numpy(synthetic.gaussian_heatmaps(w, 1)).to(dev)
    meta1 = {"seq": [seq]}

    def step1():
        cube, xy = layer.forward_fused(hm1, meta1, cams, rt, want_cube=True, want_xy=True)
        return nms2D_columns(xy[:, root:root + 1], K, cube)[3]

    stream = torch.cuda.current_stream(dev)
    ev = torch.cuda.Event()

    def timed(run, wait):
        for _ in range(10):
            run()
            wait()
        lat = []
        for _ in range(args.iters):
            t1 = time.perf_counter()
            run()
            wait()
            lat.append((time.perf_counter() - t1) * 1e3)
        return round(float(np.median(lat)), 4), round(float(np.percentile(lat, 90)), 4)

    def ev_sync():
        ev.record(stream)
        ev.synchronize()

    def ev_spin():
        ev.record(stream)
        while not ev.query():
            pass

    out = {"workload": w.name, "iters": args.iters}
    out["eager_device_sync_ms"] = timed(step1, torch.cuda.synchronize)
    cap = CapturedStep(step1)
    out["graph_device_sync_ms"] = timed(cap.replay, torch.cuda.synchronize)
    out["graph_stream_sync_ms"] = timed(cap.replay, stream.synchronize)
    out["graph_event_sync_ms"] = timed(cap.replay, ev_sync)
    out["graph_event_spin_ms"] = timed(cap.replay, ev_spin)
    # the same step through the C ABI directly (what a C/C++ host would bind,
    # INTEGRATION.md): two calls per frame -- fvp_voxelize (layout + gather)
    # and fvp_nms_topk_columns -- on preallocated buffers, then the stream sync
    from fvp import _lib
    X, Y, Z = w.voxels_per_axis
    B, V, J, H, W = hm1.shape
    grids, _ = layer._grids_for_batch(hm1, meta1, cams, rt)
    L = _lib.load()
    ws_bytes = L.fvp_voxelize_workspace_bytes(B, V, J, H, W)
    ws = torch.empty((ws_bytes + 3) // 4, device=dev)
    cube = torch.empty((B, J, X, Y, Z), device=dev)
    xy = torch.empty((B, J, X, Y), device=dev)
    vals = torch.empty((B, K), device=dev)
    flat = torch.empty((B, K), dtype=torch.int64, device=dev)
    kxy = torch.empty((B, K, 2), dtype=torch.int64, device=dev)
    cols = torch.empty((B, K, J, Z), device=dev)
    st = stream.cuda_stream
    a_vox = (hm1.data_ptr(), B, V, J, H, W, grids.data_ptr(), None, X, Y, Z, cube.data_ptr(), xy.data_ptr(),
             ws.data_ptr(), ws_bytes, st)
    a_nms = (xy.data_ptr() + root * X * Y * 4, B, X, Y, J * X * Y, K, vals.data_ptr(), flat.data_ptr(),
             kxy.data_ptr(), cube.data_ptr(), J, Z, cols.data_ptr(), st)
    f_vox, f_nms = L.fvp_voxelize, L.fvp_nms_topk_columns

    def abi_step():
        f_vox(*a_vox)
        f_nms(*a_nms)

    abi_step()
    torch.cuda.synchronize()
    ref = step1()
    torch.cuda.synchronize()
    out["abi_matches_op_path"] = bool(torch.equal(cols, ref))
    out["abi_direct_stream_sync_ms"] = timed(abi_step, stream.synchronize)
    out["note"] = "(median, p90) host wall ms per step, inputs resident on the GPU"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
