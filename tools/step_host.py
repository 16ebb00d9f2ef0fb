#!/usr/bin/env python3
"""Where bench.py's step goes at small batches: host time
of each part of the step (vox, post = NMS + columns, collect = the proposal
all-gather, one-rank group) issued back to back without synchronising, the
GPU time of each part by HIP events, and the step rate; one JSON line.

    python3 tools/step_host.py [--workload c3] [--batch 8] [--steps 300]
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=300)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    import bench
    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    fd, path = tempfile.mkstemp(prefix="fvp_step_pg_")
    os.close(fd)
    dist.init_process_group("nccl", store=dist.FileStore(path, 1), rank=0, world_size=1, device_id=dev)
    w = WORKLOADS[a.workload]
    cams, seq = w.cameras()
    layer = ProjectLayer(w.cfg(str(dev)))
    layer.verbose = False
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, a.batch)).to(dev)
    meta = {"seq": [seq] * a.batch}
    X = w.voxels_per_axis[0]
    vox, post, collect = bench.step_functions(bench.HipCompute(layer, cams, rt), hm, meta, 0, X, X, 1, True, False,
                                              2, w.max_people)
    for _ in range(20):
        bench.run_step(vox, post, collect)
    torch.cuda.synchronize()
    host = {"vox": [], "post": [], "collect": []}
    gpu = {"vox": [], "post": [], "collect": []}
    evs = []
    for _ in range(a.steps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record()
        t0 = time.perf_counter()
        cube, xy = vox()
        t1 = time.perf_counter()
        e[1].record()
        vals, flat, cols = post(cube, xy)
        t2 = time.perf_counter()
        e[2].record()
        collect(vals, flat)
        t3 = time.perf_counter()
        e[3].record()
        host["vox"].append(t1 - t0)
        host["post"].append(t2 - t1)
        host["collect"].append(t3 - t2)
        evs.append(e)
    torch.cuda.synchronize()
    for e in evs:
        gpu["vox"].append(e[0].elapsed_time(e[1]) * 1e-3)
        gpu["post"].append(e[1].elapsed_time(e[2]) * 1e-3)
        gpu["collect"].append(e[2].elapsed_time(e[3]) * 1e-3)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        bench.run_step(vox, post, collect)
    torch.cuda.synchronize()
    step_us = (time.perf_counter() - t0) / a.steps * 1e6
    med = lambda xs: round(statistics.median(xs) * 1e6, 2)  # noqa: E731
    print(json.dumps({"workload": a.workload, "batch": a.batch, "step_us": round(step_us, 2),
                      "frames_per_s": round(a.batch / step_us * 1e6, 1),
                      "host_us": {k: med(v) for k, v in host.items()},
                      "gpu_us": {k: med(v) for k, v in gpu.items()}}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
