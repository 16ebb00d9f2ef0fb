#!/usr/bin/env python3
"""Where the registered-op (dispatcher) call of fvp::person_planes spends its host
time on bench_jln.py's C3 setup: torch.profiler's CPU table of one call through
the dispatcher and one through the eager fast path, and host times of variants."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    import numpy as np
    import torch

    from fvp import geometry, ops, synthetic
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
    meta = {"seq": [seq] * F}
    props = allp.reshape(-1, 7).contiguous()
    frame_of = torch.arange(F, dtype=torch.int32, device=dev).repeat_interleave(P)
    grid = layer._seq_grid(hm, 0, meta, cams, rt)
    a = layer._args()

    def host_us(fn, n=20):
        tot = 0.0
        for _ in range(n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            tot += time.perf_counter() - t0
        torch.cuda.synchronize()
        return tot / n * 1e6

    small = hm[:1].contiguous()
    cases = {
        "fast path": lambda: ops.person_planes(hm, grid, props, frame_of, *a, False, True),
        "dispatcher": lambda: ops.person_planes.op(hm, grid, props, frame_of, *a, False, True),
        "torch.ops.fvp.person_planes.default": lambda: torch.ops.fvp.person_planes.default(hm, grid, props, frame_of, *a, False, True),
        "dispatcher, 1 frame x 1 proposal": lambda: ops.person_planes.op(small, grid, props[:1], frame_of[:1] * 0, *a, False, True),
        "fast path, 1 frame x 1 proposal": lambda: ops.person_planes(small, grid, props[:1], frame_of[:1] * 0, *a, False, True),
    }
    for name, fn in cases.items():
        fn()
        print(f"{name}: {host_us(fn):.1f} us host", flush=True)
    from torch.profiler import ProfilerActivity, profile
    for name in ("dispatcher", "fast path"):
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            cases[name]()
            torch.cuda.synchronize()
        print(f"== {name}", flush=True)
        print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25), flush=True)


if __name__ == "__main__":
    main()
