#!/usr/bin/env python3
"""Fixed costs under the B=1 latency line: host time of a replayed hipGraph of
1 / 3 trivial kernels (graph launch + synchronise), and the float4 copy of one
C2 frame's heatmaps (9.2 MB) as the floor of a one-frame layout pass.

    python tools/latency_floor.py
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def main():
    import numpy as np
    import torch
    from fvp import _lib
    from fvp.graphs import CapturedStep

    dev = torch.device("cuda:0")
    x = torch.zeros(64, device=dev)
    src = torch.rand(5 * 15 * 128 * 240, device=dev)
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream().cuda_stream

    def host_ms(fn, n=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        lat = []
        for _ in range(n):
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t) * 1e3)
        return round(float(np.median(lat)), 4)

    def dev_ms(fn, n=50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / n, 5)

    def copy():
        _lib.call("fvp_copy_f4", src.data_ptr(), dst.data_ptr(), src.numel() * 4, torch.cuda.current_stream().cuda_stream)

    one = CapturedStep(lambda: x.add_(1.0))
    three = CapturedStep(lambda: (x.add_(1.0), x.add_(1.0), x.add_(1.0)))
    cp = CapturedStep(copy)
    del stream
    out = {"graph_1_trivial_kernel_ms": host_ms(one.replay), "graph_3_trivial_kernels_ms": host_ms(three.replay),
           "eager_1_trivial_kernel_ms": host_ms(lambda: x.add_(1.0)),
           "copy_9p2MB_device_ms": dev_ms(copy), "copy_9p2MB_graph_host_ms": host_ms(cp.replay)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
