#!/usr/bin/env python3
"""Host overhead of the torch.ops.fvp custom-op dispatch vs calling the op's
implementation directly (eager), on a tiny NMS and a per-frame JLN planes call."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    import torch

    from fvp import ops

    dev = torch.device("cuda:0")
    side = int(os.environ.get("NMS_SIDE", "80"))
    prob = torch.rand((1, 1, side, side), device=dev)

    def bench(fn, n=2000):
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    raw = ops.nms_topk.impl
    K = int(os.environ.get("NMS_K", "10"))
    print(f"nms_topk via dispatcher {bench(lambda: ops.nms_topk.op(prob, K)):.1f} us/call, "
          f"direct {bench(lambda: raw(prob, K)):.1f} us/call", flush=True)


if __name__ == "__main__":
    main()
