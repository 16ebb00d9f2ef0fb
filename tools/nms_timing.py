#!/usr/bin/env python3
"""Kernel-time breakdown of fvp_nms_topk: launches over K and map size, timed
with HIP events around 200 back-to-back launches (run under rocprofv3
--kernel-trace --stats for per-kernel durations)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))

import torch  # noqa: E402

from fvp import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    res = []
    for (X, Y) in [(80, 80), (40, 40), (20, 20), (128, 128)]:
        for B in (1, 8):
            smooth = torch.nn.functional.avg_pool2d(torch.rand((B, 1, X + 8, Y + 8), generator=g), 9, 1)
            for kind, m in (("noise", torch.rand((B, 1, X, Y), generator=g)), ("smooth", smooth)):
                m = m.to(dev)
                for K in (1, 5, 10, 16):
                    for _ in range(5):
                        ops.nms_topk(m, K)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(200):
                        ops.nms_topk(m, K)
                    e1.record()
                    torch.cuda.synchronize()
                    res.append({"X": X, "Y": Y, "B": B, "map": kind, "K": K, "us": e0.elapsed_time(e1) * 1e3 / 200})
                    print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
