#!/usr/bin/env python3
"""Time fvp_up2_head_nchw (P2PNet's fused tail) at the pipeline's shape: 240
planes, x [240][32][32][64] -> NCHW [240][15][64][64], HIP events, mean of 20
calls (the median of 3 batches); the algorithmic bytes and GB/s with it.

    [FVP_LIB=ab_libs/<lib>.so] python3 tools/up2_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd"), os.path.join(REPO, "tests")]


def main():
    import torch

    import cnn_arch
    from fvp import cnn, synthetic

    dev = torch.device("cuda:0")
    p2p = cnn_arch.P2PNet(15, 15).eval()
    p2p.load_state_dict(synthetic.seeded_state_dict(p2p, 11))
    f = cnn.FvpCNN(p2p.to(dev))
    n = 240
    g = torch.Generator().manual_seed(3)
    x = cnn.to_nhwc(torch.rand((n, 64, 32, 32), generator=g).to(dev), 64)
    skip = cnn.to_nhwc(torch.rand((n, 32, 64, 64), generator=g).to(dev), 32)
    for _ in range(3):
        f._tail_nchw(x, skip)
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f._tail_nchw(x, skip)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    us = sorted(ts)[1]
    nbytes = x.t.numel() * 4 + skip.t.numel() * 4 + n * 15 * 64 * 64 * 4
    print(json.dumps({"kernel": "fvp_up2_head_nchw", "planes": n, "us": round(us, 2), "mb": round(nbytes / 1e6, 1),
                      "gbs": round(nbytes / us / 1e3, 1), "lib": os.environ.get("FVP_LIB", "libfvp.so")}))


if __name__ == "__main__":
    main()
