#!/usr/bin/env python3
"""fvp_weight_net (FvpWeightNet, the JLN's fused WeightNet) on 3P joint-feature
stacks of J x 64 x 64 (C3 B = 8, 10 proposals: 240 x 15 maps): us per call
(HIP events, median of 3 batches of 20) and a SHA-256 of the output, for the
library named by FVP_LIB (A/B builds).

    [FVP_LIB=ab_libs/<lib>.so] python3 tools/weightnet_probe.py
"""
import hashlib
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
    wn = cnn_arch.WeightNet(15).eval()
    wn.load_state_dict(synthetic.seeded_state_dict(wn, 15))
    f = cnn.FvpWeightNet(wn.to(dev))
    x = torch.randn((240, 15, 64, 64), generator=torch.Generator().manual_seed(1)).to(dev)
    y = f(x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f(x)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    print(json.dumps({"lib": os.environ.get("FVP_LIB", "libfvp.so"), "us": round(sorted(ts)[1], 1),
                      "out_sha256": hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()[:16]}))


if __name__ == "__main__":
    main()
