#!/usr/bin/env python3
"""Tile-shape sweep of fvp_conv2d_nhwc on the P2PNet layer shapes (tuning aid):
every tile id of fvp_conv_set_tile against the automatic choice (0)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def main():
    import numpy as np
    import torch
    import torch.nn as nn

    from fvp import _lib, cnn

    dev = torch.device("cuda:0")
    imgs = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    shapes = [("7x7 15->16 @64", 15, 16, 7, 64, False), ("3x3 32->32 @64", 32, 32, 3, 64, False),
              ("3x3 64->64 @32", 64, 64, 3, 32, False), ("3x3 128->128 @16", 128, 128, 3, 16, False),
              ("convT 128->64 @16", 128, 64, 2, 16, True), ("3x3 16->32 @64", 16, 32, 3, 64, False)]
    lib = _lib.load()
    for name, cin, cout, k, hw, up in shapes:
        conv = (nn.ConvTranspose2d(cin, cout, 2, stride=2) if up else nn.Conv2d(cin, cout, k, padding=k // 2)).to(dev)
        layer = cnn.ConvLayer(conv, None)
        x = cnn.to_nhwc(torch.rand((imgs, cin, hw, hw), device=dev))
        flops = layer.flops(x)
        res = []
        for tid in range(8):
            lib.fvp_conv_set_tile(tid)
            try:
                layer(x, relu=True)
                torch.cuda.synchronize()
            except _lib.FvpError:
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(3):
                e0.record()
                for _ in range(10):
                    layer(x, relu=True)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            t = float(np.median(ts))
            res.append((tid, t, flops / (t * 1e-3) / 1e12))
        lib.fvp_conv_set_tile(0)
        best = max(res[1:], key=lambda r: r[2])
        print(f"{name:20s} auto {res[0][2]:6.1f} TF  best tile {best[0]:2d} {best[2]:6.1f} TF  | " +
              " ".join(f"{tid}:{tf:.0f}" for tid, _, tf in res), flush=True)


if __name__ == "__main__":
    main()
