#!/usr/bin/env python3
"""Winograd F(2x2, 3x3) (fvp_conv3x3_wino_nhwc) against the direct fp32 kernels
(AUTO without Winograd) on the 3x3 layer shapes of P2PNet (240 plane images of
64^2 -- C3 B=8, 10 proposals), CenterNet (8 frames of 80^2) and PoseResNet-50
(40 images), fused BN + ReLU (+ residual): kernel time by HIP events (mean of
--reps back-to-back calls, the median of 3 such batches), TF/s of the direct-conv FLOPs, and the max error of
each against torch's conv (fraction of the output scale).  One JSON line each.

    python3 tools/wino_probe.py [--reps 20]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]

SHAPES = [  # (name, N, Cin, Cout, H, W, residual)
    ("p2p 16->32 @64", 240, 16, 32, 64, 64, False), ("p2p 32->32 @64", 240, 32, 32, 64, 64, True),
    ("p2p 32->64 @32", 240, 32, 64, 32, 32, False), ("p2p 64->64 @32", 240, 64, 64, 32, 32, True),
    ("p2p 64->128 @16", 240, 64, 128, 16, 16, False), ("p2p 128->128 @16", 240, 128, 128, 16, 16, True),
    ("cn 32->32 @80", 8, 32, 32, 80, 80, True), ("cn 64->64 @40", 8, 64, 64, 40, 40, True),
    ("cn 128->128 @20", 8, 128, 128, 20, 20, True),
    ("r50 64->64 @128x240", 40, 64, 64, 128, 240, False), ("r50 128->128 @64x120", 40, 128, 128, 64, 120, False),
    ("r50 256->256 @32x60", 40, 256, 256, 32, 60, False), ("r50 512->512 @16x30", 40, 512, 512, 16, 30, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated name prefixes (p2p, cn, r50)")
    args = ap.parse_args()
    import torch
    import torch.nn as nn

    from fvp import cnn, synthetic

    dev = torch.device("cuda:0")
    for name, N, cin, cout, H, W, res in SHAPES:
        if args.only and not any(name.startswith(p) for p in args.only.split(",")):
            continue
        seq = nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout)).eval()
        seq.load_state_dict(synthetic.seeded_state_dict(seq, cin * 7 + cout))
        seq = seq.to(dev)
        g = torch.Generator().manual_seed(cin)
        x = (torch.rand((N, cin, H, W), generator=g) - 0.5).to(dev)
        r = torch.rand((N, cout, H, W), generator=g).to(dev) if res else None
        with torch.no_grad():
            ref = seq(x)
            ref = torch.relu(ref + r) if res else torch.relu(ref)
        xa = cnn.to_nhwc(x)
        ra = cnn.to_nhwc(r) if res else None
        line = {"layer": name, "N": N, "gflop": round(2 * N * H * W * cin * cout * 9 / 1e9, 2)}
        for tag, algo in (("direct", cnn.CONV_AUTO), ("wino", cnn.CONV_WINO)):
            wino_auto = cnn.WINO_AUTO
            cnn.WINO_AUTO = False  # the direct arm: AUTO's own choice among the direct kernels
            try:
                layer = cnn.ConvLayer(seq[0], seq[1], algo=algo)
                out = layer(xa, relu=True, res_pre=ra)
                torch.cuda.synchronize()
                times = []
                for _ in range(3):  # (the median of 3 batches: a host stall inside one batch idles the GPU)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        layer(xa, relu=True, res_pre=ra, out=out.t)
                    e1.record()
                    torch.cuda.synchronize()
                    times.append(e0.elapsed_time(e1) / args.reps)
            finally:
                cnn.WINO_AUTO = wino_auto
            ms = sorted(times)[1]
            got = cnn.to_nchw(out)
            err = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-6))
            line[tag] = {"us": round(ms * 1e3, 1), "tflops": round(line["gflop"] / ms, 1), "err": float(f"{err:.3g}"),
                         "kernel": [k for _, k in layer._ws.values()][0]}
        line["speedup"] = round(line["direct"]["us"] / line["wino"]["us"], 3)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
