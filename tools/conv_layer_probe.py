#!/usr/bin/env python3
"""One backbone-shaped convolution, repeated: the unit for rocprofv3 kernel
stats and PMC passes on the conv kernels (bf16 operands and activations by
default).

    python tools/conv_layer_probe.py [--k 3] [--cin 64] [--cout 64] [--hw 128 240]
                                     [--images 40] [--iters 20] [--fp32]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--cout", type=int, default=64)
    ap.add_argument("--hw", type=int, nargs=2, default=[128, 240])
    ap.add_argument("--images", type=int, default=40)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--fp32", action="store_true")
    args = ap.parse_args()
    import torch
    import torch.nn as nn

    from fvp import cnn, synthetic

    dev = torch.device("cuda:0")
    seq = nn.Sequential(nn.Conv2d(args.cin, args.cout, args.k, stride=args.stride, padding=args.k // 2, bias=False),
                        nn.BatchNorm2d(args.cout)).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, 5))
    seq = seq.to(dev)
    bf16 = not args.fp32
    layer = cnn.ConvLayer(seq[0], seq[1], torch.bfloat16 if bf16 else torch.float32)
    layer.act_bf16 = bf16
    H, W = args.hw
    x = torch.rand((args.images, args.cin, H, W), device=dev)
    a = cnn.to_nhwc(x)
    if bf16:
        a = cnn.Act(a.t.to(torch.bfloat16), a.C)
    with torch.no_grad():
        layer(a, relu=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            y = layer(a, relu=True)
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    fl = layer.flops(a)
    print(json.dumps({"k": args.k, "stride": args.stride, "cin": args.cin, "cout": args.cout, "hw": [H, W],
                      "images": args.images, "dtype": "bf16" if bf16 else "fp32", "ms": round(ms, 4),
                      "tflops": round(fl / ms / 1e9, 1), "out": list(y.t.shape)}))


if __name__ == "__main__":
    main()
