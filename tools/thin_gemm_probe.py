#!/usr/bin/env python3
"""The PoseResNet-50 head's final 1x1 conv (256 -> 15 joints, padded to 16, at 40 x
128 x 240) and the stage-1 downsample (64 -> 256, no residual) on the fvp kernels
vs one hipBLASLt GEMM with the bias in its epilogue (torch.addmm): us per call.

    python3 tools/thin_gemm_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def main():
    import torch
    import torch.nn as nn

    from fvp import cnn

    dev = torch.device("cuda:0")

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        return sorted(ts)[2]

    for cin, cout, bn in ((256, 15, False), (64, 256, True), (256, 64, True), (512, 128, True)):
        torch.manual_seed(cin)
        conv = nn.Conv2d(cin, cout, 1, bias=not bn).to(dev).eval()
        b = nn.BatchNorm2d(cout).to(dev).eval() if bn else None
        layer = cnn.ConvLayer(conv, b, algo=cnn.CONV_AUTO)
        x = cnn.Act(torch.randn((40, 128, 240, layer.Cpi), device=dev), cin)
        out = torch.empty((40, 128, 240, layer.Cpo), device=dev)
        saved, cnn.BLAS_1X1 = cnn.BLAS_1X1, False
        t_fvp = timeit(lambda: layer(x, relu=bn, out=out))
        cnn.BLAS_1X1 = saved
        w = torch.zeros((layer.Cpo, layer.Cpi), device=dev)
        w[:cout, :cin] = conv.weight.detach()[:, :, 0, 0] * layer.scale[:cout, None]
        a, o = x.t.view(-1, layer.Cpi), out.view(-1, layer.Cpo)
        t_blas = timeit(lambda: torch.addmm(layer.shift, a, w.t(), out=o))
        t_blas_relu = timeit(lambda: torch._addmm_activation(layer.shift, a, w.t(), out=o))
        print(json.dumps({"cin": cin, "cout": cout, "fvp_us": round(t_fvp, 1), "addmm_us": round(t_blas, 1),
                          "addmm_relu_us": round(t_blas_relu, 1)}), flush=True)


if __name__ == "__main__":
    main()
