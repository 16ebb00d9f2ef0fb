#!/usr/bin/env python3
"""The PoseResNet-50 backbone's 1x1 convolutions as plain fp32 GEMMs through
torch.mm (hipBLASLt / rocBLAS on ROCm) -- a reference point for the fvp LDS-DMA
kernel's 1x1 layers (tools/backbone_layers.py): [pixels, Cin] x [Cin, Cout]
at 40 images, us per call and TF/s, TF32 off.

    python3 tools/gemm_probe.py
"""
import json


def main():
    import torch

    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda:0")
    shapes = [(40 * 128 * 240, 64, 256), (40 * 128 * 240, 256, 64), (40 * 128 * 240, 64, 64),
              (40 * 64 * 120, 128, 512), (40 * 64 * 120, 512, 128), (40 * 32 * 60, 256, 1024),
              (40 * 32 * 60, 1024, 256), (40 * 16 * 30, 512, 2048), (40 * 16 * 30, 2048, 512),
              (40 * 64 * 120, 256, 512), (40 * 32 * 60, 512, 1024)]
    for M, K, N in shapes:
        a = torch.randn((M, K), device=dev)
        b = torch.randn((K, N), device=dev)
        c = torch.empty((M, N), device=dev)
        for _ in range(3):
            torch.mm(a, b, out=c)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                torch.mm(a, b, out=c)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        us = sorted(ts)[1]
        print(json.dumps({"M": M, "K": K, "N": N, "us": round(us, 1), "tflops": round(2 * M * K * N / us / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
