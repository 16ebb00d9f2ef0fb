#!/usr/bin/env python3
"""The PoseResNet-50 1x1 / stride-2 downsample layers (40 images) on the fvp kernel vs a
batched library GEMM over the row-strided NHWC view (no gather copy): torch.bmm and
torch.baddbmm with the BN shift as the C matrix, us per call.

    python3 tools/strided_gemm_probe.py
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

    for cin, cout, h, w in ((256, 512, 128, 240), (512, 1024, 64, 120), (1024, 2048, 32, 60)):
        torch.manual_seed(cin)
        conv = nn.Conv2d(cin, cout, 1, stride=2, bias=False).to(dev).eval()
        bn = nn.BatchNorm2d(cout).to(dev).eval()
        layer = cnn.ConvLayer(conv, bn, algo=cnn.CONV_AUTO)
        N = 40
        x = cnn.Act(torch.randn((N, h, w, cin), device=dev), cin)
        out = torch.empty((N, h // 2, w // 2, cout), device=dev)
        t_fvp = timeit(lambda: layer(x, relu=False, out=out))
        ref = layer(x, relu=False).t
        wf = (conv.weight.detach()[:, :, 0, 0] * layer.scale[:cout, None]).t().contiguous()  # [cin, cout]
        a = x.t[:, ::2, ::2, :].reshape(N * (h // 2), w // 2, cin) if False else \
            x.t.as_strided((N * (h // 2), w // 2, cin), (2 * w * cin, 2 * cin, 1))
        o = out.view(N * (h // 2), w // 2, cout)
        wb = wf.expand(N * (h // 2), cin, cout)
        t_bmm = timeit(lambda: torch.bmm(a, wb, out=o))
        sh = layer.shift[:cout].expand(N * (h // 2), w // 2, cout)
        t_baddbmm = timeit(lambda: torch.baddbmm(sh, a, wb, out=o))
        torch.baddbmm(sh, a, wb, out=o)
        err = float((o.view_as(ref) - ref).abs().max() / ref.abs().max())
        print(json.dumps({"cin": cin, "cout": cout, "in_hw": [h, w], "fvp_us": round(t_fvp, 1),
                          "bmm_us": round(t_bmm, 1), "baddbmm_us": round(t_baddbmm, 1), "rel_err": err}),
              flush=True)


if __name__ == "__main__":
    main()
