#!/usr/bin/env python3
"""Per-layer time of the fvp PoseResNet-50 (fp32 or bf16) on B x V images of
960x512: each ConvLayer call timed with HIP events, reported with its geometry,
GFLOP and TF/s (which layers run below the engine's average).

    python tools/backbone_layers.py [--images 40] [--bf16]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=40)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--no-dma", action="store_true", help="fp32: keep AUTO off the LDS-DMA kernel")
    args = ap.parse_args()
    import torch

    import cnn_arch
    from fvp import cnn, synthetic
    from fvp.backbone import FvpPoseResNet

    dev = torch.device("cuda:0")
    m = cnn_arch.PoseResNet(50, 15).eval()
    m.load_state_dict(synthetic.seeded_state_dict(m, 21))
    bb = FvpPoseResNet(m.to(dev), torch.bfloat16 if args.bf16 else torch.float32,
                       algo=cnn.CONV_AUTO_NO_DMA if args.no_dma else cnn.CONV_AUTO)
    x = torch.randn((args.images, 3, 512, 960), device=dev)
    rec = []
    orig = cnn.ConvLayer.__call__

    def timed(self, a, relu, res_pre=None, res_post=None, out=None, pool=False):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        y = orig(self, a, relu, res_pre, res_post, out, pool)
        e1.record()
        rec.append((self, a.H, a.W, a.Cp, e0, e1, self.flops(a)))
        return y

    with torch.no_grad():
        bb.forward_nhwc(x)
        torch.cuda.synchronize()
        cnn.ConvLayer.__call__ = timed
        try:
            bb.forward_nhwc(x)
        finally:
            cnn.ConvLayer.__call__ = orig
        torch.cuda.synchronize()
    rows, tot_ms, tot_gf = [], 0.0, 0.0
    for (l, H, W, Cp, e0, e1, fl) in rec:
        ms = e0.elapsed_time(e1)
        tot_ms += ms
        tot_gf += fl / 1e9
        rows.append({"k": f"{l.KH}x{l.KW}", "mode": l.mode, "stride": l.stride[0], "in": [H, W, Cp], "cout": l.Cout,
                     "dma": any(v[1] for v in l._ws.values()),
                     "ms": round(ms, 3), "gflop": round(fl / 1e9, 1), "tflops": round(fl / 1e9 / ms, 1)})
    agg = {}
    for r in rows:
        key = f"{r['k']} mode{r['mode']} s{r['stride']}"
        a = agg.setdefault(key, [0.0, 0.0])
        a[0] += r["ms"]
        a[1] += r["gflop"]
    print(json.dumps({"images": args.images, "dtype": "bf16" if args.bf16 else "fp32", "f32_dma": not args.no_dma,
                      "total_ms": round(tot_ms, 2),
                      "total_tflops": round(tot_gf / tot_ms, 1),
                      "by_kind": {k: {"ms": round(v[0], 2), "tflops": round(v[1] / v[0], 1)} for k, v in agg.items()},
                      "layers": rows}))


if __name__ == "__main__":
    main()
