#!/usr/bin/env python3
"""Per-layer time of the fvp P2PNet (JLN) or CenterNet (HDN), fp32 or bf16:
each ConvLayer call timed with HIP events (as tools/backbone_layers.py).

    python tools/cnn_layers.py [--net p2p|centernet] [--images 240] [--bf16]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--net", choices=["p2p", "centernet"], default="p2p")
    ap.add_argument("--images", type=int, default=240)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--algo", choices=["auto", "dma", "halo", "pertap"], default="auto",
                    help="fp32 kernel choice (algo of fvp.cnn.FvpCNN)")
    args = ap.parse_args()
    import torch

    import cnn_arch
    from fvp import cnn, synthetic

    dev = torch.device("cuda:0")
    J = 15
    if args.net == "p2p":
        m = cnn_arch.P2PNet(J, J).eval()
        hw = (64, 64)
    else:
        m = cnn_arch.CenterNet(J, 1).eval()
        hw = (80, 80)
    m.load_state_dict(synthetic.seeded_state_dict(m, 11))
    algo = {"auto": cnn.CONV_AUTO, "dma": cnn.CONV_DMA, "halo": cnn.CONV_HALO, "pertap": cnn.CONV_PER_TAP}[args.algo]
    f = cnn.FvpCNN(m.to(dev), torch.bfloat16 if args.bf16 else torch.float32, algo=algo)
    x = torch.rand((args.images, J) + hw, device=dev)
    run = (lambda: f(x)) if args.net == "p2p" else (lambda: f.from_xy(x))
    rec = []
    orig = cnn.ConvLayer.__call__

    def timed(self, a, relu, res_pre=None, res_post=None, out=None, pool=False):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        y = orig(self, a, relu, res_pre, res_post, out, pool)
        e1.record()
        rec.append((self, a.H, a.W, a.Cp, a.t.dtype, e0, e1, self.flops(a)))
        return y

    with torch.no_grad():
        run()
        torch.cuda.synchronize()
        cnn.ConvLayer.__call__ = timed
        try:
            run()
        finally:
            cnn.ConvLayer.__call__ = orig
        torch.cuda.synchronize()
    rows, tot = [], 0.0
    for (l, H, W, Cp, dt, e0, e1, fl) in rec:
        ms = e0.elapsed_time(e1)
        tot += ms
        rows.append({"k": f"{l.KH}x{l.KW}", "mode": l.mode, "in": [H, W, Cp], "in_dtype": str(dt).split(".")[-1],
                     "cout": l.Cout, "dma": any(v[1] for v in l._ws.values()), "ms": round(ms, 4),
                     "tflops": round(fl / 1e9 / ms, 1)})
    print(json.dumps({"net": args.net, "images": args.images, "dtype": "bf16" if args.bf16 else "fp32", "algo": args.algo,
                      "total_ms": round(tot, 3), "layers": rows}))


if __name__ == "__main__":
    main()
