#!/usr/bin/env python3
"""fvp_conv1d_net (one-launch C2CNet) at C3 B = 8 (80 columns of 15 x 20): kernel
time per positions-per-item choice (lg 4 / 8) against the per-layer kernels.

    python3 tools/c2c_probe.py [--cols 80] [--L 20]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd"), os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cols", type=int, default=80)
    ap.add_argument("--L", type=int, default=20)
    args = ap.parse_args()
    import torch

    import cnn_arch
    from fvp import cnn, synthetic
    from fvp.graphs import CapturedStep

    dev = torch.device("cuda:0")
    m = cnn_arch.C2CNet(15, 1).eval()
    m.load_state_dict(synthetic.seeded_state_dict(m, 14))
    m = m.to(dev)
    x = torch.rand((args.cols, 15, args.L), generator=torch.Generator().manual_seed(1)).to(dev)
    with torch.no_grad():
        ref = m(x)

    def timeit(fn, reps=50):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / reps * 1e3)
        return sorted(ts)[1]

    out = {"cols": args.cols, "L": args.L}
    n0 = cnn.Net1D.build(m, 15, args.L)
    out["wchunk"] = None if n0 is None else n0.wchunk
    for lg in (4, 8):
        n = cnn.Net1D.build(m, 15, args.L)
        if n is None:
            continue
        n.lg = lg
        try:
            y = n(x)
        except Exception as e:  # lg 8's partial sums may not fit next to this length's buffers
            out[f"one_launch_lg{lg}"] = f"not run: {e}"
            continue
        err = float((y - ref).abs().max() / ref.abs().max())
        out[f"one_launch_lg{lg}_us"] = round(timeit(lambda: n(x)), 1)
        out[f"one_launch_lg{lg}_err"] = err
    per_layer = cnn.FvpCNN(m, algo=cnn.CONV_PER_TAP)
    out["per_layer_us"] = round(timeit(lambda: per_layer(x)), 1)
    cap = CapturedStep(lambda: per_layer(x))
    out["per_layer_graph_us"] = round(timeit(cap.replay), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
