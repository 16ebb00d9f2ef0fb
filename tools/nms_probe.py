#!/usr/bin/env python3
"""NMS top-K + column gather (fvp_nms_topk_columns) at C3 B = 8 shapes: GPU time per
launch from a hipGraph of 50 back-to-back launches (HIP events, median of 3
replays; no host time), for the library named by FVP_LIB (probe builds of
fvp_proposal.hip).

    [FVP_LIB=ab_libs/<lib>.so] python3 tools/nms_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    import torch

    from fvp import ops

    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    out = {"lib": os.environ.get("FVP_LIB", "libfvp.so")}
    for B, mname in ((1, ""), (8, ""), (8, "plateau_")):
        prob = torch.nn.functional.avg_pool2d(torch.rand((B, 1, 88, 88), generator=g), 9, 1).to(dev)
        if mname:  # a few peaks on exact zeros: hundreds of tied candidates
            prob = torch.rand((B, 1, 80, 80), generator=g)
            prob[prob < 0.999] = 0.0
            prob = prob.to(dev)
        cube = torch.rand((B, 15, 80, 80, 20), generator=g).to(dev)
        for tag, fn in ((f"{mname}topk", lambda: ops.nms_topk(prob, 10)),
                        (f"{mname}topk_columns", lambda: ops.nms_topk_columns(prob, 10, cube))):
            from fvp.graphs import CapturedStep

            def many(fn=fn):
                for _ in range(50):
                    r = fn()
                return r
            cap = CapturedStep(many)
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                cap.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 50 * 1e3)
            out[f"B{B}_{tag}_us"] = round(sorted(ts)[1], 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
