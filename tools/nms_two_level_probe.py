#!/usr/bin/env python3
"""The two-level NMS (fvp_nms_topk_columns_ws: tiles of rows on many CUs, the
last tile block of a frame merges) against the one-block kernel
(fvp_nms_topk_columns: one 1024-thread block per frame), GPU time per launch
from a hipGraph of 50 back-to-back launches (HIP events, median of 3 replays),
at several batch sizes on C3-shaped maps (80 x 80, K = 10, J = 15, Z = 20):
smooth maps (the bench's xy planes) and plateaus of exact zeros (CenterNet's
masked output).  One JSON line per (B, map).

    python3 tools/nms_two_level_probe.py [--batches 1,8,16,32,64,128,256]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,16,32,64,128,256")
    a = ap.parse_args()
    import torch

    from fvp import ops
    from fvp.graphs import CapturedStep

    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    for B in [int(x) for x in a.batches.split(",")]:
        cube = torch.rand((B, 15, 80, 80, 20), generator=g).to(dev)
        smooth = torch.nn.functional.avg_pool2d(torch.rand((B, 1, 88, 88), generator=g), 9, 1).to(dev)
        plateau = torch.rand((B, 1, 80, 80), generator=g)
        plateau[plateau < 0.999] = 0.0
        plateau = plateau.to(dev)
        for mname, prob in (("smooth", smooth), ("plateau", plateau)):
            out = {"B": B, "map": mname}
            for tag, two in (("two_level", True), ("one_block", False)):
                def fn(two=two):
                    vals = torch.empty((B, 10), device=dev)
                    flat = torch.empty((B, 10), dtype=torch.int64, device=dev)
                    return ops._nms_topk_columns_into(prob, 10, cube, vals, flat, two_level=two)

                fn()  # the workspace is allocated outside the capture
                torch.cuda.synchronize()

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
                out[f"{tag}_us"] = round(sorted(ts)[1], 2)
                res = fn()
                torch.cuda.synchronize()
                out.setdefault("_res", []).append([r.cpu() for r in res])
            r2, r1 = out.pop("_res")
            out["identical"] = all(torch.equal(x, y) for x, y in zip(r2, r1))
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
