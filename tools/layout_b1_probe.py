#!/usr/bin/env python3
"""B=1 kernel durations under rocprofv3 --kernel-trace: the one-frame voxelize
step (layout pass + gather) next to a float4 copy of the same 9.2 MB, each
launched in isolation (synchronised), to see how far the one-frame layout pass
is from a plain copy.

    rocprofv3 --kernel-trace --stats -d DIR -- python3 tools/layout_b1_probe.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def main():
    import torch
    from fvp import _lib, geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    w = WORKLOADS["c2"]
    layer = ProjectLayer(w.cfg(str(dev)))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float32, device=dev)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 1)).to(dev)
    meta = {"seq": [seq]}
    dst = torch.empty_like(hm)
    for _ in range(30):
        layer.forward_fused(hm, meta, cams, rt, want_cube=True, want_xy=True)
        torch.cuda.synchronize()
        _lib.call("fvp_copy_f4", hm.data_ptr(), dst.data_ptr(), hm.numel() * 4, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
