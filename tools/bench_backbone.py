#!/usr/bin/env python3
"""Backbone line: the PoseResNet-50 heatmap backbone
(resnet.py:98-201, the default RESNET config, seeded weights) on the fvp MFMA
convolutions vs torch's own GPU forward (MIOpen) of the same eval module, on
B frames x V views of the Panoptic IMAGE_SIZE (960x512 -> 240x128 heatmaps);
then the views -> cube path at C2's voxel geometry:

  reference flow : per-view backbone + torch.stack (faster_voxelpose.py:73-75)
                   -> planar voxelize (layout pass + gather)
  fvp flow       : one backbone pass over all B*V views writing channels-last
                   heatmaps -> fvp_voxelize_cl (gather only, no layout pass)

    python tools/bench_backbone.py [--frames 8] [--views 5] [--iters 5] [--layers 50]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

MFMA_F32_PEAK_TF = 157.3
MFMA_BF16_PEAK_TF = 2500.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--views", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--layers", type=int, default=50)
    ap.add_argument("--torch", choices=["on", "off"], default="on")
    args = ap.parse_args()
    import numpy as np
    import torch

    import cnn_arch
    from fvp import geometry, synthetic
    from fvp.backbone import FvpPoseResNet
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    w = WORKLOADS["c2"]
    J = w.num_joints
    Wh, Hh = w.heatmap_size
    B, V = args.frames, args.views
    m = cnn_arch.PoseResNet(args.layers, J).eval()
    m.load_state_dict(synthetic.seeded_state_dict(m, 21))
    m = m.to(dev)
    views = torch.randn((B, V, 3, 4 * Hh, 4 * Wh), generator=torch.Generator().manual_seed(1)).to(dev)
    imgs = views.reshape(B * V, 3, 4 * Hh, 4 * Wh)
    f32, b16 = FvpPoseResNet(m), FvpPoseResNet(m, torch.bfloat16)
    gflop = f32.flops(B * V, 4 * Hh, 4 * Wh) / 1e9

    def timeit(fn, iters=args.iters):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(3):
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / iters)
        return float(np.median(ts))

    out = {"images": B * V, "image_hw": [4 * Hh, 4 * Wh], "heatmap_hw": [Hh, Wh], "gflop": round(gflop, 1)}
    with torch.no_grad():
        t_f = timeit(lambda: f32.forward_nhwc(imgs))
        t_b = timeit(lambda: b16.forward_nhwc(imgs))
        out.update(fvp_f32_ms=round(t_f, 3), fvp_f32_tflops=round(gflop / t_f, 1),
                   fvp_f32_frac_of_peak=round(gflop / t_f / MFMA_F32_PEAK_TF, 4),
                   fvp_bf16_ms=round(t_b, 3), fvp_bf16_tflops=round(gflop / t_b, 1),
                   fvp_bf16_frac_of_bf16_peak=round(gflop / t_b / MFMA_BF16_PEAK_TF, 4))
        if args.torch == "on":
            t_t = timeit(lambda: m(imgs))
            out.update(torch_f32_ms=round(t_t, 3), torch_f32_tflops=round(gflop / t_t, 1),
                       speedup_f32_vs_torch=round(t_t / t_f, 3))
            # torch's bf16 forward of the same module (MIOpen bf16 convolutions), NCHW and channels_last
            import copy
            mb = copy.deepcopy(m).to(torch.bfloat16)
            ib = imgs.to(torch.bfloat16)
            t_tb = timeit(lambda: mb(ib))
            mbc = copy.deepcopy(mb).to(memory_format=torch.channels_last)
            ibc = ib.contiguous(memory_format=torch.channels_last)
            t_tbc = timeit(lambda: mbc(ibc))
            out.update(torch_bf16_ms=round(t_tb, 3), torch_bf16_channels_last_ms=round(t_tbc, 3),
                       speedup_bf16_vs_torch_bf16=round(min(t_tb, t_tbc) / t_b, 3))
            del mb, mbc

        # views -> cube at C2's voxel geometry
        layer = ProjectLayer(w.cfg(str(dev)))
        layer.verbose = False
        cams, seq = w.cameras()
        rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float32,
                             device=dev)
        meta = {"seq": [seq] * B}
        cl = f32.heatmaps_cl(views)
        layer.prepare(cl, meta, cams, rt)
        planar = torch.stack([f32(views[:, c]) for c in range(V)], dim=1)

        def ref_flow():
            hm = torch.stack([f32(views[:, c]) for c in range(V)], dim=1)
            return layer.forward_fused(hm, meta, cams, rt)

        def fvp_flow():
            return layer.forward_fused(f32.heatmaps_cl(views), meta, cams, rt)

        def fvp_flow_bf16():  # bf16 backbone (opt-in precision), fp32 heatmaps and voxelize
            return layer.forward_fused(b16.heatmaps_cl(views), meta, cams, rt)

        t_vox_planar = timeit(lambda: layer.forward_fused(planar, meta, cams, rt), 20)
        t_vox_cl = timeit(lambda: layer.forward_fused(cl, meta, cams, rt), 20)
        t_ref, t_fvp, t_fvp_b = timeit(ref_flow), timeit(fvp_flow), timeit(fvp_flow_bf16)
        out["views_to_cube"] = {
            "frames": B, "geometry": "c2 (5 Shelf cams, 80x80x20, J=15)",
            "reference_flow_ms": round(t_ref, 3), "fvp_flow_ms": round(t_fvp, 3),
            "reference_flow_frames_per_s": round(B / t_ref * 1e3, 1), "fvp_flow_frames_per_s": round(B / t_fvp * 1e3, 1),
            "fvp_flow_bf16_backbone_ms": round(t_fvp_b, 3),
            "fvp_flow_bf16_backbone_frames_per_s": round(B / t_fvp_b * 1e3, 1),
            "voxelize_planar_ms": round(t_vox_planar, 4), "voxelize_channels_last_ms": round(t_vox_cl, 4),
            "layout_pass_removed_ms": round(t_vox_planar - t_vox_cl, 4)}
    print(json.dumps({"metric": f"PoseResNet-{args.layers} backbone on fp32 MFMA + views->cube",
                      "peak_tflops_f32": MFMA_F32_PEAK_TF, "weights": "seeded (synthetic.seeded_state_dict)",
                      **out}))


if __name__ == "__main__":
    main()
