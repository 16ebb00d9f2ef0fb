#!/usr/bin/env python3
"""End-to-end HDN + JLN inference after the backbone, on fvp:
heatmaps -> voxel cube + xy plane -> CenterNet -> NMS top-K -> bbox / z-column
gathers -> C2CNet -> proposals -> per-person planes -> P2PNet -> soft-argmax +
offsets -> WeightNet -> fusion, for B frames at C3 geometry.

CenterNet / C2CNet / P2PNet run on the fvp MFMA convolutions and WeightNet on
its fused kernel (install(cnn=True)), all with the reference architectures
(tests/cnn_arch.py) and seeded weights; --torch-cnn runs the same modules on
torch.  Reports frames/s and a per-stage breakdown (HIP events).

    python tools/bench_pipeline.py [--frames 8] [--steps 10] [--views]

--views starts from the camera images instead: the PoseResNet-50 backbone
(seeded weights) on B x V images of the IMAGE_SIZE (fvp.backbone: all views
in one pass, heatmaps written channels-last and read in place by the HDN / JLN;
with --torch-cnn the reference flow: per-view torch backbone + torch.stack).
"""
import argparse
import json
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--torch-cnn", action="store_true", help="CNNs on torch's convolution instead of fvp")
    ap.add_argument("--bf16", action="store_true", help="fvp CNNs with bf16 operands (opt-in precision)")
    ap.add_argument("--views", action="store_true", help="start from the images: PoseResNet-50 backbone first")
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.nn as nn

    import cnn_arch
    from fvp import geometry, integration, jln, synthetic
    from fvp.config import AttrDict
    from fvp.project_individual import ProjectLayer as PI
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    w = WORKLOADS[args.workload]
    J, B, K = w.num_joints, args.frames, w.max_people
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, B)).to(dev)
    meta = {"seq": [seq] * B}

    class Proposal(nn.Module):  # test-mode ProposalLayer (human_detection_net.py:99-124)
        # the constants the fused HDN's proposal_centers kernel reads; min_score -1:
        # every proposal valid, so the JLN runs at full K (stand-in confidences)
        scale = [float(s) / (float(n) - 1) for s, n in zip(w.space_size, w.voxels_per_axis)]
        bias = [float(c) - float(s) / 2.0 for c, s in zip(w.space_center, w.space_size)]
        min_score = -1.0

        def forward(self, topk_index, topk_confs, match_bbox, meta):
            scale = torch.tensor(w.space_size, device=dev) / (torch.tensor(w.voxels_per_axis, device=dev) - 1)
            bias = torch.tensor(w.space_center, device=dev) - torch.tensor(w.space_size, device=dev) / 2.0
            out = torch.zeros(topk_confs.shape + (7,), device=dev)
            out[:, :, 0:3] = topk_index.float() * scale + bias
            out[:, :, 4] = topk_confs
            out[:, :, 3] = 0.0  # every proposal valid: the JLN runs at full K (stand-in confidences)
            out[:, :, 5:7] = match_bbox.clamp(0.3, 0.8)
            return out

    hdn = types.SimpleNamespace(max_people=K)
    hdn.project_layer = ProjectLayer(w.cfg(str(dev)))
    hdn.project_layer.verbose = False
    hdn.center_net = cnn_arch.CenterNet(J, 1).eval()
    hdn.center_net.load_state_dict(synthetic.seeded_state_dict(hdn.center_net, 12))
    hdn.center_net = hdn.center_net.to(dev)
    hdn.c2c_net = cnn_arch.C2CNet(J, 1).eval()
    hdn.c2c_net.load_state_dict(synthetic.seeded_state_dict(hdn.c2c_net, 14))
    hdn.c2c_net = hdn.c2c_net.to(dev)
    hdn.proposal_layer = Proposal()
    jl = types.SimpleNamespace(training=False)
    jl.project_layer = PI(w.cfg(str(dev)))
    jl.project_layer.verbose = False
    jl.conv_net = cnn_arch.P2PNet(J, J).eval()
    jl.conv_net.load_state_dict(synthetic.seeded_state_dict(jl.conv_net, 11))
    jl.conv_net = jl.conv_net.to(dev)
    jl.weight_net = cnn_arch.WeightNet(J).eval()
    jl.weight_net.load_state_dict(synthetic.seeded_state_dict(jl.weight_net, 15))
    jl.weight_net = jl.weight_net.to(dev)
    jl.soft_argmax_layer = jln.SoftArgmaxLayer(AttrDict.wrap({"NETWORK": {"BETA": 100}}))
    for net in (hdn, jl):
        integration.set_options(net, cnn=not args.torch_cnn,
                                cnn_dtype=torch.bfloat16 if args.bf16 else torch.float32)
    backbone = None
    if args.views:
        from fvp.backbone import FvpPoseResNet

        rn = cnn_arch.PoseResNet(50, J).eval()
        rn.load_state_dict(synthetic.seeded_state_dict(rn, 21))
        rn = rn.to(dev)
        Wi, Hi = w.image_size
        views = torch.randn((B, len(cams[seq]), 3, Hi, Wi), generator=torch.Generator().manual_seed(2)).to(dev)
        if args.torch_cnn:  # the reference flow (faster_voxelpose.py:75)
            backbone = lambda: torch.stack([rn(views[:, c]) for c in range(views.shape[1])], dim=1)  # noqa: E731
        else:
            fb = FvpPoseResNet(rn, torch.bfloat16 if args.bf16 else torch.float32)
            backbone = lambda: fb.heatmaps_cl(views).planar()  # noqa: E731  (channels-last copy attached)

    def step(record=None):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if record is not None else None
        if ev:
            ev[3].record()
        heat = backbone() if backbone is not None else hm
        if ev:
            ev[0].record()
        _, _, centers, _ = integration.fused_hdn_forward(hdn, heat, meta, cams, rt)
        centers[:, :, 5:7].clamp_(0.3, 0.8)  # seeded bbox head: keep every person window non-empty
        if ev:
            ev[1].record()
        mask = centers[:, :, 3] >= 0
        fused, _ = jln.fused_jln_forward(jl, meta, heat, centers, mask, cams, rt)
        if ev:
            ev[2].record()
            record.append(ev)
        return fused

    reps = []  # three timed repeats, the median reported (one-off box hiccups seen at ~2x)
    with torch.no_grad():
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        for _ in range(3):
            evs = []
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                step(evs)
            e1.record()
            torch.cuda.synchronize()
            reps.append((e0.elapsed_time(e1) / args.steps, evs))
    reps.sort(key=lambda r: r[0])
    ms, evs = reps[1]
    hdn_ms = float(np.mean([a.elapsed_time(b) for a, b, _, _ in evs]))
    jln_ms = float(np.mean([b.elapsed_time(c) for _, b, c, _ in evs]))
    bb_ms = float(np.mean([d.elapsed_time(a) for a, _, _, d in evs]))
    print(json.dumps({
        "metric": ("views -> backbone -> HDN+JLN (images -> fused 3-D poses)" if args.views else
                   "HDN+JLN inference after the backbone (heatmaps -> fused 3-D poses)"), "unit": "frames/s",
        "backbone_ms": round(bb_ms, 3) if args.views else None,
        "value": round(B / (ms * 1e-3), 1), "ms_per_batch": round(ms, 3),
        "ms_per_batch_repeats": [round(r[0], 3) for r in reps], "frames": B, "proposals_per_frame": K,
        "hdn_ms": round(hdn_ms, 3), "jln_ms": round(jln_ms, 3),
        "cnn": "torch (MIOpen)" if args.torch_cnn else ("fvp bf16 MFMA" if args.bf16 else "fvp fp32 MFMA"),
        "config": f"{w.name}: {len(cams[seq])} cams, J={J}, {w.voxels_per_axis} whole grid, 64^3 per person; "
                  "CenterNet/C2CNet/P2PNet/WeightNet reference architectures with seeded weights"}))


if __name__ == "__main__":
    main()
