#!/usr/bin/env python3
"""JLN per-person line (SURVEY.md §8(d) "JLN, per proposal (separate line)"):
project_individual.ProjectLayer.forward (64^3 cubes) + xy/xz/yz max planes for
K proposals per frame, Panoptic demo geometry (configs/panoptic/jln64.yaml).

    python tools/bench_jln.py [--frames 16] [--proposals 10] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--proposals", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--on-the-fly", action="store_true",
                    help="project the fine grid in the kernel (fvp_person_planes_cams) instead of the packed grid")
    args = ap.parse_args()

    import numpy as np
    import torch

    from fvp import geometry, synthetic
    from fvp.project_individual import ProjectLayer
    from fvp.workloads import WORKLOADS

    dev = torch.device("cuda:0")
    w = WORKLOADS[args.workload]
    cams, seq = w.cameras()
    layer = ProjectLayer(w.cfg("cuda:0"))
    layer.verbose = False
    if args.on_the_fly:
        layer.on_the_fly = True
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    F, P = args.frames, args.proposals
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, F)).to(dev)
    rng = np.random.default_rng(5)
    props = []
    for f in range(F):
        pr = synthetic.proposals_for_frame(w, f, 4)
        extra = np.zeros((P - 4, 7), np.float32)
        extra[:, 0] = w.space_center[0] + rng.uniform(-3500, 3500, P - 4)
        extra[:, 1] = w.space_center[1] + rng.uniform(-3500, 3500, P - 4)
        extra[:, 2] = 900.0
        extra[:, 4] = 0.5
        extra[:, 5:7] = 0.5
        props.append(torch.from_numpy(np.concatenate([pr, extra])[:P]).to(dev))
    meta = {"seq": [seq] * F}
    # the first call per sequence: library / code-object load + the fine sample
    # grid build (project_individual.py:192-220, 4.1 M points x V cameras) + one
    # planes launch; then a second sequence key on the same cameras times the
    # grid build alone (project_grid + pack, wall and HIP events)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    layer.forward_planes(hm, 0, meta, props[0], cams, rt)
    torch.cuda.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    seq_b = seq + "#second"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    layer.build_sample_grid({seq_b: cams[seq]}, seq_b, rt, dev)
    e1.record()
    torch.cuda.synchronize()
    cache = {"first_call_ms": round(first_ms, 2), "sequence_build_ms": round((time.perf_counter() - t0) * 1e3, 3),
             "sequence_build_gpu_ms": round(e0.elapsed_time(e1), 3),
             "what": "fine sample grid [V,253,253,64,2] (fvp_project_grid) + its voxel-major pack (fvp_pack_grid)"}

    allp = torch.stack(props)
    mask = torch.ones((F, P), dtype=torch.bool, device=dev)

    def per_frame():
        for f in range(F):
            layer.forward_planes(hm, f, meta, props[f], cams, rt)

    def batched():
        layer.forward_batch(hm, meta, allp, mask, cams, rt)

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.steps

    ms_frame = timeit(per_frame)
    ms = timeit(batched)

    # the same batched op on heatmaps held channels-last, as the fvp backbone writes
    # them ([B,V,H,W,16]: no layout pass; the bench's other lines take planar input)
    from fvp.heatmaps import ChannelsLastHeatmaps
    cp = 16 * ((w.num_joints + 15) // 16)
    hm_cl = torch.zeros(hm.shape[0], hm.shape[1], hm.shape[3], hm.shape[4], cp, device=dev)
    hm_cl[..., : w.num_joints] = hm.permute(0, 1, 3, 4, 2)
    hcl = ChannelsLastHeatmaps(hm_cl.contiguous(), w.num_joints)

    def batched_cl():
        layer.forward_batch(hcl, meta, allp, mask, cams, rt)

    ms_cl = timeit(batched_cl)

    # the drop-in flow on planar input: the fused HDN forward lays the batch out
    # channels-last once and attaches the copy to the heatmaps tensor
    # (fvp.heatmaps.share_channels_last, integration.FvpOptions.share_layout),
    # and the JLN, handed the same tensor, reads it in place
    from fvp.heatmaps import share_channels_last
    hm_shared = hm.clone()
    share_channels_last(hm_shared)

    def batched_shared():
        layer.forward_batch(hm_shared, meta, allp, mask, cams, rt)

    ms_shared = timeit(batched_shared)

    # JLN post-processing on device (soft-argmax + offsets + fusion) on stand-in
    # CNN outputs of the same shape: reads 3*J*S*S*4 B of joint maps per proposal
    from fvp import ops
    n_prop0 = F * P
    feats = torch.from_numpy(synthetic.joint_features(n_prop0, w.num_joints, 64, 3)).to(dev)
    wts = torch.from_numpy(synthetic.jln_weights(n_prop0, w.num_joints, 3)).to(dev)
    offs = torch.from_numpy(synthetic.jln_offsets(n_prop0, 3)).to(dev)

    def post():
        pose, mp = ops.soft_argmax(feats, layer.center_grid, offs, 100.0)
        ops.fuse_poses(pose, wts, mp)

    ms_post = timeit(post)

    # tap stream of the person kernel (project_individual.py:255-269 windows):
    # in-window voxels x cameras x 4 bilinear taps x one 64-B channels-last pixel
    c = layer._const
    pc = allp.reshape(-1, 7).cpu().numpy().astype(np.float32)
    fine = c["fine"].astype(np.int64)
    ctl = np.rint(pc[:, 0:3] * c["scale"] + c["bias"]).astype(np.int64)
    m = np.zeros((pc.shape[0], 3), np.int64)
    m[:, 0:2] = np.maximum(((1.0 - pc[:, 5:7]) / 2.0 * (64 - 1)).astype(np.int64), 0)
    start = np.where(ctl + m >= 0, ctl + m, 0)
    end = np.where(ctl + 64 - m <= fine, ctl + 64 - m, fine)
    win = np.where((end > start).all(axis=1), np.prod(np.clip(end - start, 0, None), axis=1), 0)
    V = len(cams[seq])
    tap_bytes = float(win.sum()) * V * 4 * 64
    tap_tbs = tap_bytes / (ms * 1e-3) / 1e12
    post_bytes = 3 * w.num_joints * 64 * 64 * 4 * n_prop0
    J = w.num_joints
    n_prop = F * P
    print(json.dumps({
        "metric": "JLN per-person voxelize + xy/xz/yz max planes", "unit": "proposals/s",
        "value": round(n_prop / (ms * 1e-3), 1), "us_per_proposal": round(ms * 1e3 / n_prop, 2),
        "frames_per_s_at_K": round(F / (ms * 1e-3), 1), "K": P, "frames": F,
        "config": f"{w.name}: {len(cams[seq])} cams, J={J}, 64^3 person cubes from a 253x253x64 fine grid",
        "cube_bytes_per_proposal": J * 64 ** 3 * 4, "plane_bytes_per_proposal": 3 * J * 64 * 64 * 4,
        "per_frame_calls_us_per_proposal": round(ms_frame * 1e3 / n_prop, 2),
        "channels_last_input_us_per_proposal": round(ms_cl * 1e3 / n_prop, 2),
        "planar_drop_in_us_per_proposal": round(ms_shared * 1e3 / n_prop, 2),
        "path": "forward_batch: one fvp_person_planes launch for all frames' proposals (fused planes, no cubes)",
        "cache_build": cache,
        "tap_stream": {"window_voxels_per_proposal": round(float(win.mean()), 1),
                       "bytes_per_proposal": round(tap_bytes / n_prop), "achieved_tb_s": round(tap_tbs, 2),
                       "l2_gather_ceiling_tb_s": "16.8-18.8 (MI355X_MICROARCH.md, random 16-B row gathers from L2)"},
        "post": {"op": "fvp_soft_argmax + fvp_fuse_poses (SoftArgmaxLayer, offsets, fuse_pose_preds)",
                 "us_per_proposal": round(ms_post * 1e3 / n_prop0, 3),
                 "hbm_gbs": round(post_bytes / (ms_post * 1e-3) / 1e9, 1),
                 "hbm_frac": round(post_bytes / (ms_post * 1e-3) / 8e12, 4)}}))


if __name__ == "__main__":
    main()
