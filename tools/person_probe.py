#!/usr/bin/env python3
"""Replay probe of the JLN person kernel (tools/person_probe.hip; VERDICT r3
item 5): bench_jln.py's C3 setup (32 frames x 10 proposals, channels-last
heatmaps read in place, the packed fine grid), each MODE timed with HIP events
(mean of --iters launches) next to the product's fvp_person_planes_cl; FULL
must equal the product's planes.  One JSON line per mode.

    python tools/person_probe.py [--frames 32] [--iters 20]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]
MODES = {"FULL": 0, "NOPLANES": 1, "NOTAPS": 2, "ALL_OOB": 3, "SETUP": 4, "NO_XZ_ATOMICS": 5, "NO_XY_ATOMICS": 6, "HALF_XZ_ATOMICS": 7, "XZ_STORES": 8}


def build():
    import torch

    src = os.path.join(REPO, "tools", "person_probe.hip")
    out = os.path.join(REPO, "tools", "bin", "libpprobe.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    csrc = os.path.join(REPO, "faster-voxelpose_amd", "csrc")
    deps = [src] + [os.path.join(csrc, f) for f in ("fvp_person.hip", "fvp_layout.h", "fvp_device.h")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        tl = os.path.join(os.path.dirname(torch.__file__), "lib")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-c", src, "-o", out + ".o"],
                       check=True)
        subprocess.run(["g++", "-shared", "-o", out, out + ".o", f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"],
                       check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--proposals", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    path = build()
    if args.build_only:
        return
    import numpy as np
    import torch

    from fvp import _lib, geometry, ops, synthetic
    from fvp.ops import _f3, _i3
    from fvp.project_individual import ProjectLayer
    from fvp.workloads import WORKLOADS

    lib = ctypes.CDLL(path)
    vp, i = ctypes.c_void_p, ctypes.c_int
    lib.person_probe.argtypes = [i, vp, i, vp, ctypes.POINTER(_lib.PersonSpec), vp, vp, i, i, i, i, i, vp, vp, vp]
    dev = torch.device("cuda:0")
    w = WORKLOADS["c3"]
    cams, seq = w.cameras()
    layer = ProjectLayer(w.cfg("cuda:0"))
    layer.verbose = False
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    F, P = args.frames, args.proposals
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, F)).to(dev)
    rng = np.random.default_rng(5)  # bench_jln.py's proposals
    props = []
    for f in range(F):
        pr = synthetic.proposals_for_frame(w, f, 4)
        extra = np.zeros((P - 4, 7), np.float32)
        extra[:, 0] = w.space_center[0] + rng.uniform(-3500, 3500, P - 4)
        extra[:, 1] = w.space_center[1] + rng.uniform(-3500, 3500, P - 4)
        extra[:, 2] = 900.0
        extra[:, 4] = 0.5
        extra[:, 5:7] = 0.5
        props.append(np.concatenate([pr, extra])[:P])
    pc = torch.from_numpy(np.concatenate(props)).to(dev).contiguous()
    frame_of = torch.arange(F, dtype=torch.int32, device=dev).repeat_interleave(P)
    B, V, J, H, W = hm.shape
    cl = torch.zeros((B, V, H, W, 16), device=dev)
    cl[..., :J] = hm.permute(0, 1, 3, 4, 2)
    meta = {"seq": [seq] * F}
    fg = layer._seq_grid(hm, 0, meta, cams, rt)
    args_ = layer._args()
    ref_planes = ops.person_planes_cl(cl, J, fg, pc, frame_of, *args_, False, True)[1]
    spec = _lib.PersonSpec(_i3(args_[0]), _f3(args_[1]), _f3(args_[2]), _f3(args_[3]), _f3(args_[4]),
                           _i3(args_[5]))
    S = args_[5]
    NP = pc.shape[0]
    planes = torch.empty((3 * NP, J, S[0], S[1]), device=dev)
    offset = torch.empty((NP, 3), device=dev)
    stream = torch.cuda.current_stream(dev)

    def probe(mode):
        rc = lib.person_probe(mode, cl.data_ptr(), 16, fg.data_ptr(), ctypes.byref(spec), pc.data_ptr(),
                              frame_of.data_ptr(), NP, V, J, H, W, planes.data_ptr(), offset.data_ptr(),
                              stream.cuda_stream)
        assert rc == 0, rc

    def product():
        ops.person_planes_cl(cl, J, fg, pc, frame_of, *args_, False, True)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.iters):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.iters

    print(json.dumps({"mode": "product fvp_person_planes_cl", "us": round(timed(product), 1), "proposals": NP,
                      "us_per_proposal": round(timed(product) / NP, 3)}), flush=True)
    probe(0)
    torch.cuda.synchronize()
    assert torch.equal(planes, ref_planes), "FULL differs from fvp_person_planes_cl"
    for name, m in MODES.items():
        us = timed(lambda: probe(m))
        print(json.dumps({"mode": name, "us": round(us, 1), "us_per_proposal": round(us / NP, 3)}), flush=True)


if __name__ == "__main__":
    main()
