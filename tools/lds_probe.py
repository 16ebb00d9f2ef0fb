#!/usr/bin/env python3
"""Cycles per ds_read_b128 wave instruction by lane-address pattern (tools/lds_probe.hip).

Patterns (16-B slots of a 32 KB LDS image): linear (conflict-free), one
address (broadcast), uniform random, 2x2 tap quads (4 lanes = one bilinear
footprint at a 60-slot row pitch, 4 footprints per 16-lane group), and the
real top-left taps of C2 voxels (Shelf camera 0, 8x8-column tiles, relative
to the tile's footprint box, 64 consecutive voxels per instruction)."""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "faster-voxelpose_amd")]


def build():
    import torch

    src = os.path.join(REPO, "tools", "lds_probe.hip")
    out = os.path.join(REPO, "tools", "bin", "libldsprobe.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        tl = os.path.join(os.path.dirname(torch.__file__), "lib")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-c", src, "-o", out + ".o"],
                       check=True)
        subprocess.run(["g++", "-shared", "-o", out, out + ".o", f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"],
                       check=True)
    return out


def c2_taps(n_pat):
    import warnings

    warnings.filterwarnings("ignore")
    from fvp.geometry import camera_list, resize_transform
    from fvp.workloads import WORKLOADS
    from oracle import fvp_oracle as O

    w = WORKLOADS["c2"]
    cams, seq = w.cameras()
    X, Y, Z = w.voxels_per_axis
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    rt = resize_transform(w.ori_image_size, w.image_size).astype(np.float32)
    Wh, Hh = w.heatmap_size
    g = O.project_grid(grid, camera_list(cams, seq)[0], w.ori_image_size, w.image_size, w.heatmap_size, rt)
    g = g.reshape(X, Y, Z, 2)
    ix = np.floor((g[..., 0] + 1) * np.float32((Wh - 1) / 2)).astype(int)
    iy = np.floor((g[..., 1] + 1) * np.float32((Hh - 1) / 2)).astype(int)
    pats = []
    for a in range(0, X, 8):
        for b in range(0, Y, 8):
            xs, ys = ix[a:a + 8, b:b + 8].ravel(), iy[a:a + 8, b:b + 8].ravel()
            m = (xs >= 0) & (xs < Wh - 1) & (ys >= 0) & (ys < Hh - 1)
            if m.sum() < 64:
                continue
            xs, ys = xs[m], ys[m]
            bw = xs.max() - xs.min() + 2
            if bw * (ys.max() - ys.min() + 2) > 2048:
                continue
            off = (ys - ys.min()) * bw + (xs - xs.min())
            for k in range(0, len(off) - 63, 64):
                pats.append(off[k:k + 64])
            if len(pats) >= n_pat:
                return np.array(pats[:n_pat])
    return np.array(pats)


def main():
    path = build()
    import torch

    lib = ctypes.CDLL(path)
    lib.lds_probe_run.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_void_p]
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(0)
    npat = 64
    lane = np.arange(64)
    pats = {
        "linear": np.tile(lane, (npat, 1)),
        "broadcast": np.zeros((npat, 64), int),
        "random": rng.integers(0, 2048, (npat, 64)),
        "quad2x2_pitch60": np.stack([np.repeat(rng.integers(0, 1900, 16), 4) + np.tile([0, 1, 60, 61], 16)
                                     for _ in range(npat)]),
        "c2_taps_cam0": c2_taps(npat),
    }
    blocks, iters = ncu * 2, 2000
    out = torch.empty(blocks * 512, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for name, p in pats.items():
        t = torch.from_numpy(np.ascontiguousarray(p, np.int64) % 2048).to(torch.int32).to(dev)
        n = t.shape[0]
        lib.lds_probe_run(t.data_ptr(), n, 10, out.data_ptr(), blocks, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.lds_probe_run(t.data_ptr(), n, iters, out.data_ptr(), blocks, s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        instr_per_cu = 2 * 8 * iters * 8  # blocks/CU * waves * iters * reads
        cyc = ms * 1e-3 * 2.4e9 / instr_per_cu
        print(f"{name:18s} {cyc:6.2f} cycles per ds_read_b128 per CU (4 = conflict-free), "
              f"{1024 / cyc:6.1f} B/clk/CU", flush=True)


if __name__ == "__main__":
    main()
