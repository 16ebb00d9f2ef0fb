#!/usr/bin/env python3
"""A/B of the next-generation gather variants (tools/vox_next.hip) against the
product fvp_voxelize op, interleaved in one process, exactness checked.

    python tools/microbench2.py [--workload c2] [--batch 256] [--rounds 5]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def build():
    src = os.path.join(REPO, "tools", "vox_next.hip")
    out = os.path.join(REPO, "tools", "libvoxnext.so")
    deps = [src, os.path.join(REPO, "faster-voxelpose_amd", "csrc", "fvp_layout.h"),
            os.path.join(REPO, "faster-voxelpose_amd", "csrc", "fvp_device.h")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        import torch

        tl = os.path.join(os.path.dirname(torch.__file__), "lib")
        obj = out + ".o"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-c", src, "-o", obj],
                       check=True)
        subprocess.run(["g++", "-shared", "-o", out, obj, f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"],
                       check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--uniform", action="store_true", help="uniform-random heatmaps instead of Gaussian blobs")
    args = ap.parse_args()
    path = build()

    import numpy as np
    import torch

    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    lib = ctypes.CDLL(path)
    vp, i_ = ctypes.c_void_p, ctypes.c_int
    lib.voxnext_regrid.argtypes = [vp, vp, i_, i_, ctypes.c_longlong, vp]
    lib.voxnext_qg.argtypes = [vp, i_] + [i_] * 5 + [vp, i_] + [i_] * 3 + [vp, vp, vp, i_, i_, i_, i_, vp]

    dev = torch.device("cuda:0")
    w = WORKLOADS[args.workload]
    B = args.batch
    layer = ProjectLayer(w.cfg("cuda:0"))
    layer.verbose = False
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    if args.uniform:
        hm = torch.from_numpy(synthetic.uniform_heatmaps(w, B)).to(dev)
    else:
        hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, B)).to(dev)
    if w.dtype == "float16":
        hm = hm.half()
    meta = {"seq": [seq] * B}
    ref_cube, ref_xy = layer.forward_fused(hm, meta, cams, rt)
    torch.cuda.synchronize()
    grids = layer.build_sample_grid(cams, seq, rt, dev).contiguous()  # [V,1,N,2]
    _, V, J, H, W = hm.shape
    X, Y, Z = w.voxels_per_axis
    N = X * Y * Z
    stream = torch.cuda.current_stream().cuda_stream
    lpv = 4
    GV = 2 * lpv * ((V + 2 * lpv - 1) // (2 * lpv))
    gq = torch.empty((N, GV, 2), device=dev)
    assert lib.voxnext_regrid(grids.data_ptr(), gq.data_ptr(), V, GV, N, stream) == 0
    GV2 = 2 * ((V + 1) // 2)
    gq2 = torch.empty((N, GV2, 2), device=dev)
    assert lib.voxnext_regrid(grids.data_ptr(), gq2.data_ptr(), V, GV2, N, stream) == 0
    lib.voxnext_mf.argtypes = [vp, i_] + [i_] * 5 + [vp, i_] + [i_] * 3 + [vp, vp, vp, i_, i_, i_, i_, vp]

    def mf(chunk, cols, F, pf):
        def f():
            rc = lib.voxnext_mf(hm.data_ptr(), int(hm.dtype == torch.float16), B, V, J, H, W, gq2.data_ptr(), GV2,
                                X, Y, Z, cube.data_ptr(), xy.data_ptr(), ws.data_ptr(), chunk, cols, F, pf, stream)
            assert rc == 0, rc
        return f
    lib.voxnext_h.argtypes = [vp] + [i_] * 5 + [vp] + [i_] * 3 + [vp, vp, vp, i_, i_, vp, i_, vp]
    hper = V * H * (W + 1) * 64
    wsh = torch.empty(max(1, (80 << 20) // hper) * hper * 2, dtype=torch.uint8, device=dev)

    def hvar(chunk, cols, quad=False):
        def f():
            rc = lib.voxnext_h(hm.data_ptr(), B, V, J, H, W, grids.data_ptr(), X, Y, Z, cube.data_ptr(),
                               xy.data_ptr(), wsh.data_ptr(), chunk, cols, gq2.data_ptr() if quad else None, GV2,
                               stream)
            assert rc == 0, rc
        return f
    from fvp import _lib as fl
    lib.voxnext_otf.argtypes = [vp, i_] + [i_] * 5 + [vp, vp, ctypes.POINTER(fl.GridSpec), ctypes.POINTER(fl.ImageSpec),
                                                     vp, vp, vp, i_, i_, vp]
    cams_t = torch.from_numpy(geometry.pack_cameras(cams, seq)).to(dev)
    st_, en_, ce_, nb_ = layer.grid_spec()
    gspec = fl.GridSpec((ctypes.c_float * 3)(*st_), (ctypes.c_float * 3)(*en_), (ctypes.c_float * 3)(*ce_),
                        (ctypes.c_int32 * 3)(*nb_))
    ispec = fl.ImageSpec(float(max(w.ori_image_size)), float(w.image_size[0]), float(w.image_size[1]),
                         int(w.heatmap_size[0]), int(w.heatmap_size[1]))

    def otf(chunk, cols):
        def f():
            rc = lib.voxnext_otf(hm.data_ptr(), int(hm.dtype == torch.float16), B, V, J, H, W, cams_t.data_ptr(),
                                 rt.data_ptr(), ctypes.byref(gspec), ctypes.byref(ispec), cube.data_ptr(),
                                 xy.data_ptr(), (wsh if hm.dtype == torch.float16 else ws).data_ptr(), chunk, cols, stream)
            assert rc == 0, rc
        return f
    lib.voxnext_occ.argtypes = [vp] + [i_] * 5 + [vp] + [i_] * 3 + [vp, vp, vp, i_, i_, i_, vp]

    def occ(chunk, cols, lds):
        def f():
            rc = lib.voxnext_occ(hm.data_ptr(), B, V, J, H, W, gq2.data_ptr(), X, Y, Z, cube.data_ptr(),
                                 xy.data_ptr(), ws.data_ptr(), chunk, cols, lds, stream)
            assert rc == 0, rc
        return f
    lib.voxnext_co.argtypes = lib.voxnext_otf.argtypes[:1] + lib.voxnext_otf.argtypes[2:]

    def co(chunk, cols):
        def f():
            rc = lib.voxnext_co(hm.data_ptr(), B, V, J, H, W, cams_t.data_ptr(), rt.data_ptr(), ctypes.byref(gspec),
                                ctypes.byref(ispec), cube.data_ptr(), xy.data_ptr(), wsh.data_ptr(), chunk, cols,
                                stream)
            assert rc == 0, rc
        return f
    cube = torch.empty_like(ref_cube)
    xy = torch.empty_like(ref_xy)
    per = V * H * W * 16 * 4
    chunk0 = max(1, min(B, (80 << 20) // per))
    ws = torch.empty(max(2 * chunk0, 16) * per // 4, device=dev)

    def product():
        layer.forward_fused(hm, meta, cams, rt)

    def qg(chunk, cols, mode=0, pf=1):
        def f():
            rc = lib.voxnext_qg(hm.data_ptr(), int(hm.dtype == torch.float16), B, V, J, H, W, gq.data_ptr(), GV, X, Y, Z, cube.data_ptr(),
                                xy.data_ptr(), ws.data_ptr(), chunk, cols, mode, pf, stream)
            assert rc == 0, rc
        return f

    lib.voxnext_layout.argtypes = [vp, i_] + [i_] * 5 + [vp, vp]
    fbytes = V * J * H * W * hm.element_size()

    cols0 = 1 if Z >= 320 else 320 // Z
    cands = {"product": product}

    hchunk = max(1, (80 << 20) // hper)
    if hm.dtype == torch.float16:
        for chunk in sorted({hchunk, 2 * hchunk}):
            for cols in sorted({cols0, max(1, cols0 // 2)}):
                cands[f"fp16 pair chunk={chunk} cols={cols}"] = hvar(chunk, cols)
                cands[f"fp16 pair qg chunk={chunk} cols={cols}"] = hvar(chunk, cols, True)
    if hm.dtype == torch.float32:
        for lds in (0, -1):
            cands[f"occ chunk={chunk0} cols={cols0} lds={lds >> 10}K"] = occ(chunk0, cols0, lds)
        cands[f"occ chunk={2 * chunk0} cols={cols0} lds=0"] = occ(2 * chunk0, cols0, 0)
        cands[f"occ chunk={2 * chunk0} cols={cols0} lds=40K"] = occ(2 * chunk0, cols0, 40 << 10)
    ochunk = hchunk * 2 if hm.dtype == torch.float16 else chunk0
    for cols in sorted({cols0, max(1, cols0 // 2)}):
        cands[f"otf chunk={ochunk} cols={cols}"] = otf(ochunk, cols)
    if hm.dtype == torch.float16:
        for chunk in (1, 2):
            for cols in (1, 2, 4, 5):
                cands[f"co chunk={chunk} cols={cols}"] = co(chunk, cols)
    probes = {f"probe L1-taps chunk={chunk0}": qg(chunk0, cols0, 1)}
    lay = lambda: [lib.voxnext_layout(hm.data_ptr() + c * chunk0 * fbytes, int(hm.dtype == torch.float16),
                                      min(chunk0, B - c * chunk0), V, J, H, W, ws.data_ptr(), stream)
                   for c in range((B + chunk0 - 1) // chunk0)]
    probes["layout only"] = lay
    ok = {}
    for name, f in cands.items():
        if name == "product":
            ok[name] = True
            continue
        cube.fill_(-7.0)
        xy.fill_(-7.0)
        f()
        torch.cuda.synchronize()
        ok[name] = bool(torch.equal(cube, ref_cube) and torch.equal(xy, ref_xy))
        print(f"{name}: {'exact' if ok[name] else 'MISMATCH'}", flush=True)
    cands.update(probes)
    for k in probes:
        ok[k] = True
    times = {k: [] for k in cands}
    for r in range(args.rounds):
        for name, f in cands.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / args.iters)
    per_frame = V * J * H * W * hm.element_size() + J * N * 4 + J * X * Y * 4
    for name in cands:
        t = float(np.median(times[name]))
        gbs = B * per_frame / (t * 1e-3) / 1e9
        print(f"{name:28s} {t:8.3f} ms {B / (t * 1e-3):10.0f} FPS {gbs:7.1f} GB/s ({gbs / 80:.1f}%)"
              f" {'' if ok[name] else 'WRONG'}", flush=True)


if __name__ == "__main__":
    main()
