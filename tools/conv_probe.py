#!/usr/bin/env python3
"""Where a conv launch's time goes (tuning aid): each P2PNet / CenterNet layer
shape with the automatic choice, timed on the per-tap kernel only (pt), as is
(probe 0: the halo kernel where it applies), and on the per-tap kernel without
epilogue stores (1), without global loads after the first chunk (2), and with
neither (3).
Builds faster-voxelpose_amd/csrc/fvp_conv.hip with -DFVP_CONV_PROBES into
tools/libconvprobe.so."""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))


def build():
    src = os.path.join(REPO, "faster-voxelpose_amd", "csrc", "fvp_conv.hip")
    out = os.path.join(REPO, "tools", "libconvprobe.so")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        import torch

        tl = os.path.join(os.path.dirname(torch.__file__), "lib")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-DFVP_CONV_PROBES", "-I", os.path.join(REPO, "include"), "-c", src,
                        "-o", out + ".o"], check=True)
        subprocess.run(["g++", "-shared", "-o", out, out + ".o", f"-L{tl}", "-l:libamdhip64.so",
                        f"-Wl,-rpath,{tl}"], check=True)
    return out


def main():
    path = build()
    import numpy as np
    import torch
    import torch.nn as nn

    from fvp import cnn
    from fvp.ops import _ptr, _stream

    lib = ctypes.CDLL(path)
    vp, i_ = ctypes.c_void_p, ctypes.c_int
    lib.fvp_conv_probe.argtypes = [i_, vp, i_, i_, i_, i_, vp, i_, i_, i_, i_, vp, vp, vp, vp, i_, i_, vp, vp]
    dev = torch.device("cuda:0")
    imgs = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    lib.fvp_conv_set_tile.argtypes = [i_]
    shapes = [("7x7 15->16 @64", 15, 16, 7, 64, False), ("3x3 16->32 @64", 16, 32, 3, 64, False),
              ("3x3 32->32 @64", 32, 32, 3, 64, False), ("3x3 64->64 @32", 64, 64, 3, 32, False),
              ("3x3 128->128 @16", 128, 128, 3, 16, False), ("convT 128->64 @16", 128, 64, 2, 16, True)]
    cn_imgs = int(sys.argv[2]) if len(sys.argv) > 2 else 8  # CenterNet's shapes (80x80 maps per frame)
    shapes += [(f"CN {n}", ci, co, k, hw, up, cn_imgs) for n, ci, co, k, hw, up in
               [("7x7 15->16 @80", 15, 16, 7, 80, False), ("3x3 16->32 @80", 16, 32, 3, 80, False),
                ("3x3 32->32 @80", 32, 32, 3, 80, False), ("3x3 64->64 @40", 64, 64, 3, 40, False),
                ("3x3 128->128 @20", 128, 128, 3, 20, False)]]
    for shp in shapes:
        name, cin, cout, k, hw, up = shp[:6]
        n_img = shp[6] if len(shp) > 6 else imgs
        conv = (nn.ConvTranspose2d(cin, cout, 2, stride=2) if up else nn.Conv2d(cin, cout, k, padding=k // 2)).to(dev)
        L = cnn.ConvLayer(conv, None)
        x = cnn.to_nhwc(torch.rand((n_img, cin, hw, hw), device=dev))
        Ho, Wo = (2 * hw, 2 * hw) if up else (hw, hw)
        out = torch.empty((n_img, Ho, Wo, L.Cpo), device=dev)
        flops = L.flops(x)
        row = []
        # "pt": probe 0 with the halo kernel off (per-tap implicit GEMM); p0 = default choice
        for probe in ["pt", 0, 1, 2, 3]:
            lib.fvp_conv_set_tile(-1 if probe == "pt" else -2)
            pr = 0 if probe == "pt" else probe

            def f():
                rc = lib.fvp_conv_probe(pr, _ptr(x.t), x.N, x.H, x.W, x.Cp, _ptr(L.wpack), L.KH, L.KW, L.Cpo,
                                        L.Cpo_w, _ptr(L.scale), _ptr(L.shift), None, None, 1, L.up2, _ptr(out),
                                        _stream(out))
                assert rc == 0, rc
            f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(3):
                e0.record()
                for _ in range(10):
                    f()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            t = float(np.median(ts))
            row.append(f"{probe if probe == 'pt' else 'p' + str(probe)} {t * 1e3:7.1f} us {flops / (t * 1e-3) / 1e12:6.1f} TF")
        print(f"{name:20s} " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
