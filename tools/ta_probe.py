#!/usr/bin/env python3
"""Measure per-CU cost of one wave64 vector load vs access pattern (see ta_probe.hip)."""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build():
    import torch

    src = os.path.join(REPO, "tools", "ta_probe.hip")
    out = os.path.join(REPO, "tools", "libtaprobe.so")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        tl = os.path.join(os.path.dirname(torch.__file__), "lib")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-c", src, "-o", out + ".o"],
                       check=True)
        subprocess.run(["g++", "-shared", "-o", out, out + ".o", f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"],
                       check=True)
    return out


def patterns(width, rng):
    lane = np.arange(64)
    p = {
        "coalesced": lane * width,
        "same_addr": np.zeros(64, int),
        "lane_per_128B": lane * 128,
        "lane_per_64B": lane * 64,
        "2_per_128B_adj": (lane // 2) * 128 + (lane % 2) * width,
        "4_per_128B_adj": (lane // 4) * 128 + (lane % 4) * width,
        "4_per_128B_scat": (lane % 16) * 128 + (lane // 16) * width,
        "16_per_128B_adj": (lane // 16) * 128 + (lane % 16) * min(width, 8),
        "voxel_like_16rows": (lane // 4) * 960 + rng.integers(0, 15, 64) * 4 // width * width,
        "voxel_like_8rows": (lane // 8) * 960 + rng.integers(0, 30, 64) * 4 // width * width,
    }
    return {k: np.asarray(v, np.uint32) for k, v in p.items()}


def main():
    path = build()
    import torch

    lib = ctypes.CDLL(path)
    lib.ta_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint,
                             ctypes.c_uint, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    buf = torch.rand(64 * 1024 * 1024 // 4 + 65536, device=dev)
    blocks = ncu * 8
    out = torch.empty(blocks * 256, device=dev)
    iters = 200
    rng = np.random.default_rng(0)
    stream = torch.cuda.current_stream().cuda_stream
    print(f"CUs={ncu}; cycles per wave-load per CU assume 2.4 GHz")
    for span_name, span, step in (("L1 (16KB)", 16384, 1024), ("L2 (2MB)", 2 << 20, 16384 + 128),
                                  ("MALL (48MB)", 48 << 20, 262144 + 128)):
        for width in (4, 8, 16):
            for name, offs in patterns(width, rng).items():
                lo = torch.from_numpy(offs.astype(np.int64)).to(torch.int32).to(dev)
                lib.ta_probe(width, buf.data_ptr(), lo.data_ptr(), 5, step, span, out.data_ptr(), blocks, stream)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                lib.ta_probe(width, buf.data_ptr(), lo.data_ptr(), iters, step, span, out.data_ptr(), blocks, stream)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1)
                instr = blocks * 4 * iters * 16
                cyc = ms * 1e-3 * 2.4e9 * ncu / instr
                gbs = instr * 64 * width / (ms * 1e-3) / 1e9
                print(f"{span_name:12s} w={width:2d} {name:20s} {cyc:7.2f} cyc/instr/CU  {gbs:8.0f} GB/s lane-bytes",
                      flush=True)


if __name__ == "__main__":
    main()
