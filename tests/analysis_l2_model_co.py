#!/usr/bin/env python3
"""LRU model of one XCD's 4 MB L2 (tests/analysis_l2_model.py's C2 geometry and
line stream) for the camera-outer block the round-3 VERDICT asked about:
blocks of `cols` columns x all z, layer-major slots (a wave = 16 columns of one
z-layer when cols = 16), each block processing all its voxels camera by camera
(accumulators held in the block's stage), 256 resident blocks per XCD refilled
in the product's band-16 walk -- against the product's order (`base`: 8-column
blocks, cameras inner per 64-voxel pass).  CPU analysis (minutes).

    python tests/analysis_l2_model_co.py base 8 256 1      # -> see DESIGN.md section 5
    python tests/analysis_l2_model_co.py co 16 256 1       # -> 145536 (per-camera grid layout)
(round 4; compulsory: 77 k table + 40 k grid lines)
"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
_src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "analysis_l2_model.py")).read()
exec(_src.split("cols=8\nvariants")[0])  # geometry, per-voxel tap lines, block_cols (no simulation runs)


def sim_co(order_blocks, resident=256, cap_lines=32768, camouter=True, frames=1):
    cache = collections.OrderedDict()
    st = [0, 0]

    def acc(line):
        if line in cache:
            cache.move_to_end(line)
            st[0] += 1
        else:
            st[1] += 1
            cache[line] = 1
            if len(cache) > cap_lines:
                cache.popitem(last=False)

    queue = [(f, b) for f in range(frames) for b in order_blocks]
    active = []

    def start():
        f, cols_ = queue.pop(0)
        T = len(cols_) * Z
        slots = [(cols_[s % len(cols_)], s // len(cols_)) for s in range(T)]
        return [f, slots, 0, (T + 63) // 64]

    while queue and len(active) < resident:
        active.append(start())
    while active:
        nxt = []
        for a in active:
            f, slots, u, P = a
            if camouter:
                ci, p = divmod(u, P)
                cams_ = [ci]
            else:
                p, cams_ = u, range(V)
            part = slots[p * 64:(p + 1) * 64]
            if not camouter:  # the product's packed grid [N][GV][2]: 48 B per voxel, read once per pass
                for (col, z) in part:
                    acc(GRID_BASE + ((col * Z + z) * 48) // 128)
            for ci in cams_:
                if camouter:  # a per-camera coordinate layout [V][N][2]
                    for (col, z) in part:
                        acc(GRID_BASE + ci * 10 ** 7 + ((col * Z + z) * 8) // 128)
                for (col, z) in part:
                    for ln in lines[col * Z + z, ci]:
                        if ln >= 0:
                            acc(int(ln) + f * 10 ** 8)
            a[2] += 1
            if a[2] < (P * V if camouter else P):
                nxt.append(a)
            elif queue:
                nxt.append(start())
        active = nxt
    return st


if __name__ == "__main__":
    mode, cols, res = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    frames = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    order = [block_cols(cb, cols, 16) for cb in range((X * Y) // cols)]
    h, m = sim_co(order, resident=res, camouter=(mode == "co"), frames=frames)
    print(mode, "cols", cols, "resident", res, "frames", frames, "misses", m, "per frame", m / frames, flush=True)
