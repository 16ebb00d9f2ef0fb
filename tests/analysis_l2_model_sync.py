#!/usr/bin/env python3
"""LRU model of one XCD's 4 MB L2 for a camera-synchronous C2 gather at a
residency a real kernel can hold: accumulators in LDS
(64 B per voxel: 16 joints fp32), so a CU holds at most 160 KB / 64 B = 2,560
voxels; R resident blocks of T voxels per XCD (32 CUs) take the frame's
columns in rounds (each block's tile = its columns x all z, layer-major
slots as in the product), and within a round every block walks its tile
camera by camera, 64-voxel passes, the camera's coordinates read from a
per-camera [V][N][2] grid (8 B per voxel-camera).  Blocks drift: block i runs
`off_i` passes behind the front, off_i uniform in [0, DRIFT passes]; with the
per-XCD camera phase a block never runs more than one camera ahead of the
slowest, which bounds the drift to one camera's passes.

CPU analysis over the oracle geometry (tests/analysis_l2_model.py's line
stream); minutes.

    python tests/analysis_l2_model_sync.py T R DRIFT_CAMERAS [frames [zsplit]]
    python tests/analysis_l2_model_sync.py 240 256 1        # 8 blocks/CU x 240 voxels (15 KB LDS each)
    python tests/analysis_l2_model_sync.py base             # the product's order, for comparison
    GRID=packed python tests/analysis_l2_model_sync.py 160 192 1   # coordinates from the packed [N][GV][2] grid
"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
_src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "analysis_l2_model.py")).read()
exec(_src.split("cols=8\nvariants")[0])  # geometry, per-voxel tap lines, block_cols (no simulation runs)


PACKED = os.environ.get("GRID", "percam") == "packed"


def band_columns(band=16):
    """The frame's columns in the product's band walk (column groups of 8, bands of 16 x-rows)."""
    out = []
    for cb in range((X * Y) // 8):
        out += block_cols(cb, 8, band)
    return out


def sim_sync(T, R, drift_cams, frames=1, cap_lines=32768, seed=0, zsplit=1):
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

    cols_per_block = max(1, T // Z)
    walk = band_columns()
    rng = np.random.default_rng(seed)
    for f in range(frames):
        # rounds: R blocks take consecutive runs of columns of the walk; with
        # zsplit > 1 the frame is taken as zsplit z-ranges (all columns of the
        # lower layers first), a tile = cols x the range's layers
        zl = (Z + zsplit - 1) // zsplit
        cpb = max(1, T // zl)
        tiles = [(walk[i:i + cpb], z0, min(Z, z0 + zl)) for z0 in range(0, Z, zl)
                 for i in range(0, len(walk), cpb)]
        for r0 in range(0, len(tiles), R):
            blocks = tiles[r0:r0 + R]
            P = [(len(b) * (z1 - z0) + 63) // 64 for b, z0, z1 in blocks]
            slots = [[(b[s % len(b)], z0 + s // len(b)) for s in range(len(b) * (z1 - z0))] for b, z0, z1 in blocks]
            Pm = max(P)
            off = rng.integers(0, int(drift_cams * Pm) + 1, len(blocks)) if drift_cams else np.zeros(len(blocks), int)
            steps = Pm * V + int(off.max())
            for t in range(steps):
                for i in range(len(blocks)):
                    tt = t - off[i]
                    if tt < 0 or tt >= P[i] * V:
                        continue
                    ci, p = divmod(tt, P[i])
                    part = slots[i][p * 64:(p + 1) * 64]
                    if PACKED:  # [N][GV][2] records of 48 B, cameras (ci, ci + 1) from one 16-B load
                        if ci % 2 == 0:
                            for (col, z) in part:
                                acc(GRID_BASE + ((col * Z + z) * 48 + 8 * ci) // 128)
                    else:  # per-camera [V][N][2]
                        for (col, z) in part:
                            acc(GRID_BASE + ci * 10 ** 7 + ((col * Z + z) * 8) // 128)
                    for (col, z) in part:
                        for ln in lines[col * Z + z, ci]:
                            if ln >= 0:
                                acc(int(ln) + f * 10 ** 8)
    return st


if __name__ == "__main__":
    if sys.argv[1] == "base":
        import analysis_l2_model_co as co  # noqa: E402  (the product's order)
        h, m = co.sim_co([block_cols(cb, 8, 16) for cb in range((X * Y) // 8)], resident=256, camouter=False)
        print("product order: misses", m, flush=True)
        sys.exit(0)
    T, R, drift = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
    frames = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    zsplit = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    h, m = sim_sync(T, R, drift, frames, zsplit=zsplit)
    table = len(set(int(x) for x in lines[lines >= 0].ravel()))
    print(f"sync T {T} R {R} drift {drift} cameras zsplit {zsplit}: misses per frame {m / frames:.0f} "
          f"(table lines {table}, grid lines {X * Y * Z * V * 8 // 128}), hit {h / (h + m):.3f}", flush=True)
