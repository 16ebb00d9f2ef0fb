"""Heatmap footprint of voxel tiles per camera (analysis for LDS-staged gathers).

For each tile of TXxTYxTZ voxels and each camera: the row hulls of the pixels
its bilinear taps read, against the tap count.  A staged/taps ratio well
below 1 means staging the footprint moves fewer bytes than reading the taps.

    python tools/footprint_stats.py c5 8x8x64 16x16x16
"""
import sys
import warnings

import numpy as np

sys.path[:0] = ['.', 'faster-voxelpose_amd']
from fvp.geometry import camera_list, resize_transform  # noqa: E402
from fvp.workloads import WORKLOADS  # noqa: E402
from oracle import fvp_oracle as O  # noqa: E402

warnings.filterwarnings('ignore')


def main():
    name = sys.argv[1]
    shapes = [tuple(map(int, s.split('x'))) for s in sys.argv[2:]]
    w = WORKLOADS[name]
    cams, seq = w.cameras()
    X, Y, Z = w.voxels_per_axis
    grid = O.compute_grid(w.space_size, w.space_center, w.voxels_per_axis)
    rt = resize_transform(w.ori_image_size, w.image_size).astype(np.float32)
    Wh, Hh = w.heatmap_size
    res = {s: [0, 0, []] for s in shapes}
    tile_sum = {s: {} for s in shapes}  # per tile: pixels summed over cameras (4-px units, +2 pad px per row)
    for c in camera_list(cams, seq)[:6]:
        g = O.project_grid(grid, c, w.ori_image_size, w.image_size, w.heatmap_size, rt).reshape(X, Y, Z, 2)
        ix = (g[..., 0] + 1) * np.float32((Wh - 1) / 2)
        iy = (g[..., 1] + 1) * np.float32((Hh - 1) / 2)
        x0 = np.floor(ix).astype(np.int32)
        y0 = np.floor(iy).astype(np.int32)
        for (tx, ty, tz) in shapes:
            r = res[(tx, ty, tz)]
            for a in range(0, X, tx):
                for b in range(0, Y, ty):
                    for cz in range(0, Z, tz):
                        xs = x0[a:a + tx, b:b + ty, cz:cz + tz].ravel()
                        ys = y0[a:a + tx, b:b + ty, cz:cz + tz].ravel()
                        m = (xs >= -1) & (xs < Wh) & (ys >= -1) & (ys < Hh)
                        if not m.any():
                            continue
                        xs, ys = xs[m], ys[m]
                        r[0] += 4 * int(m.sum())
                        lo = np.full(Hh, 10 ** 9)
                        hi = np.full(Hh, -10 ** 9)
                        for dy in (0, 1):
                            yy = ys + dy
                            k = (yy >= 0) & (yy < Hh)
                            np.minimum.at(lo, yy[k], xs[k])
                            np.maximum.at(hi, yy[k], xs[k] + 1)
                        lo = np.maximum(lo, 0)
                        hi = np.minimum(hi, Wh - 1)
                        px = int(np.where(hi >= lo, hi - lo + 1, 0).sum())
                        r[1] += px
                        r[2].append(px)
                        u = np.where(hi >= lo, (hi >> 2) - (lo >> 2) + 1, 0)
                        tile_sum[(tx, ty, tz)][(a, b, cz)] = (tile_sum[(tx, ty, tz)].get((a, b, cz), 0)
                                                             + int((4 * u + 2 * (u > 0)).sum()))
    for s, (taps, px, lst) in res.items():
        a = np.array(lst)
        print(f"{name} tile {s}: staged px/taps {px / taps:.3f}; per tile-camera px mean {a.mean():.0f} "
              f"p99 {np.percentile(a, 99):.0f} max {a.max()} (KB at 64 B/px: mean {a.mean() * 64 / 1024:.0f}, "
              f"max {a.max() * 64 / 1024:.0f})")
        ts = np.array(list(tile_sum[s].values()))
        print(f"   per tile, summed over cameras (4-px units + pad): mean {ts.mean():.0f} px, p99 "
              f"{np.percentile(ts, 99):.0f}, max {ts.max()} -> KB per fp32 joint: mean {ts.mean() * 4 / 1024:.1f} "
              f"max {ts.max() * 4 / 1024:.1f}")


if __name__ == "__main__":
    main()
