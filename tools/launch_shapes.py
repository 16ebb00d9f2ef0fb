"""Per-launch-shape summary of a rocprofv3 kernel trace (`--kernel-trace`,
`*_kernel_trace.csv`): one row per (kernel, grid, workgroup) with the dispatch
count and the median / mean / p5 / p95 duration, so a roofline fraction can be
recomputed from tracked files (kernel_stats.csv averages every shape of a
kernel into one row).

    python3 tools/launch_shapes.py <rocprofv3 output dir> [--csv out.csv] [--top N]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import statistics


def load(d):
    files = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {d}")
    shapes = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                grid = tuple(int(r[f"Grid_Size_{a}"]) for a in "XYZ")
                wg = tuple(int(r[f"Workgroup_Size_{a}"]) for a in "XYZ")
                us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
                shapes.setdefault((name, grid, wg), []).append(us)
    return shapes


def summarise(shapes):
    rows = []
    for (name, grid, wg), ts in shapes.items():
        ts = sorted(ts)
        n = len(ts)
        blocks = 1
        for g, w in zip(grid, wg):
            blocks *= max(1, g // max(1, w))
        rows.append({"kernel": name.split("(")[0][:120], "grid": "x".join(map(str, grid)),
                     "workgroup": "x".join(map(str, wg)), "blocks": blocks, "count": n,
                     "median_us": round(statistics.median(ts), 3), "mean_us": round(sum(ts) / n, 3),
                     "p5_us": round(ts[int(0.05 * (n - 1))], 3), "p95_us": round(ts[int(0.95 * (n - 1))], 3),
                     "total_us": round(sum(ts), 1)})
    rows.sort(key=lambda r: -r["total_us"])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    rows = summarise(load(a.dir))
    if a.csv:
        with open(a.csv, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(rows)
    for r in rows[:a.top]:
        print(f"{r['kernel'][:60]:60s} blocks {r['blocks']:>7d} n {r['count']:>5d} "
              f"median {r['median_us']:>9.2f} us  mean {r['mean_us']:>9.2f}  p5-p95 {r['p5_us']:.1f}-{r['p95_us']:.1f}")


if __name__ == "__main__":
    main()
