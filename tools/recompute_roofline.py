#!/usr/bin/env python3
"""Recompute the headline roofline fraction from tracked files.

Reads a closing run's bench line (bench.json: algorithmic bytes per op, the
event-timed op time, the counter traffic) and the per-launch-shape summary of
the rocprofv3 kernel trace of the same command (launch_shapes.csv, from
tools/launch_shapes.py), and prints the op's kernel time rebuilt from the
launch shapes: per step, ceil(B / 12) layout + gather launches of the 12-frame
chunks plus the tail chunk's pair.  The shapes are told apart by their
dispatch counts: (steps + warmup) x chunks for the full chunks,
(steps + warmup) for the tail; the 256-frame channels-last launches and the
one-frame latency launches of the same run have other counts and are left out.

    python3 tools/recompute_roofline.py profiles/round5/closing
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

GATHER, LAYOUT = "voxelize_kernel", "heatmaps_to_cl_kernel"
CHUNK = 12  # frames per layout + gather launch pair (fvp_voxelize's chunking)


def main(d):
    line = json.loads(open(os.path.join(d, "bench.json")).read().splitlines()[-1])
    r = line["roofline"]
    runs = line["steps"] + line["warmup"]
    B = line["config"]["frames_per_gpu_step"]
    full, tail = B // CHUNK, B % CHUNK
    rows = list(csv.DictReader(open(os.path.join(d, "launch_shapes.csv"))))

    def pick(kernel, count):
        hits = [x for x in rows if kernel in x["kernel"] and int(x["count"]) == count]
        if len(hits) != 1:
            raise SystemExit(f"{kernel}: {len(hits)} launch shapes with {count} dispatches")
        return float(hits[0]["median_us"]), int(hits[0]["blocks"])

    g, gb = pick(GATHER, runs * full)
    lay, lb = pick(LAYOUT, runs * full)
    us = full * (g + lay)
    print(f"12-frame chunk: gather {g:.2f} us ({gb} blocks) + layout {lay:.2f} us ({lb} blocks), x {full}")
    if tail:
        tg, _ = pick(GATHER, runs)
        tl, _ = pick(LAYOUT, runs)
        us += tg + tl
        print(f"{tail}-frame tail: gather {tg:.2f} us + layout {tl:.2f} us")
    alg = r["algorithmic_bytes_per_launch"]
    per_chunk = alg / B * CHUNK / ((g + lay) * 1e-6)
    print(f"op from the trace medians: {us / 1e3:.4f} ms; from the bench's HIP events: {r['kernel_ms']:.4f} ms")
    print(f"algorithmic bytes per op: {alg / 1e9:.4f} GB ({B} frames)")
    print(f"frac per 12-frame chunk: {per_chunk / 1e9:.1f} GB/s = {per_chunk / (r['peak'] * 1e9):.4f}")
    print(f"frac of the op (trace): {alg / (us * 1e-6) / (r['peak'] * 1e9):.4f}; bench line: {r['frac']:.4f}")
    fetch = glob.glob(os.path.join(d, "pmc_fetch", "**", "*counter_collection.csv"), recursive=True)
    write = glob.glob(os.path.join(d, "pmc_write", "**", "*counter_collection.csv"), recursive=True)
    if fetch and write:
        # the same split and corrections as bench.py (layout FETCH x2; gather FETCH raw .. x2)
        t = bench.traffic_from_csvs(fetch, write, bench.CHILD_OPS)
        print(f"counter traffic per op (pmc_fetch/, pmc_write/): layout pass {t['layout'] / 1e9:.3f} GB "
              f"(2 x {t['layout_fetch_raw'] / 1e9:.3f} fetch + {t['layout_write'] / 1e9:.3f} write), gather "
              f"{t['gather'] / 1e9:.3f} GB ({t['gather_fetch_raw'] / 1e9:.3f} raw fetch + {t['gather_write'] / 1e9:.3f} write)")
        print(f"traffic {t['traffic'] / 1e9:.3f} GB = {t['traffic'] / alg:.2f}x algorithmic; with the gather's fetch "
              f"doubled too {t['traffic_upper'] / 1e9:.3f} GB = {t['traffic_upper'] / alg:.2f}x")
        if r.get("traffic") is not None:
            print(f"bench line: traffic {r['traffic'] / 1e9:.3f} GB"
                  + (f", traffic_upper {r['traffic_upper'] / 1e9:.3f} GB" if "traffic_upper" in r else ""))
    if "ceiling" in r:
        c = r["ceiling"]
        print(f"ceiling: {c['frac']:.4f} ({c['tap_floor_us_per_frame']} us/frame tap floor + "
              f"{c['layout_us_per_frame']} us/frame layout); frac of ceiling {r['frac'] / c['frac']:.4f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/round5/closing")
