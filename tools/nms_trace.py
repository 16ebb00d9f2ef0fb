#!/usr/bin/env python3
"""Median kernel duration per configuration of tools/nms_timing.py from a
rocprofv3 kernel trace (5 warm-up + 200 timed launches per configuration)."""
import csv
import json
import statistics
import sys

trace, log = sys.argv[1], sys.argv[2]
rows = [r for r in csv.DictReader(open(trace)) if "nms" in r["Kernel_Name"]]
cfgs = [json.loads(l) for l in open(log) if l.startswith("{")]
for n, c in enumerate(cfgs):
    blk = rows[n * 205 + 5:(n + 1) * 205]
    d = statistics.median(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in blk) / 1e3
    print(f'{c["X"]}x{c["Y"]} B={c["B"]} {c["map"]:6s} K={c["K"]:2d}: {d:6.2f} us  ({blk[0]["Kernel_Name"][:40]})')
