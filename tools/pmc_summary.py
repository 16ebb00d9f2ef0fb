#!/usr/bin/env python3
"""Sum PMC counters per kernel over the dispatches of a tools/pmc.sh run."""
import csv
import glob
import sys

root = sys.argv[1]
agg = {}
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        d = agg.setdefault(k, {})
        c = r["Counter_Name"]
        v = d.setdefault(c, [0.0, 0])
        v[0] += float(r["Counter_Value"])
        v[1] += 1
for k, d in agg.items():
    print(k)
    for c, (s, n) in sorted(d.items()):
        print(f"   {c:40s} per-dispatch {s / n:16.1f}  (n={n})")
