#!/usr/bin/env python3
"""Per-kernel mean of each counter in rocprofv3 --pmc output directories
(*counter_collection.csv): one line per (directory, kernel, counter)."""
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = (r["Kernel_Name"].split("(")[0][:70], r["Counter_Name"])
                s = acc.setdefault(k, [0.0, 0])
                s[0] += float(r["Counter_Value"])
                s[1] += 1
    for (kn, cn), (tot, n) in sorted(acc.items(), key=lambda kv: -kv[1][0])[:6]:
        print(f"{os.path.basename(d):32s} {kn:70s} {cn:14s} mean {tot / n:14.1f} over {n}")
