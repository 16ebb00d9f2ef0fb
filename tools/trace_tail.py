#!/usr/bin/env python3
"""Print the last dispatches of a rocprofv3 --kernel-trace CSV in launch order
(one pipeline step's kernels, with the gap before each), so host glue kernels
can be attributed to the code that issues them.

    python tools/trace_tail.py <run_kernel_trace.csv> [--last 400]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=400)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.last:]
    prev = None
    tot = 0.0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        prev = e
        tot += (e - s) / 1e3
        print(f"{(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {r['Kernel_Name'][:110]}")
    print(f"total kernel time {tot:.1f} us over {len(rows)} dispatches")


if __name__ == "__main__":
    main()
