#!/usr/bin/env python3
"""Per-kernel PMC counters (summed over a dispatch's counter instances, then
averaged over dispatches) and kernel durations from rocprofv3's default SQLite
output (run_results.db), for runs made without --output-format csv.

    python tools/pmc_db.py [--match fvp] DIR [DIR ...]
"""
import argparse
import glob
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("--match", default="fvp")
ap.add_argument("dirs", nargs="+")
args = ap.parse_args()
for root in args.dirs:
    for f in sorted(glob.glob(f"{root}/**/*.db", recursive=True)):
        c = sqlite3.connect(f)
        name_of, agg = {}, defaultdict(lambda: defaultdict(list))
        q = ("select s.kernel_name, d.start, d.end, d.event_id from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        for name, st, en, eid in c.execute(q):
            if args.match not in name:
                continue
            name_of[eid] = name
            agg[name]["duration_us"].append((en - st) / 1e3)
        per = defaultdict(float)
        for eid, pname, val in c.execute("select e.event_id, p.name, e.value from rocpd_pmc_event e "
                                         "join rocpd_info_pmc p on e.pmc_id = p.id"):
            if eid in name_of:
                per[(eid, pname)] += val
        for (eid, pname), v in per.items():
            agg[name_of[eid]][pname].append(v)
        print(f)
        for k, d in agg.items():
            print("  " + k[:110])
            for n, v in sorted(d.items()):
                print(f"     {n:28s} {sum(v) / len(v):18.1f}  (n={len(v)})")
