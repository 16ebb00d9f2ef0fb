"""Print the top kernels of rocprofv3 kernel_stats.csv files and the bench line (A/B helper)."""
import csv
import json
import sys

for d in sys.argv[1:]:
    print("==", d)
    rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    for x in rows[:6]:
        print(f"  {x['Name'][:64]:64s} {x['Calls']:>5s} {float(x['AverageNs']) / 1000:9.1f} us avg")
    try:
        line = [l for l in open(d + ".log") if l.startswith("{")][-1]
        b = json.loads(line)
        print(f"  value {b['value']:.0f} {b['unit']}  op {b['roofline']['kernel_ms']} ms  frac {b['roofline']['frac']}")
    except (IndexError, OSError, KeyError):
        pass
