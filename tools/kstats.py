"""Print per-kernel averages from a rocprofv3 kernel_stats.csv: python tools/kstats.py FILE [substr...]"""
import csv, sys
subs = sys.argv[2:] or [""]
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(x in n for x in subs):
        print(f"{n[:64]:64s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e6:9.3f} ms")
