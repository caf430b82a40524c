"""Summarise a rocprofv3 --stats kernel CSV (and the per-iteration trace) for quick reading."""
import csv
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(d + "/run_kernel_stats.csv")))
tot = sum(float(x["TotalDurationNs"]) for x in rows)
for x in rows:
    print(f"{x['Name'][:70]:70s} calls={int(x['Calls']):6d} total_ms={float(x['TotalDurationNs'])/1e6:9.2f} "
          f"avg_us={float(x['AverageNs'])/1e3:9.2f} pct={float(x['Percentage']):6.2f}")
print(f"total kernel time {tot/1e6:.2f} ms")
