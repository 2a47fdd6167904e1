"""Summarise a rocprofv3 --stats kernel_stats.csv: per-kernel calls / total / average."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':78s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for r in rows:
    print(f"{r['Name'][:78]:78s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:10.2f} "
          f"{float(r['AverageNs'])/1e3:9.2f} {100*float(r['TotalDurationNs'])/tot:6.1f}")
print(f"{'TOTAL':78s} {'':7s} {tot/1e6:10.2f}")
