"""Summarise a rocprofv3 kernel trace: per-kernel calls / total / average.

Accepts either the --stats kernel_stats.csv (``--output-format csv``), the default
rocpd SQLite database (``*_results.db``, view ``top_kernels``), or a kernel_trace.csv --
the last one grouped by (kernel, grid size), so launches of one kernel on different shapes
(O vs down projection) get rows of their own."""
import csv
import sqlite3
import sys


def rows_of(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, calls, total, avg, _ in c.execute("select * from top_kernels"):
            yield name, int(calls), float(total) * 1e3, float(avg) * 1e3  # view is in us
    elif path.endswith("kernel_trace.csv"):
        agg = {}
        for r in csv.DictReader(open(path)):
            grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
            k = f"{r['Kernel_Name'][:60]} g={grid}"
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            c, t = agg.get(k, (0, 0))
            agg[k] = (c + 1, t + d)
        for k, (c, t) in agg.items():
            yield k, c, float(t), float(t) / c
    else:
        for r in csv.DictReader(open(path)):
            yield r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"])


rows = sorted(rows_of(sys.argv[1]), key=lambda r: -r[2])
tot = sum(r[2] for r in rows)
print(f"{'kernel':78s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for name, calls, total, avg in rows:
    print(f"{name[:78]:78s} {calls:7d} {total / 1e6:10.2f} {avg / 1e3:9.2f} {100 * total / tot:6.1f}")
print(f"{'TOTAL':78s} {'':7s} {tot / 1e6:10.2f}")
