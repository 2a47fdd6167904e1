"""Summarise a rocprofv3 --pmc counter_collection.csv: mean counter value per dispatch,
per kernel name (FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced streaming reads -- MI355X_MICROARCH.md §HBM -- so x2 is shown)."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: [0.0, 0])
for r in csv.DictReader(open(sys.argv[1])):
    name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
    cname = r.get("Counter_Name") or r.get("Counter-Name")
    val = float(r.get("Counter_Value") or r.get("Counter-Value") or 0)
    key = (name, cname)
    acc[key][0] += val
    acc[key][1] += 1
print(f"{'kernel':70s} {'counter':12s} {'dispatches':>10s} {'mean/dispatch':>14s} {'x2 (gfx950 FETCH corr.)':>24s}")
for (name, cname), (tot, n) in sorted(acc.items(), key=lambda kv: -kv[1][0]):
    mean = tot / n
    corr = mean * 2 if cname == "FETCH_SIZE" else mean
    print(f"{name[:70]:70s} {cname:12s} {n:10d} {mean:14.1f} {corr:24.1f}")
