"""HBM traffic per launch of one kernel class from two rocprofv3 --pmc passes.

usage: traffic_from_pmc.py <fetch counter_collection.csv> <write counter_collection.csv>
                           <kernel-name substring> <out.json> [chunks_per_gpu prompt_len]

The optional workload (default 8 x 2048, bench.py's default) is stored with the result:
bench.py only quotes the figure for a run of the same workload.

FETCH_SIZE and WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads (MI355X_MICROARCH.md §HBM), so it is doubled; WRITE_SIZE
is exact for 16-B/lane stores and float atomics.  traffic = 1024 * (2*FETCH + WRITE)
averaged over the class's dispatches.
"""
import collections
import csv
import json
import sys


def per_dispatch(path, counter, sub):
    vals = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if sub not in name or (r.get("Counter_Name") or r.get("Counter-Name")) != counter:
            continue
        d = r.get("Dispatch_Id") or r.get("Dispatch-Id") or r.get("Correlation_Id")
        vals[d] += float(r.get("Counter_Value") or r.get("Counter-Value") or 0)
        names[d] = name
    return vals, names


def main():
    fpath, wpath, sub, out = sys.argv[1:5]
    B = int(sys.argv[5]) if len(sys.argv) > 5 else 8
    P = int(sys.argv[6]) if len(sys.argv) > 6 else 2048
    f, fn = per_dispatch(fpath, "FETCH_SIZE", sub)
    w, _ = per_dispatch(wpath, "WRITE_SIZE", sub)
    assert f and w, "no dispatches of that kernel in the counter files"
    fetch = sum(f.values()) / len(f) * 1024
    write = sum(w.values()) / len(w) * 1024
    by_inst = collections.defaultdict(list)
    for d, v in f.items():
        by_inst[fn[d].split("(")[0]].append(v * 2 * 1024)
    res = {"kernel_substring": sub, "dispatches_fetch": len(f), "dispatches_write": len(w),
           "fetch_size_bytes_raw": round(fetch), "fetch_bytes_corrected_x2": round(2 * fetch),
           "write_bytes": round(write), "traffic_bytes_per_launch": round(2 * fetch + write),
           "fetch_x2_by_instantiation": {k: round(sum(v) / len(v)) for k, v in by_inst.items()},
           "workload": {"chunks_per_gpu": B, "prompt_len": P}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
