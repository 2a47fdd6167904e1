"""Summary of tools/qdgemm_traffic.sh: per shape, the K-quant launches' (QT 12 / 14) HBM bytes
(2 x FETCH_SIZE + WRITE_SIZE, KB counters; gfx950 FETCH_SIZE halves wide streaming reads,
MI355X_MICROARCH.md §HBM) against the algorithmic bytes of one launch: the packed weight blocks
and the M x K fp16 activations read once, the outputs written once (fp32 split-K slabs, fp16
SwiGLU rows, or the argmax partials).

usage: qdgemm_traffic.py <dir of <shape>.<COUNTER>/ runs> <rows M>"""
import collections
import csv
import glob
import json
import os
import sys

SHAPES = {"qkv": (5120, 3072, 144), "o": (3072, 3072, 144), "gu": (16384, 3072, 144),
          "down": (3072, 8192, 144), "down6": (3072, 8192, 224), "lm_head6": (128256, 3072, 224)}


def per_launch(path, counter):
    """{S-less instantiation: [bytes per dispatch]} of the K-quant qdgemm launches."""
    vals, names = collections.defaultdict(float), {}
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or ""
        if "qdgemm_kernel<" not in name or r.get("Counter_Name") != counter:
            continue
        targs = [a.strip() for a in name.split("<", 1)[1].split(">", 1)[0].split(",")]
        if targs[2] not in ("12", "14"):  # <MT, EPI, QT, DPF>: skip the fp16-rows form (QT 1)
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[d] += float(r.get("Counter_Value") or 0) * 1024
        names[d] = "qdgemm_kernel<" + ", ".join(targs) + ">"
    out = collections.defaultdict(list)
    for d, v in vals.items():
        out[names[d]].append(v)
    return out


def main():
    root, M = sys.argv[1], int(sys.argv[2])
    res = {"rows": M, "method": __doc__.split("\n\n")[0], "shapes": {}}
    for sh, (N, K, bpb) in SHAPES.items():
        fc = glob.glob(os.path.join(root, f"{sh}.FETCH_SIZE", "**", "*counter_collection.csv"), recursive=True)
        wc = glob.glob(os.path.join(root, f"{sh}.WRITE_SIZE", "**", "*counter_collection.csv"), recursive=True)
        if not fc or not wc:
            continue
        f, w = per_launch(fc[0], "FETCH_SIZE"), per_launch(wc[0], "WRITE_SIZE")
        fetch = [2 * v for vs in f.values() for v in vs]
        write = [v for vs in w.values() for v in vs]
        if not fetch or not write:
            continue
        wbytes = N * (K // 256) * bpb
        rd = wbytes + M * K * 2
        # the microbench's launches: S = 1 for gu / lm_head (SwiGLU, argmax), else split-K slabs
        outb = M * N if sh == "gu" else (M * (N // 16) * 8 if sh == "lm_head6" else None)
        fa, wa = sum(fetch) / len(fetch), sum(write) / len(write)
        e = {"weight_bytes": wbytes, "algorithmic_read_bytes": rd, "fetch_x2_per_launch": round(fa),
             "read_ratio": round(fa / rd, 3), "write_per_launch": round(wa), "dispatches": len(fetch),
             "instantiations": sorted(f)}
        if outb is not None:
            e["algorithmic_write_bytes"] = outb
            e["traffic_ratio"] = round((fa + wa) / (rd + outb), 3)
        res["shapes"][sh] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
