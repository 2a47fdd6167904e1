"""Idle gaps inside the prefill passes of a rocprofv3 kernel trace (--kernel-trace CSV).

A pass runs from an embed_kernel followed by the plain rmsnorm_kernel (the prefill layer
path; decode starts with residual_rmsnorm) to the argmax after it; prints, per pass, the wall span, the summed kernel time, and the largest gaps
between consecutive kernels with the names on both sides.
    usage: python3 tools/trace_gaps.py <kernel_trace.csv>
"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows)
    passes, cur = [], None
    for i, k in enumerate(ks):
        if "embed_kernel" in k[2] and i + 1 < len(ks) and ks[i + 1][2].startswith("ms::rmsnorm_kernel"):
            cur = [k]
            continue
        if cur is not None:
            cur.append(k)
            if "argmax_kernel" in k[2]:
                passes.append(cur)
                cur = None
    for i, p in enumerate(passes):
        span = (p[-1][1] - p[0][0]) / 1e6
        busy = sum(k[1] - k[0] for k in p) / 1e6
        gaps = sorted(((p[j + 1][0] - p[j][1]) / 1e3, p[j][2], p[j + 1][2]) for j in range(len(p) - 1))[::-1]
        print(f"pass {i}: {len(p)} kernels, span {span:.2f} ms, kernels {busy:.2f} ms, idle {span - busy:.2f} ms")
        for g in gaps[:3]:
            print(f"   gap {g[0]:9.1f} us  after {g[1]}  before {g[2]}")
        per = {}
        for k in p:
            t = per.setdefault(k[2], [0, 0.0])
            t[0] += 1
            t[1] += (k[1] - k[0]) / 1e3
        for name, (n, us) in sorted(per.items(), key=lambda x: -x[1][1])[:8]:
            print(f"   {us / 1e3:8.2f} ms  {n:4d} x {us / n:8.1f} us  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
