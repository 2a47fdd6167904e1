"""Prefill MFMA utilisation per kernel from one rocprofv3 --pmc pass
(SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE; SURVEY.md §8d / north_star "prefill MFMA
utilisation against bf16 peak").

usage: mfma_from_pmc.py <counter_collection.csv> <out.json> [kernel substrings...]

Per dispatch, rows of one counter are summed (rocprofv3 may split a counter over
instances).  MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe cycles
(16 per v_mfma_f32_16x16x32_f16 (or _bf16) = 16,384 FLOP, i.e. 1,024 FLOP per busy cycle) summed over
every SIMD; GRBM_GUI_ACTIVE is the busy clock summed over the 8 XCDs.  So
    util = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
is the fraction of the chip's matrix-pipe cycles the kernel kept busy while it ran,
clock-independent; implied_flop = MFMA_BUSY * 1024 cross-checks the algorithmic FLOP.
"""
import collections
import csv
import json
import sys

SIMDS = 256 * 4
FLOP_PER_BUSY_CYCLE = 1024


def main():
    path, out = sys.argv[1], sys.argv[2]
    subs = sys.argv[3:] or ["gemm256_kernel", "gemm4w_kernel", "gemm_kernel", "attn_prefill_kernel"]
    val = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        d = r.get("Dispatch_Id") or r.get("Dispatch-Id") or r.get("Correlation_Id")
        c = r.get("Counter_Name") or r.get("Counter-Name")
        val[d][c] += float(r.get("Counter_Value") or r.get("Counter-Value") or 0)
        names[d] = name
    res = {}
    for sub in subs:
        by_inst = collections.defaultdict(lambda: [0, 0.0, 0.0])
        for d, cs in val.items():
            if sub not in names[d]:
                continue
            k = names[d].split("(")[0]
            by_inst[k][0] += 1
            by_inst[k][1] += cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            by_inst[k][2] += cs.get("GRBM_GUI_ACTIVE", 0.0)
        for k, (n, busy, gui) in by_inst.items():
            res[k] = {"dispatches": n, "mfma_busy_cycles": busy, "grbm_gui_active": gui,
                      "util": round(busy / (gui / 8 * SIMDS), 4) if gui else None,
                      "implied_flop_per_dispatch": busy * FLOP_PER_BUSY_CYCLE / n}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
