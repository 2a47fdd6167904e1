"""Measurement tooling on synthetic rocprofv3 outputs: the PMC traffic reduction
(tools/traffic_from_pmc.py) applies the gfx950 FETCH_SIZE x2 correction per dispatch."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _csv(path, counter, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, name, v in rows:
            w.writerow({"Dispatch_Id": d, "Kernel_Name": name, "Counter_Name": counter, "Counter_Value": v})


def test_traffic_from_pmc(tmp_path):
    g1, g2, other = "void ms::gemv_kernel<1, 1, 3, 1, true>(x)", "void ms::gemv_kernel<1, 2, 2, 3, true>(x)", "ms::argmax_kernel(x)"
    # FETCH_SIZE in KB, possibly split over several rows of one dispatch (per-XCD instances)
    _csv(tmp_path / "f.csv", "FETCH_SIZE", [(1, g1, 500), (1, g1, 500), (2, g2, 3000), (3, other, 99999)])
    _csv(tmp_path / "w.csv", "WRITE_SIZE", [(1, g1, 10), (2, g2, 30), (3, other, 5)])
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic_from_pmc.py"), str(tmp_path / "f.csv"),
                    str(tmp_path / "w.csv"), "gemv_kernel", str(out)], check=True, capture_output=True)
    r = json.load(open(out))
    assert r["dispatches_fetch"] == 2 and r["dispatches_write"] == 2
    fetch = (1000 + 3000) / 2 * 1024
    assert r["fetch_bytes_corrected_x2"] == round(2 * fetch)
    assert r["traffic_bytes_per_launch"] == round(2 * fetch + (10 + 30) / 2 * 1024)
    assert r["fetch_x2_by_instantiation"]["void ms::gemv_kernel<1, 1, 3, 1, true>"] == 2 * 1000 * 1024
