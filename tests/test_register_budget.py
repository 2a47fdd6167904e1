"""Register-budget guard for the decode GEMVs whose speed depends on occupancy (CPU: reads the
built library's code-object metadata).

The gate/up GEMV of the fp16 decode step (k_gemv.hip gemv_kernel<1, 2, SWIGLU, 3, kXLds, RS>)
runs 1024-thread blocks and streams its weights with two blocks co-resident per CU, which
needs <= 64 VGPRs per lane (2 x 16 waves over 4 SIMDs x 512 VGPRs).  One extra live register
-- a row statistic held across the weight stream -- took it to 67 and cost 1.6 us per launch
(20.8 -> 22.4 us, profiles/r03/v9_rs_hold_ab.txt), a regression no numerics test sees.
"""
import os
import re
import subprocess

import pytest

from test_isa_order import LIB, LLVM, _code_objects

# (mangled-name prefix, max VGPRs): the instantiations the bench's decode step launches
BUDGET = [
    ("_ZN2ms11gemv_kernelILi1ELi2ELi2ELi3ELi1ELb1E", 64),  # gate/up + SwiGLU, deferred norm
    ("_ZN2ms11gemv_kernelILi1ELi2ELi2ELi3ELi1ELb0E", 64),  # gate/up + SwiGLU, plain
]


def _kernel_meta(tmp_path):
    meta = {}
    for i, co in enumerate(_code_objects(LIB)):
        p = tmp_path / f"co{i}.elf"
        p.write_bytes(co)
        txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(p)],
                             check=True, capture_output=True, text=True).stdout
        name = None
        for line in txt.splitlines():
            m = re.match(r"\s+\.(name|vgpr_count|max_flat_workgroup_size):\s+(\S+)", line)
            if not m:
                continue
            k, v = m.groups()
            if k == "name":
                name = v
                meta[name] = {}
            elif name:
                meta[name][k] = int(v)
    return meta


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmapsum.so not built")
def test_gate_up_gemv_keeps_two_blocks_per_cu(tmp_path):
    meta = _kernel_meta(tmp_path)
    for prefix, limit in BUDGET:
        hits = [(n, d) for n, d in meta.items() if n.startswith(prefix)]
        assert hits, f"{prefix} not found in the library"
        for n, d in hits:
            assert d["max_flat_workgroup_size"] == 1024, n
            assert d["vgpr_count"] <= limit, f"{n}: {d['vgpr_count']} VGPRs > {limit}"
