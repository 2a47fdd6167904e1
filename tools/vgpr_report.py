"""Per-kernel VGPR / AGPR / occupancy table of one HIP source, from hipcc's resource-usage
remarks (cross-compiled for gfx950, no GPU needed).
  usage: python3 tools/vgpr_report.py k_gemv.hip [name-substring]   (run from csrc/)"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-I.",
                    "-I../../include", "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"],
                   capture_output=True, text=True)
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for name, d in rows.items():
    if pat in name:
        print(f"{d.get('VGPRs', '?'):>4} {d.get('AGPRs', '?'):>4} occ={d.get('Occupancy [waves/SIMD]', '?'):>2} "
              f"lds={d.get('LDS Size [bytes/block]', '?'):>6} scratch={d.get('ScratchSize [bytes/lane]', '?'):>3}  {name}")
