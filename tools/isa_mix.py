"""Static instruction mix of one kernel of a HIP source (gfx950 cross-compile, no GPU): counts
per opcode in the kernel's disassembly, for hot-loop reasoning (VALU vs MFMA vs LDS).
  usage (from csrc/): python3 ../../tools/isa_mix.py k_attn.hip attn_prefill_kernelILi3 [top]"""
import collections
import glob
import os
import subprocess
import sys
import tempfile

src, pat = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
here = os.getcwd()
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", f"-I{here}",
                    f"-I{here}/../../include", "--save-temps", "-c", os.path.join(here, src), "-o",
                    os.path.join(d, "x.o")], cwd=d, check=True, capture_output=True)
    s = open(glob.glob(os.path.join(d, "*gfx950.s"))[0]).read()
names = [l.split(":")[0] for l in s.split("\n") if pat in l and not l.startswith((".", "\t", " ")) and ":" in l]
name = names[0]
a = s.index(name + ":")
b = s.index(".Lfunc_end", a)
c = collections.Counter()
for line in s[a:b].split("\n"):
    t = line.strip()
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    c[t.split()[0]] += 1
print(name, "total", sum(c.values()))
groups = collections.Counter()
for k, v in c.items():
    g = ("mfma" if "mfma" in k else "lds" if k.startswith("ds_") else "vmem" if k.startswith(("global_", "buffer_")) else
         "salu/smem" if k.startswith("s_") else "valu" if k.startswith("v_") else "other")
    groups[g] += v
print(dict(groups))
for k, v in c.most_common(top):
    print(f"{v:6d} {k}")
