"""Timeline of decode attention v2 (k_attn.hip attn_decode2_kernel) from its in-kernel stamps.

Runs the configs[1] decode on a full-width 2-layer engine (8 slots, 2048-token prompts, eager
launches) with MS_A2_STAMPS=1, reads the latest launch's s_memrealtime stamps (100 MHz) of every
block (ms_debug_a2_stamps) and prints per phase the min / median / p90 / max time since the
earliest block entry, the block end times per XCD and the per-wave page landing spread.
Diagnostic only (the stamps cost time of their own).
  usage: python3 tools/a2_stamps.py [--gen 32]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))
os.environ["MS_A2_STAMPS"] = "1"
os.environ["MAPSUM_NO_GRAPHS"] = "1"

from mapsum import _lib as L  # noqa: E402
from mapsum.config import LLAMA32_3B  # noqa: E402
from mapsum.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gen", type=int, default=32)
ap.add_argument("--prompt", type=int, default=2048)
args = ap.parse_args()
import bench  # noqa: E402

NB, NS = 1024, 32
cfg = LLAMA32_3B.with_(n_layers=2)
chunks = bench.synthetic_chunks(8, args.prompt, doc=0, vocab=cfg.vocab, bos=cfg.bos_id)
with Engine(cfg, device=0, max_batch=8, max_ctx=args.prompt + 256, max_prefill_tokens=8 * args.prompt) as e:
    e.init_synthetic(0, 0.02, 0.0)
    e.generate(chunks, num_predict=args.gen, ignore_eos=True)
    buf = (C.c_uint64 * (NB * NS))()
    L.load().ms_debug_a2_stamps(C.cast(buf, C.c_void_p), NB * NS)
st = np.frombuffer(buf, dtype=np.uint64).reshape(NB, NS)
live = st[:, 0] > 0
st = st[live]
hw = st[:, 1]
xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xF
cu = ((hw >> np.uint64(8)) & np.uint64(0xF)).astype(np.int64)
se = ((hw >> np.uint64(13)) & np.uint64(0x7)).astype(np.int64)
ts = st.astype(np.int64)
t0 = ts[:, 0].min()


def row(name, v):
    v = v[v > 0]
    if len(v) == 0:
        return
    us = (v - t0) / 100.0
    print(f"{name:34s} {us.min():7.2f} {np.median(us):7.2f} {np.percentile(us, 90):7.2f} {us.max():7.2f}  {len(v)}")


print(f"decode attention v2, latest launch ({len(ts)} blocks), {args.prompt}-token prompts + {args.gen} steps; "
      f"us since the first block entry")
print(f"{'phase':34s} {'min':>7s} {'median':>7s} {'p90':>7s} {'max':>7s}  n")
row("block entry", ts[:, 0])
row("last wave entry", ts[:, 24])
row("wave 0 prologue loads issued", ts[:, 26])
row("last wave prologue loads issued", ts[:, 25])
row("wave 0 prologue loads landed", ts[:, 22])
row("last wave prologue loads landed", ts[:, 23])
row("prologue done (wave 0)", ts[:, 2])
sd = ts[:, 3:12]
pv = ts[:, 12:21]
row("wave S done (K landed), all waves", sd.ravel())
row("wave P.V done, all waves", pv.ravel())
row("first wave S done per block", np.where(sd > 0, sd, np.iinfo(np.int64).max).min(axis=1))
row("last wave S done per block", sd.max(axis=1))
row("partial stored (block end)", ts[:, 21])
print("\nblock end (us) by XCC: median / max, blocks")
end = (ts[:, 21] - t0) / 100.0
for x in sorted(set(xcc.tolist())):
    m = xcc == x
    print(f"  xcc {x}: {np.median(end[m]):6.2f} / {end[m].max():6.2f}  {m.sum()}")
lastS = (sd.max(axis=1) - t0) / 100.0
print(f"\nblock end - its last S done: median {np.median(end - lastS):.2f} us, max {np.max(end - lastS):.2f} us")
ent = (ts[:, 0] - t0) / 100.0
print(f"block entry spread: median {np.median(ent):.2f}, p90 {np.percentile(ent, 90):.2f}, max {ent.max():.2f} us")
pairs = {}
for x, s_, c in zip(xcc.tolist(), se.tolist(), cu.tolist()):
    pairs[(x, s_, c)] = pairs.get((x, s_, c), 0) + 1
print(f"distinct (xcc, se, cu) slots: {len(pairs)}; blocks per slot: max {max(pairs.values())}")
