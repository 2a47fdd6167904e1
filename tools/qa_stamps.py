"""Timeline of the fused QKV + attention launch (k_qkvattn.hip) from its in-kernel stamps.

Runs the configs[1] decode on a full-width 2-layer engine (8 slots, 2048-token prompts) with
MS_QA_STAMPS=1, reads the latest launch's s_memrealtime stamps (100 MHz) of every workgroup
(ms_debug_qa_stamps) and prints, per phase boundary, the median / 90th percentile / max time
since the earliest workgroup start.  Diagnostic only (the stamps cost time of their own).
  usage: python3 tools/qa_stamps.py [--gen 32]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))
os.environ["MS_QA_STAMPS"] = "1"

from mapsum import _lib as L  # noqa: E402
from mapsum.config import LLAMA32_3B  # noqa: E402
from mapsum.engine import Engine  # noqa: E402

NAMES = {0: "pub wave entry", 8: "page wave 0 entry", 1: "pub wave: weights multiplied",
         9: "page wave 0: weights multiplied", 2: "pub wave: exchange done", 3: "published (drained + arrived)",
         4: "poll satisfied", 5: "prologue done (q/k/v in LDS)", 10: "page wave 0: K landed, S done",
         11: "page wave 0: P.V done", 12: "merge done (end)"}

ap = argparse.ArgumentParser()
ap.add_argument("--gen", type=int, default=32)
ap.add_argument("--prompt", type=int, default=2048)
args = ap.parse_args()
import bench  # noqa: E402

cfg = LLAMA32_3B.with_(n_layers=2)
chunks = bench.synthetic_chunks(8, args.prompt, doc=0, vocab=cfg.vocab, bos=cfg.bos_id)
with Engine(cfg, device=0, max_batch=8, max_ctx=args.prompt + 256, max_prefill_tokens=8 * args.prompt) as e:
    e.init_synthetic(0, 0.02, 0.0)
    e.generate(chunks, num_predict=args.gen, ignore_eos=True)
    buf = (C.c_uint64 * (256 * 16))()
    L.load().ms_debug_qa_stamps(C.cast(buf, C.c_void_p), 256 * 16)
st = np.frombuffer(buf, dtype=np.uint64).reshape(256, 16).astype(np.int64)
t0 = st[:, 0][st[:, 0] > 0].min()
print(f"fused QKV + attention, latest launch, {args.prompt}-token prompts + {args.gen} steps; us since the first workgroup start")
print(f"{'phase':36s} {'min':>7s} {'median':>7s} {'p90':>7s} {'max':>7s}  n")
for k in (0, 8, 1, 9, 2, 3, 4, 5, 10, 11, 12):
    v = st[:, k]
    v = v[v > 0]
    if len(v) == 0:
        continue
    us = (v - t0) / 100.0
    print(f"{NAMES[k]:36s} {us.min():7.2f} {np.median(us):7.2f} {np.percentile(us, 90):7.2f} {us.max():7.2f}  {len(v)}")
