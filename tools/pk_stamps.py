"""In-kernel timeline of the persistent decode step (k_persist.hip, MS_PK_STAMPS=1).

Runs the configs[1] batch (8 x 2048-token chunks, 8 slots) for a few decode steps with the
stamps on, reads the LAST launch's per-CU stamps (ms_debug_pk_stamps) and prints, per layer
(median over layers 1..L-2) and per phase stamp, the min / median / max over the 256 CUs of
the time since the layer's earliest loader start (us).
  usage: python3 tools/pk_stamps.py [--layers 28] [--gen 8]"""
import argparse
import ctypes as C
import os
import sys

os.environ["MS_PK_STAMPS"] = "1"
os.environ.setdefault("MS_PERSIST", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))
import numpy as np  # noqa: E402

from bench import synthetic_chunks  # noqa: E402
from mapsum import _lib as L  # noqa: E402
from mapsum.config import LLAMA32_3B  # noqa: E402
from mapsum.engine import Engine  # noqa: E402

NAMES = {0: "ldr layer start", 1: "ldr READY dn(l-1) -> QKV X", 2: "ldr READY qkv(g) -> gather",
         3: "ldr READY att -> O X", 4: "ldr READY o -> GU X", 5: "ldr READY gu -> h", 6: "ldr last slot issued",
         7: "cw0 QKV units done", 15: "cw1/2 QKV units done", 8: "cw0 prologue done", 9: "cw0 merge done",
         10: "O epilogue published", 11: "GU tile 0 published", 12: "GU tile 1 published",
         13: "down published"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=28)
    ap.add_argument("--gen", type=int, default=8)
    a = ap.parse_args()
    cfg = LLAMA32_3B.with_(n_layers=a.layers)
    chunks = synthetic_chunks(8, 2048, doc=0, vocab=cfg.vocab, bos=cfg.bos_id)
    with Engine(cfg, device=0, max_batch=8, max_ctx=2048 + 64, max_prefill_tokens=8 * 2048) as e:
        e.init_synthetic(0, 0.02, 0.0)
        e.generate(chunks, num_predict=a.gen, ignore_eos=True)
        n = 256 * 28 * 16
        buf = (C.c_uint64 * (n + 160 * 4))()
        L.load().ms_debug_pk_stamps(C.cast(buf, C.c_void_p), n + 160 * 4)
    allv = np.frombuffer(buf, np.uint64)
    s = allv[:n].reshape(256, 28, 16).astype(np.float64)[:, :a.layers]
    tr = allv[n:].reshape(160, 4).astype(np.float64)
    t0 = s[:, :, 0].min(axis=0)  # per layer: the earliest loader start
    rel = (s - t0[None, :, None]) * 0.01  # 100 MHz ticks -> us
    span = np.diff(t0) * 0.01
    print(f"layer period (us): median {np.median(span):.2f}  min {span.min():.2f}  max {span.max():.2f}")
    mid = slice(1, max(2, a.layers - 1))
    for k in sorted(NAMES):
        v = rel[:, mid, k]
        ok = s[:, mid, k] > 0
        if not ok.any():
            continue
        v = np.where(ok, v, np.nan)
        print(f"{k:2d} {NAMES[k]:32s} min {np.nanmedian(np.nanmin(v, axis=0)):8.2f}  "
              f"med {np.nanmedian(np.nanmedian(v, axis=0)):8.2f}  max {np.nanmedian(np.nanmax(v, axis=0)):8.2f}")
    if a.layers > 5:
        trace(tr, s[0, 5, 0])
        # the slowest attention items of layer 5: (cu, split, seq, kv head) and their stamps
        r5 = rel[:, 5]
        order = np.argsort(-r5[:, 9])
        print("slowest merges, layer 5: cu s b g | gather prologue merge  (us)")
        for cu in order[:12]:
            print(f"  {cu:3d} {cu // 64} {(cu % 64) // 8} {cu % 8} | {r5[cu, 2]:7.2f} {r5[cu, 8]:7.2f} {r5[cu, 9]:7.2f}")
        print("fastest merges:")
        for cu in order[-6:]:
            print(f"  {cu:3d} {cu // 64} {(cu % 64) // 8} {cu % 8} | {r5[cu, 2]:7.2f} {r5[cu, 8]:7.2f} {r5[cu, 9]:7.2f}")
        for sp in range(4):
            sel = [cu for cu in range(256) if cu // 64 == sp]
            print(f"split {sp}: merge median {np.median(r5[sel, 9]):.2f} max {np.max(r5[sel, 9]):.2f}")


def trace(tr, t0):
    """CU 0, layer 5: per ring slot issue / FULL published / consumer saw FULL / released (us)."""
    print("slot  issue   full    saw     rel    (CU 0, layer 5; us since the layer's loader start)")
    for i in range(tr.shape[0]):
        if tr[i, 0] == 0:
            continue
        v = (tr[i] - t0) * 0.01
        print(f"{i:4d} " + " ".join(f"{x:7.2f}" for x in v))


if __name__ == "__main__":
    main()
