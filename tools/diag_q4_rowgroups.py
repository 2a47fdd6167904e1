"""Diagnostic (GPU): K-quant engine batch invariance across row-group counts.

A 128-slot Q4_K_M engine runs chunk 0 of bench.py's workload alone and among n - 1 other
chunks; the chunk's greedy ids must not depend on n (the K-quant GEMVs run in row groups of
<= 64 rows whose arithmetic is per row).  Prints the first differing step per n.

    python tools/diag_q4_rowgroups.py --layers 2 --gen 32 --counts 1,8,64,65,72,128
"""
import argparse
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--gen", type=int, default=32)
    ap.add_argument("--slots", type=int, default=128)
    ap.add_argument("--counts", default="1,8,64,65,72,128")
    ap.add_argument("--fp16", action="store_true")
    ap.add_argument("--prompt", type=int, default=2048)
    args = ap.parse_args()
    from mapsum.config import LLAMA32_3B
    from mapsum.engine import Engine
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cfg = LLAMA32_3B.with_(n_layers=args.layers)
    counts = [int(c) for c in args.counts.split(",")]
    chunks = [c[:args.prompt] for d in range((max(counts) + 7) // 8)
              for c in bench.synthetic_chunks(8, 2048, doc=d, vocab=cfg.vocab, bos=cfg.bos_id)]
    e = Engine(cfg, device=0, max_batch=args.slots, max_ctx=args.prompt + args.gen + 64,
               max_prefill_tokens=8 * args.prompt)
    try:
        if args.fp16:
            e.init_synthetic(0, 0.02, 0.0)
        else:
            e.init_synthetic_q(seed=2, scale=0.02, norm_jitter=0.0)
        ref = None
        for n in counts:
            res = e.generate(chunks[:n], num_predict=args.gen, ignore_eos=True)
            ids = np.asarray(res[0].ids)
            if ref is None:
                ref = ids
            diff = np.nonzero(ids != ref)[0]
            print(f"n={n:4d}: chunk 0 first difference vs n={counts[0]}: "
                  f"{int(diff[0]) if diff.size else 'none'} ({diff.size} of {len(ids)} differ)", flush=True)
            if n > 1:
                alone = np.asarray(e.generate([chunks[n - 1]], num_predict=args.gen, ignore_eos=True)[0].ids)
                last = np.asarray(res[n - 1].ids)
                dl = np.nonzero(alone != last)[0]
                print(f"        chunk {n - 1} (last row) alone vs in batch: "
                      f"{int(dl[0]) if dl.size else 'none'} ({dl.size} differ)", flush=True)
    finally:
        e.close()


if __name__ == "__main__":
    main()
