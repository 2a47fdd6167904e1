"""BASELINE configs[3] on one GPU: hierarchical map level with ragged section-sized chunks.

Section token lengths are log-normal (median 600, sigma 1.0, clipped to [64, 4096],
seed 1). One level is submitted as one batch (level-synchronous,
mapsum/hierarchical.py), and the engine packs the ragged prompts into varlen prefill
passes and continuous-batching decode. Prints one JSON line: sections/s and generated
tokens/s over the whole level.

usage: python tools/bench_ragged.py [--sections 64] [--max-batch 64] [--gen-len 256]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd")]


def section_lengths(n, seed=1):
    rng = np.random.default_rng(seed)
    return np.clip(np.round(np.exp(np.log(600) + rng.standard_normal(n))), 64, 4096).astype(int)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sections", type=int, default=64)
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--gen-len", type=int, default=256)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()

    from mapsum.config import LLAMA32_3B as cfg
    from mapsum.engine import Engine

    lens = section_lengths(args.sections)
    rng = np.random.default_rng(0)
    prompts = [np.concatenate([[cfg.bos_id], rng.integers(0, 128000, size=n - 1)]).astype(np.int32) for n in lens]
    with Engine(cfg, device=0, max_batch=args.max_batch, max_ctx=int(lens.max()) + args.gen_len,
                max_prefill_tokens=16384) as eng:
        eng.init_synthetic(seed=0, std=0.02, norm_jitter=0.0)
        eng.generate(prompts[:4], num_predict=8, ignore_eos=True)  # warm-up (graphs, caches)
        times, outs = [], []
        for _ in range(args.reps):
            eng.synchronize()
            t0 = time.perf_counter()
            res = eng.generate(prompts, num_predict=args.gen_len, ignore_eos=True)
            eng.synchronize()
            times.append(time.perf_counter() - t0)
            outs.append([r.ids for r in res])
        st = eng.stats()
        # self-checks outside the timed region (as bench.py): same summaries every repetition,
        # full length, and a section's summary independent of its companions (the shortest,
        # the median and the longest section rerun alone)
        order = np.argsort(lens)
        picks = [int(order[0]), int(order[len(order) // 2]), int(order[-1])]
        alone = {i: eng.generate([prompts[i]], num_predict=args.gen_len, ignore_eos=True)[0].ids for i in picks}
        check = {"deterministic_across_reps": all(o == outs[0] for o in outs[1:]),
                 "full_length": all(len(x) == args.gen_len for x in outs[0]),
                 "batch_invariant": all(alone[i] == outs[0][i] for i in picks)}
        assert all(check.values()), check
    dt = min(times)
    print(json.dumps({
        "metric": "hierarchical level: ragged sections/s (configs[3])", "value": round(args.sections / dt, 3),
        "unit": "sections/s", "gen_tokens_per_s": round(args.sections * args.gen_len / dt, 1),
        "prompt_tokens_per_s": round(int(lens.sum()) / dt, 1), "seconds": round(dt, 3),
        "config": {"sections": args.sections, "max_batch": args.max_batch, "gen_len": args.gen_len,
                   "prompt_tokens": {"min": int(lens.min()), "median": int(np.median(lens)),
                                     "max": int(lens.max()), "sum": int(lens.sum())},
                   "weights": "f16 synthetic", "n_gpus": 1},
        "graphs_built": st["graphs_built"], "check": check}), flush=True)


if __name__ == "__main__":
    main()
