"""TEST INFRASTRUCTURE ONLY -- 28-layer golden fixtures of the benchmarked model.

Runs the CPU oracle (oracle/llama_ref.py) on the engine's bit-exact synthetic Llama-3.2-3B
weights (oracle/synth.py; all 28 layers, full widths) over BASELINE.json configs[1] chunks
(bench.py synthetic_chunks, doc 0) and writes what the GPU test
(tests/test_gpu_golden28.py) compares the engine with -- so no oracle runs on the GPU box.
The call being replaced: run_full_evaluation_pipeline.py:80-106 (one /api/generate per chunk).

Two models (tests/golden/sharp_model.py explains the second):
  flat  -- the bench's exact weights (bench.py: seed 0, std 0.02, norm jitter 0), chunks 0 and 5;
  sharp -- seed 77 (norm jitter 0.1) with a RoPE copy head at a late layer and a large shared
           embedding direction, chunks 0 and 3: greedy choices are decisive, so the literal
           free-running bar applies, and the head reads a residual that all the random layers
           before it have written;
  q4km  -- configs[4]: bench.py's Q4_K_M weights (ms_init_synthetic_q, seed 2; the block
           generator restated in oracle/synth.py) at their EXACT fp32 dequantisation, chunks
           0 and 5 (mode fp32 only).

Three numerics modes of the oracle (oracle/llama_ref.py OracleLlama mode):
  fp32   -- un-rounded Llama (pinned against transformers on TINY): the parity target;
  f16    -- ggml's F16 graph, what Ollama runs for the reference's llama3.2:3b-instruct-fp16;
  engine -- the engine's own fp16 rounding points (a kernel-regression mirror).

Per chunk (key prefix c<k>_):
  prompt      int32 [P]
  hpos        int32 [3]           positions whose full hidden rows are kept
  hid_rows    f32  [L][3][H]      residual after each layer at hpos
  hid_norm    f32  [L][P]         L2 norm of every position's residual, per layer
  hid_sketch  f16  [L][P/4][8]    residual[::4] @ R, R = rng(SKETCH_SEED) N(0,1) [H][8]
  lpos        int32 [nl]          prefill positions whose logits are kept
  lg_top_ids  int32 [nl][16], lg_top_vals f32 [nl][16], lg_rms f32 [nl]
  lg_sketch   f32  [nl][8]        logits @ Rv, Rv = rng(SKETCH_SEED + 1) N(0,1) [V][8]
  gen_ids     int32 [G]           free-running greedy continuation (ignore_eos)
  gen_top_ids int32 [G][16], gen_top_vals f32 [G][16]: the oracle's top-16 at each step
                                  (step j's context = prompt + gen_ids[:j])

    python tests/golden/make_fullshape_golden.py --which flat --mode fp32   (-> fullshape_flat_fp32.npz)
    python tests/golden/make_fullshape_golden.py --which sharp --mode engine
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd")
for p in (ROOT, PKG, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

MODEL = {"flat": (0, 0.02, 0.0), "sharp": (77, 0.02, 0.1), "q4km": (2, 0.02, 0.0),
         "sharpq4km": (2, 0.02, 0.0)}  # seed, std, norm jitter
P, GEN, TOPK = 2048, 128, 16
SKETCH_SEED = 1234
CHUNKS = {"flat": (0, 5), "sharp": (0, 3), "q4km": (0, 5), "sharpq4km": (0, 3)}


def sketch_mats(H, V):
    R = np.random.default_rng(SKETCH_SEED).standard_normal((H, 8), dtype=np.float32)
    Rv = np.random.default_rng(SKETCH_SEED + 1).standard_normal((V, 8), dtype=np.float32)
    return R, Rv


def hpos_of(p):
    return np.array([0, p // 2, p - 1], np.int32)


def lpos_of(p):
    return np.array(sorted(set(list(range(15, p, 64)) + [p - 1])), np.int32)


def chunks_of(cfg, idx):
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    allc = bench.synthetic_chunks(max(idx) + 1, P, doc=0, vocab=cfg.vocab, bos=cfg.bos_id)
    return [allc[i] for i in idx]


def topk(v, k=TOPK):
    i = np.argpartition(-v, k)[:k]
    i = i[np.lexsort((i, -v[i]))]  # value desc, id asc (argmax tie rule)
    return i.astype(np.int32), v[i].astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", choices=("flat", "sharp", "q4km", "sharpq4km"), required=True)
    ap.add_argument("--mode", choices=("fp32", "f16", "engine"), required=True)
    ap.add_argument("--gen", type=int, default=GEN)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from mapsum.config import LLAMA32_3B
    from oracle.llama_ref import OracleLlama
    from oracle.synth import make_weights

    cfg = LLAMA32_3B
    t0 = time.time()
    SEED, STD, JIT = MODEL[args.which]
    if args.which == "q4km":
        # configs[4]: bench.py's Q4_K_M model (ms_init_synthetic_q seed 2) at its EXACT fp32
        # dequantisation (oracle/synth.py restates the device block generator bit for bit)
        from oracle.synth import make_q4km_blocks, q4km_weights
        w = q4km_weights(cfg, make_q4km_blocks(cfg, SEED, STD), SEED, JIT)
    elif args.which == "sharpq4km":
        # the copy head on the Q4_K_M model: quantised overrides (tests/golden/sharp_model.py
        # q4km_overrides), every block at its exact fp32 dequantisation
        import sharp_model
        _, w = sharp_model.q4km_model(cfg)
    else:
        w = make_weights(cfg, SEED, std=STD, jitter=JIT)
    meta = {"model": cfg.name, "n_layers": cfg.n_layers, "seed": SEED, "std": STD, "jitter": JIT,
            "mode": args.mode,
            "prompt_len": P, "gen": args.gen, "which": args.which, "chunks_doc": 0,
            "chunks": list(CHUNKS[args.which]), "sketch_seed": SKETCH_SEED,
            "generator": "tests/golden/make_fullshape_golden.py (oracle/llama_ref.py, numpy "
                         + np.__version__ + ")"}
    if args.which == "sharpq4km":
        import sharp_model
        meta.update(copy_offset=sharp_model.COPY_OFFSET, design_seed=sharp_model.DESIGN_SEED,
                    copy_layer=sharp_model.COPY_LAYER, c_layer=sharp_model.C_LAYER_Q4KM)
    if args.which == "sharp":
        import sharp_model
        w = sharp_model.apply(w, sharp_model.copy_head_overrides(cfg, SEED, JIT))
        meta.update(copy_offset=sharp_model.COPY_OFFSET, design_seed=sharp_model.DESIGN_SEED,
                    copy_layer=sharp_model.COPY_LAYER)
    print(f"weights {time.time() - t0:.0f} s", flush=True)
    o = OracleLlama(cfg, w, mode=args.mode)
    R, Rv = sketch_mats(cfg.hidden, cfg.vocab)
    out = {"meta": np.frombuffer(json.dumps(meta).encode(), np.uint8)}
    for ci, prompt in zip(CHUNKS[args.which], chunks_of(cfg, CHUNKS[args.which])):
        t1 = time.time()
        cache = o.new_cache()
        lg, probes = o.forward(prompt, cache, collect=True, all_logits=True)
        hp, lp = hpos_of(P), lpos_of(P)
        k = f"c{ci}_"
        out[k + "prompt"] = np.asarray(prompt, np.int32)
        out[k + "hpos"] = hp
        out[k + "hid_rows"] = np.stack([h[hp] for h in probes]).astype(np.float32)
        out[k + "hid_norm"] = np.stack([np.linalg.norm(h, axis=1) for h in probes]).astype(np.float32)
        out[k + "hid_sketch"] = np.stack([h[::4] @ R for h in probes]).astype(np.float16)
        del probes
        out[k + "lpos"] = lp
        tops = [topk(lg[p]) for p in lp]
        out[k + "lg_top_ids"] = np.stack([t[0] for t in tops])
        out[k + "lg_top_vals"] = np.stack([t[1] for t in tops])
        out[k + "lg_rms"] = np.sqrt(np.mean(lg[lp].astype(np.float64) ** 2, 1)).astype(np.float32)
        out[k + "lg_sketch"] = (lg[lp] @ Rv).astype(np.float32)
        last = lg[-1].copy()
        del lg
        print(f"chunk {ci}: prefill {time.time() - t1:.0f} s", flush=True)
        gen, gti, gtv = [], [], []
        cur = last
        for j in range(args.gen):
            ti, tv = topk(cur)
            gti.append(ti)
            gtv.append(tv)
            t = int(np.argmax(cur))
            gen.append(t)
            if j + 1 < args.gen:
                cur, _ = o.forward([t], cache)
        out[k + "gen_ids"] = np.asarray(gen, np.int32)
        out[k + "gen_top_ids"] = np.stack(gti)
        out[k + "gen_top_vals"] = np.stack(gtv)
        gaps = np.stack(gtv)[:, 0] - np.stack(gtv)[:, 1]
        print(f"chunk {ci}: decode {time.time() - t1:.0f} s; top-2 gap min {gaps.min():.4f} "
              f"median {np.median(gaps):.4f}", flush=True)
    path = args.out or os.path.join(HERE, f"fullshape_{args.which}_{args.mode}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.1f} MB) in {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
