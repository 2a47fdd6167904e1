"""TEST INFRASTRUCTURE (CPU only) -- how far apart are the oracle's numerics modes after 28 layers?

Runs oracle/llama_ref.py on the full Llama-3.2-3B synthetic weights (oracle/synth.py) over one
configs[1] chunk (bench.py synthetic_chunks, doc 0) in the modes "bf16" (the engine's rounding
contract), "fp32" (un-rounded Llama) and "f16" (ggml's F16 graph, what Ollama runs for the
reference's llama3.2:3b-instruct-fp16, run_full_evaluation_pipeline.py:80-106), and prints the
per-layer relative hidden-state distance (Frobenius over every position) and the logit distance
at the fixtures' logit positions, for every pair of modes.

    python tools/parity_modes_cpu.py --seed 0 --jitter 0 --chunk 0 --modes bf16,fp32,f16
"""
import argparse
import importlib.util
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd")
for p in (ROOT, PKG):
    sys.path.insert(0, p)


def rel(a, b):
    return float(np.linalg.norm((a - b).astype(np.float64)) / np.linalg.norm(b.astype(np.float64)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--std", type=float, default=0.02)
    ap.add_argument("--jitter", type=float, default=0.0)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--prompt-len", type=int, default=2048)
    ap.add_argument("--modes", default="bf16,fp32,f16")
    ap.add_argument("--sharp", action="store_true", help="apply tests/golden/sharp_model.py")
    args = ap.parse_args()
    from mapsum.config import LLAMA32_3B as cfg
    from oracle.llama_ref import OracleLlama
    from oracle.synth import make_weights
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    prompt = bench.synthetic_chunks(args.chunk + 1, args.prompt_len, doc=0, vocab=cfg.vocab,
                                    bos=cfg.bos_id)[args.chunk]
    w = make_weights(cfg, args.seed, std=args.std, jitter=args.jitter)
    if args.sharp:
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        import sharp_model
        w = sharp_model.apply(w, sharp_model.copy_head_overrides(cfg, args.seed, args.jitter))
    P = len(prompt)
    lpos = np.array(sorted(set(list(range(15, P, 64)) + [P - 1])))
    res = {}
    for m in args.modes.split(","):
        t0 = time.time()
        lg, probes = OracleLlama(cfg, w, mode=m).forward(prompt, collect=True, all_logits=True)
        res[m] = (np.stack(probes), lg[lpos].copy())
        del lg, probes
        print(f"mode {m}: {time.time() - t0:.0f} s", flush=True)
    modes = list(res)
    pairs = [(a, b) for i, a in enumerate(modes) for b in modes[i + 1:]]
    print("layer " + " ".join(f"{a}-vs-{b:>5}" for a, b in pairs))
    for l in range(cfg.n_layers):
        print(f"{l:5d} " + " ".join(f"{rel(res[a][0][l], res[b][0][l]):12.3e}" for a, b in pairs))
    print("logits " + " ".join(f"{rel(res[a][1], res[b][1]):12.3e}" for a, b in pairs))
    for a, b in pairs:
        agree = np.mean(np.argmax(res[a][1], 1) == np.argmax(res[b][1], 1))
        print(f"argmax agreement {a} vs {b}: {agree:.4f} over {len(lpos)} positions")


if __name__ == "__main__":
    main()
