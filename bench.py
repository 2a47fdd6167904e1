"""bench.py -- map-phase chunks/s of the MI355X engine (BASELINE.json metric).

A "step" = one map phase over one batch: every GPU takes its chunks_per_gpu synthetic
2048-token chunks (the workload of BASELINE.json configs[1]: one 16k-token doc split
into 8 chunks), prefills them packed, decodes exactly 256 greedy tokens each
(ignore_eos), and the per-chunk summary ids are gathered to rank 0
over RCCL.  value = chunks of all ranks / max-over-ranks wall time.  N > 1 is weak
scaling: each rank owns its own document's chunks.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

METRIC = "map-phase chunks/sec (2k-tok chunk, 256-tok summary) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA


def synthetic_chunks(n, prompt_len, doc, vocab, bos, seed=0):
    """Token ids of n chunks: BOS + Llama-3 header ids + uniform body over [0, 128000)
    (no tokenizer / dataset offline; timing of dense ops does not depend on values)."""
    head = [bos, 128006, 9125, 128007, 271, 128009, 128006, 882, 128007, 271]
    rng = np.random.default_rng(seed + 1000 * doc)
    tail = [128009, 128006, 78191, 128007, 271]
    out = []
    for _ in range(n):
        body = rng.integers(0, min(128000, vocab), size=prompt_len - len(head) - len(tail))
        ids = np.array(head + body.tolist() + tail, np.int32)
        out.append(np.clip(ids, 0, vocab - 1))
    return out


def gemv_bytes_per_step(cfg, B):
    """Algorithmic HBM bytes of one decode step's layer projections: every weight matrix
    once + the B activation rows in/out (SURVEY.md §8d weight term, without lm_head)."""
    H, D, F = cfg.hidden, cfg.head_dim, cfg.ffn
    qkv = (cfg.n_heads + 2 * cfg.n_kv_heads) * D
    w = 2 * (qkv * H + H * cfg.n_heads * D + 2 * F * H + H * F)
    act = 2 * B * (H + qkv + cfg.n_heads * D + H + H + F + F + H) + 4 * B * H * 4
    return cfg.n_layers * (w + act)


def _q4_k_m_bytes_per_weight(tensor, layer, n_layers):
    """Device bytes per weight of one decode-GEMV operand under the Q4_K_M mix
    (csrc/engine.cpp q4_k_m_type): Q4_K 144 B / 256, Q6_K repacked 224 B / 256."""
    if tensor in ("wv", "w_down"):
        more = layer < n_layers // 8 or layer >= 7 * n_layers // 8 or (layer - n_layers // 8) % 3 == 2
        return 224 / 256 if more else 144 / 256
    return 144 / 256


def qgemv_bytes_per_step(cfg, B):
    """gemv_bytes_per_step with K-quant weight bytes (BASELINE configs[4])."""
    H, D, F = cfg.hidden, cfg.head_dim, cfg.ffn
    qkv = (cfg.n_heads + 2 * cfg.n_kv_heads) * D
    act = 2 * B * (H + qkv + cfg.n_heads * D + H + H + F + F + H) + 4 * B * H * 4
    tot = 0.0
    for l in range(cfg.n_layers):
        bpw = lambda t: _q4_k_m_bytes_per_weight(t, l, cfg.n_layers)  # noqa: E731
        tot += (bpw("wq") * (qkv - 2 * cfg.n_kv_heads * D) * H + bpw("wk") * cfg.n_kv_heads * D * H
                + bpw("wv") * cfg.n_kv_heads * D * H + bpw("wo") * H * cfg.n_heads * D
                + bpw("w_gate") * 2 * F * H + bpw("w_down") * H * F + act)
    return tot


def lm_head_bytes_per_step(cfg, B, quant=False):
    """The decode lm_head launch: the (tied) vocab matrix once -- Q6_K repacked to 224 B per
    256 weights under Q4_K_M (csrc/engine.cpp q4_k_m_type) -- plus B rows in, fp32 logits out."""
    w = cfg.vocab * cfg.hidden * (224 / 256 if quant else 2)
    return w + 2 * B * cfg.hidden + 4 * B * cfg.vocab


def prefill_flops_per_chunk(cfg, P):
    """2*params_linear*P + lm_head on the last token + causal attention."""
    H, D, F = cfg.hidden, cfg.head_dim, cfg.ffn
    lin = cfg.n_layers * ((cfg.n_heads + 2 * cfg.n_kv_heads) * D * H + H * cfg.n_heads * D + 3 * H * F)
    attn = cfg.n_layers * cfg.n_heads * 4 * D * (P * (P + 1) // 2)
    return 2 * lin * P + 2 * cfg.vocab * H + attn


def cpu_baseline(cfg, prompt_len, gen_len, decode_sample=16):
    """Oracle (numpy, CPU) on a bounded sample of the same workload, scaled to one chunk:
    one full-width layer prefilled over a prompt_len chunk + decode_sample cached decode
    steps through that layer + the tied lm_head, times n_layers / gen_len."""
    from oracle.llama_ref import OracleLlama
    one = cfg.with_(n_layers=1)
    rng = np.random.default_rng(0)
    H, D = cfg.hidden, cfg.head_dim

    def lin(r, c):
        return (rng.standard_normal((r, c), dtype=np.float32) * 0.02)

    w = {"embed": lin(cfg.vocab, H), "final_norm": np.ones(H, np.float32),
         "layers": [{"attn_norm": np.ones(H, np.float32), "ffn_norm": np.ones(H, np.float32),
                     "wq": lin(cfg.n_heads * D, H), "wk": lin(cfg.n_kv_heads * D, H),
                     "wv": lin(cfg.n_kv_heads * D, H), "wo": lin(H, cfg.n_heads * D),
                     "w_gate": lin(cfg.ffn, H), "w_up": lin(cfg.ffn, H), "w_down": lin(H, cfg.ffn)}]}
    w["lm_head"] = w["embed"]
    o = OracleLlama(one, w)
    ids = rng.integers(0, 128000, size=prompt_len)
    cache = o.new_cache()
    t0 = time.perf_counter()
    logits, _ = o.forward(ids, cache)
    t_pre = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(decode_sample):
        logits, _ = o.forward([int(np.argmax(logits))], cache)
    t_dec = (time.perf_counter() - t0) / decode_sample
    # lm_head is paid once per token, the layer n_layers times
    t0 = time.perf_counter()
    for _ in range(4):
        _ = w["embed"] @ np.ones(H, np.float32)
    t_head = (time.perf_counter() - t0) / 4
    t_layer_dec = max(t_dec - t_head, 1e-9)
    t_layer_pre = max(t_pre - t_head, 1e-9)
    chunk_s = cfg.n_layers * t_layer_pre + t_head + (gen_len - 1) * (cfg.n_layers * t_layer_dec + t_head)
    try:
        import threadpoolctl
        cores = max(p["num_threads"] for p in threadpoolctl.threadpool_info()) if threadpoolctl.threadpool_info() else 1
    except Exception:
        cores = os.cpu_count() or 1
    return {"value": 1.0 / chunk_s, "unit": "chunks/s", "cores": int(cores), "kind": "port",
            "sample": (f"numpy oracle, Llama-3.2-3B width, 1 of {cfg.n_layers} layers: {prompt_len}-tok "
                       f"prefill ({t_pre:.2f}s) + {decode_sample} cached decode steps "
                       f"({t_dec * 1e3:.1f} ms/step incl. lm_head {t_head * 1e3:.1f} ms), "
                       f"scaled to {cfg.n_layers} layers x {gen_len} tokens")}


def pmc_traffic(weights):
    """HBM bytes per GEMV launch from the committed rocprofv3 --pmc passes of this same
    workload (FETCH_SIZE x2 + WRITE_SIZE, tools/traffic_from_pmc.py, run by
    tools/gpu_round.sh); None when no such measurement is committed.  PMC counters cannot
    be read from inside a timed run, so this is the profiler's number, not a live one."""
    import glob
    hits = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                         "profiles", "r*", f"pmc_traffic_{weights}.json")))
    if not hits:
        return None, None
    return json.load(open(hits[-1]))["traffic_bytes_per_launch"], os.path.relpath(hits[-1], os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--chunks-per-gpu", type=int, default=8)
    ap.add_argument("--prompt-len", type=int, default=2048)
    ap.add_argument("--gen-len", type=int, default=256)
    ap.add_argument("--model", default="llama3.2-3b")
    ap.add_argument("--weights", choices=("bf16", "q4_k_m"), default="bf16",
                    help="q4_k_m = BASELINE configs[4]: random Q4_K/Q6_K blocks, K-quant decode GEMVs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true", help="skip HIP-event timing of the GEMV class")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from mapsum import _lib as L
    from mapsum.config import CONFIGS
    from mapsum.dist import Unit, env_rank, gather_summaries, pack_results
    from mapsum.engine import Engine

    cfg = CONFIGS[args.model]
    rank, local_rank, world = env_rank()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    B = args.chunks_per_gpu
    max_ctx = args.prompt_len + args.gen_len
    eng = Engine(cfg, device=local_rank, max_batch=B, max_ctx=max_ctx,
                 max_prefill_tokens=B * args.prompt_len)
    quant = args.weights == "q4_k_m"
    if quant:
        eng.init_synthetic_q(seed=2, scale=0.02, norm_jitter=0.0)
    else:
        eng.init_synthetic(seed=0, std=0.02, norm_jitter=0.0)
    chunks = synthetic_chunks(B, args.prompt_len, doc=rank, vocab=cfg.vocab, bos=cfg.bos_id)
    units = [Unit(rank, i, args.prompt_len) for i in range(B)]

    def one_step():
        res = eng.generate(chunks, num_predict=args.gen_len, ignore_eos=True)
        packed = pack_results(units, [r.ids for r in res], args.gen_len)
        return gather_summaries(packed, B, device=dev)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        one_step()
    eng.reset_stats()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rows = one_step()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    st = eng.stats()
    total_chunks = world * B * args.steps
    value = total_chunks / dt
    assert rows is not None and len(rows) == world * B

    roof = None
    if not args.no_roofline:
        # Roofline of the dominant kernel class (the decode projections): one more map
        # step with HIP events bracketing every gemv launch on the engine's stream.  It
        # runs after the timed region because an event pair per launch (112 per decode
        # step) costs ~0.6 ms/step and would distort `value`.
        eng.reset_stats()
        eng.set_profiling((1 << L.K_GEMV) | (1 << L.K_LMHEAD))
        one_step()
        eng.set_profiling(0)
        sp = eng.stats()
        launches = sp["kernel_launches"][L.K_GEMV] + sp["kernel_launches"][L.K_LMHEAD]
        if launches:
            gemv_s = (sp["kernel_ms"][L.K_GEMV] + sp["kernel_ms"][L.K_LMHEAD]) / 1e3
            per_step = (qgemv_bytes_per_step(cfg, B) if quant else gemv_bytes_per_step(cfg, B)) \
                + lm_head_bytes_per_step(cfg, B, quant)
            bytes_total = per_step * sp["decode_steps"]
            ach = bytes_total / gemv_s / 1e9
            traffic, traffic_src = pmc_traffic(args.weights)
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": ("qgemv_kernel (Q4_K/Q6_K" if quant else "gemv_kernel (bf16")
                              + " decode weight stream: QKV/O/gate-up/down projections + lm_head)",
                    "bytes_per_launch": int(bytes_total / launches),
                    "avg_launch_us": round(gemv_s / launches * 1e6, 2),
                    "method": "hipExtLaunchKernelGGL start/stop events per launch, one extra untimed map step"}
    pre_flops = prefill_flops_per_chunk(cfg, args.prompt_len) * B * args.steps
    out = {
        "metric": METRIC, "value": round(value, 4), "unit": "chunks/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": ("synthetic (random Q4_K/Q6_K blocks in the Q4_K_M mix, seed 2, uniform token ids)"
                 if quant else "synthetic (random-init Llama-3.2-3B bf16 weights, uniform token ids)"),
        "config": {"workload": f"{'configs[4]' if quant else 'configs[1]'}: {B} x {args.prompt_len}-tok chunks -> {args.gen_len}-tok "
                               f"greedy summaries per GPU (ignore_eos), batched prefill + decode, "
                               f"summary ids gathered to rank 0",
                   "model": cfg.name, "weights": args.weights, "chunks_per_gpu": B, "prompt_tokens": args.prompt_len,
                   "summary_tokens": args.gen_len, "global_batch": world * B,
                   "seq_len": args.prompt_len + args.gen_len, "parallelism": f"chunk-dp{world}"},
        "breakdown": {"prefill_ms_per_step": round(st["prefill_ms"] / args.steps, 2),
                      "decode_ms_per_step": round(st["decode_ms"] / args.steps, 2),
                      "decode_steps": st["decode_steps"],
                      "prefill_tflops": round(pre_flops / (st["prefill_ms"] / 1e3) / 1e12, 1)
                      if st["prefill_ms"] else None,
                      "gemv_ms_total": round(st["kernel_ms"][L.K_GEMV], 2)},
        "roofline": roof,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, args.prompt_len, args.gen_len)
    eng.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
