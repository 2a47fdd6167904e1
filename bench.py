"""bench.py -- map-phase chunks/s of the MI355X engine (BASELINE.json metric).

A "step" = one map phase over one batch of synthetic chunks.  Default (BASELINE.json
configs[1]): every GPU takes 8 synthetic 2048-token chunks (one 16k-token doc split in
8), prefills them packed, decodes exactly 256 greedy tokens each (ignore_eos, SURVEY.md
§8d), and the per-chunk summary ids are gathered to rank 0 over RCCL.  ``--docs D``
(configs[2]): D docs x 8 chunks, sharded over the ranks (chunk i -> rank i mod N), run
as one continuous batch of at most ``--max-batch`` sequences per GPU.  value = chunks of
all ranks / max-over-ranks wall time.  N > 1 is weak scaling in the default mode (each
rank owns its own document: SURVEY.md §8e).

    python bench.py [--gpus N --steps K --warmup W]      # N > 1: launches N ranks itself
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
DGEMM_MIN = 24              # engines of >= 24 slots decode on the skinny GEMM (engine.cpp dgemm_min)
F16_PEAK_TFLOPS = 2500.0    # dense fp16 (= bf16) MFMA (MI355X_MICROARCH.md chip table)
CHUNKS_PER_DOC = 8          # BASELINE.json configs[0..2]: a 16k-token doc in 2k chunks


def synthetic_chunks(n, prompt_len, doc, vocab, bos, seed=0, first_chunk=0):
    """Token ids of n chunks: BOS + Llama-3 header ids + uniform body over [0, 128000)
    (no tokenizer / dataset offline; timing of dense ops does not depend on values).
    Chunk c of doc d is the same wherever it runs (seeded by (d, c))."""
    head = [bos, 128006, 9125, 128007, 271, 128009, 128006, 882, 128007, 271]
    tail = [128009, 128006, 78191, 128007, 271]
    out = []
    for c in range(first_chunk, first_chunk + n):
        rng = np.random.default_rng((seed, doc, c))
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


def persist_bytes_per_launch(cfg, B, kv_read_tokens):
    """The persistent decode step (k_persist.hip), one launch = every layer of one decode step:
    each layer's weights once + the B activation rows in / out (gemv_bytes_per_step), the K/V of
    the cached keys it attends (SURVEY.md §8d's KV-read term; kv_read_tokens = keys summed over
    the batch rows, all layers) and the new tokens' K/V rows it writes."""
    return gemv_bytes_per_step(cfg, B) + kv_read_tokens * cfg.kv_bytes_per_token + B * cfg.kv_bytes_per_token


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


def decode_weight_bytes(cfg, quant=False):
    """Weight bytes one decode step streams (every layer matrix + the lm_head): SURVEY.md
    §8d's W = 6,425,149,440 B for 16-bit Llama-3.2-3B (the engine holds fp16)."""
    if not quant:
        return cfg.weight_bytes
    return qgemv_bytes_per_step(cfg, 0) + cfg.vocab * cfg.hidden * 224 / 256


def prefill_flops_per_chunk(cfg, P):
    """2*params_linear*P + lm_head on the last token + causal attention."""
    H, D, F = cfg.hidden, cfg.head_dim, cfg.ffn
    lin = cfg.n_layers * ((cfg.n_heads + 2 * cfg.n_kv_heads) * D * H + H * cfg.n_heads * D + 3 * H * F)
    attn = cfg.n_layers * cfg.n_heads * 4 * D * (P * (P + 1) // 2)
    return 2 * lin * P + 2 * cfg.vocab * H + attn


def cpu_baseline(cfg, prompt_ids, gen_len, decode_sample=64):
    """BASELINE.md §2 fallback (Ollama and the GGUF are absent on the box): the torch-CPU
    bf16 restatement of the same map call (oracle/torch_cpu.py), all 28 layers, on one
    chunk of this workload: its full 2048-token prefill + ``decode_sample`` greedy decode
    steps, extrapolated to the 256 generated tokens.  Threads: every CPU this process may
    run on -- its affinity mask capped by its cgroup CPU quota (BASELINE.md §2 asks for
    num_thread = physical cores; the sample text records the mask, the quota and the host's
    physical cores)."""
    import torch
    from oracle.torch_cpu import time_chunk
    allowed = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    # every CPU this process can actually run on: the affinity mask, capped by the cgroup CPU
    # quota (a GPU box's share of a big host shows every host CPU in the mask; threads past
    # the quota only oversubscribe it)
    threads = min(allowed, quota) if quota else allowed
    torch.set_num_threads(threads)
    phys = _physical_cores()
    r = time_chunk(cfg, prompt_ids, gen_len, decode_sample=decode_sample)
    # numerics: bf16, not the engine's fp16 -- torch's CPU GEMM has no fp16 fast path (measured in
    # the build container: 266 GF/s fp16 vs 1252 GF/s bf16 at 256 x 8192 x 3072, 8 threads), so an
    # fp16 sample would time torch's fp16 emulation, not a CPU running this model
    return {"value": round(1.0 / r["chunk_s"], 5), "unit": "chunks/s", "cores": int(r["threads"]),
            "kind": "port", "dtype": "bf16", "cpu_model": r["cpu_model"],
            "sample": (f"CPU restatement (not Ollama): torch {torch.__version__} CPU bf16 on {r['cpu_model']}, "
                       f"{r['threads']} threads = every CPU this process may use (affinity mask {allowed}, "
                       f"cgroup quota {quota if quota else 'none'}; {phys} physical cores on the host), "
                       f"{cfg.n_layers}-layer Llama-3.2-3B on the engine's own synthetic weights, "
                       f"1 chunk: {len(prompt_ids)}-tok prefill "
                       f"{r['prefill_s']:.2f} s + {r['decode_steps_timed']} decode steps at "
                       f"{r['decode_step_s'] * 1e3:.1f} ms, extrapolated to {gen_len} tokens "
                       f"({r['chunk_s']:.1f} s/chunk)")}


def _cgroup_cpus():
    """CPUs of this process's cgroup v2 quota (cpu.max "quota period"), or None if unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        return None


def _physical_cores():
    """Distinct (physical id, core id) pairs in /proc/cpuinfo (None if unreadable)."""
    try:
        cores, phys = set(), None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":")[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":")[1].strip()))
        return len(cores) or None
    except OSError:
        return None


def pmc_traffic(weights, B, prompt_len, kernel="gemv"):
    """HBM bytes per weight-stream launch from the committed rocprofv3 --pmc passes of the
    same launches (FETCH_SIZE x2 + WRITE_SIZE, tools/traffic_from_pmc.py, run by
    tools/gpu_round.sh / tools/gpu_r5af.sh), or (None, None) when none was taken.  B is the
    engine's max_batch = the rows in flight; a pass matches when its rows (min(chunks,
    max_batch)), hence its decode regime (skinny GEMM at >= DGEMM_MIN rows, else GEMV), and
    its prompt length are this run's.  PMC counters cannot be read inside a timed run: this
    is the profiler's number."""
    import glob
    key = (B, B >= DGEMM_MIN, prompt_len)
    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_traffic_{weights}*.json")))
    for h in reversed(hits):
        d = json.load(open(h))
        if d.get("kernel_class", "gemv") != kernel:  # the persistent step's passes say "persist"
            continue
        wl = d.get("workload", {})
        c = wl.get("chunks_per_gpu")
        if c is None:
            continue
        m = wl.get("max_batch", c)
        if (min(c, m), m >= DGEMM_MIN, wl.get("prompt_len")) == key:
            return d["traffic_bytes_per_launch"], os.path.relpath(h, ROOT)
    return None, None


def _spawn_ranks(n):
    """`python bench.py --gpus N` outside torchrun: start N ranks (one per GPU) as
    children through torch.distributed.run, before this process touches any GPU, and
    exit with their status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--chunks-per-gpu", type=int, default=8)
    ap.add_argument("--docs", type=int, default=0,
                    help="configs[2]: D docs x 8 chunks over all ranks as one continuous batch per GPU")
    ap.add_argument("--max-batch", type=int, default=64,
                    help="--docs mode: sequences in flight per GPU (continuous batching)")
    ap.add_argument("--prompt-len", type=int, default=2048)
    ap.add_argument("--gen-len", type=int, default=256)
    ap.add_argument("--model", default="llama3.2-3b")
    ap.add_argument("--weights", choices=("f16", "q4_k_m"), default="f16",
                    help="q4_k_m = BASELINE configs[4]: random Q4_K/Q6_K blocks, K-quant decode GEMVs")
    ap.add_argument("--eos", type=int, default=0,
                    help="natural-EOS mode: stop at a synthetic set of N stop ids (seeded) instead of "
                         "ignore_eos, so chunks finish at varied lengths and slots turn over")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true", help="skip HIP-event timing of the GEMV class")
    ap.add_argument("--no-check", action="store_true", help="skip the output self-checks")
    ap.add_argument("--bcast-weights", action="store_true",
                    help="N > 1: rank 0 makes the weights, the other ranks receive them over RCCL")
    return ap.parse_args(argv)


def local_units(args, rank, world):
    """(doc, chunk) units of this rank.  Default: the rank's own doc; --docs: the global
    (doc, chunk) list sharded statically (uniform chunks)."""
    from mapsum.dist import Unit, shard_static
    if args.docs:
        units = [Unit(d, c, args.prompt_len) for d in range(args.docs) for c in range(CHUNKS_PER_DOC)]
        return shard_static(units, rank, world)
    return [Unit(rank, i, args.prompt_len) for i in range(args.chunks_per_gpu)]


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    from mapsum import _lib as L
    from mapsum.config import CONFIGS
    from mapsum.dist import env_rank, gather_summaries, pack_results
    from mapsum.engine import Engine

    cfg = CONFIGS[args.model]
    rank, local_rank, world = env_rank()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    units = local_units(args, rank, world)
    n_local = len(units)
    max_rows = max(len(local_units(args, r, world)) for r in range(world))
    B = min(args.max_batch, n_local) if args.docs else n_local
    max_ctx = args.prompt_len + args.gen_len
    eng = Engine(cfg, device=local_rank, max_batch=B, max_ctx=max_ctx,
                 max_prefill_tokens=min(B, 8) * args.prompt_len)
    quant = args.weights == "q4_k_m"
    t_load = time.perf_counter()
    if rank == 0 or not (args.bcast_weights and world > 1):
        if quant:
            eng.init_synthetic_q(seed=2, scale=0.02, norm_jitter=0.0)
        else:
            eng.init_synthetic(seed=0, std=0.02, norm_jitter=0.0)
    bcast_bytes = 0
    if args.bcast_weights and world > 1:
        from mapsum.dist import broadcast_engine_weights
        bcast_bytes = broadcast_engine_weights(eng, src=0)
    t_load = time.perf_counter() - t_load
    chunks = [synthetic_chunks(1, args.prompt_len, u.doc, cfg.vocab, cfg.bos_id, first_chunk=u.chunk)[0]
              for u in units]
    ignore_eos = args.eos <= 0
    if not ignore_eos:
        # random-init weights almost never pick the three real end-of-turn ids: a seeded stop set
        # of N ids ends a chunk with probability ~N/vocab per token (mean length ~vocab/N)
        eng.set_eos_ids(np.random.default_rng(99).choice(128000, size=args.eos, replace=False))
    gather_s = [0.0]

    def one_step():
        res = eng.generate(chunks, num_predict=args.gen_len, ignore_eos=ignore_eos)
        packed = pack_results(units, [r.ids for r in res], args.gen_len)
        t0 = time.perf_counter()
        rows = gather_summaries(packed, max_rows, device=dev)
        gather_s[0] += time.perf_counter() - t0
        return res, rows

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def note(msg):  # progress on stderr (rank 0): long runs must not look hung
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)
    note(f"engine ready (B={B}, weights {args.weights}, load {t_load:.1f} s)")
    for _ in range(args.warmup):
        one_step()
    note(f"{args.warmup} warmup step(s) done")
    eng.reset_stats()
    gather_s[0] = 0.0
    outs = []
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, rows = one_step()
        outs.append([r.ids for r in res])
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    st = eng.stats()
    total_chunks = sum(len(local_units(args, r, world)) for r in range(world)) * args.steps
    value = total_chunks / dt
    assert rows is not None and int((rows[:, 2] >= 0).sum()) == total_chunks // args.steps

    # self-checks (outside the timed region): every step produced the same summaries, each
    # of the full length, and a chunk's summary does not depend on its batch companions
    check = None
    if not args.no_check:
        same = all(o == outs[0] for o in outs[1:])
        full = all(len(ids) == args.gen_len for ids in outs[0]) or not ignore_eos
        alone = eng.generate([chunks[0]], num_predict=args.gen_len, ignore_eos=ignore_eos)[0].ids
        check = {"deterministic_across_steps": same, "full_length": full,
                 "batch_invariant_chunk0": alone == outs[0][0]}
        assert same and full and check["batch_invariant_chunk0"], check

    roof = roof_lm = None
    if not args.no_roofline:
        # Roofline of the dominant kernel: one more map step with HIP events bracketing every
        # decode launch of its class on the engine's stream (an event pair per launch would
        # distort `value`, so this runs after the timed region).  Engines of <= 8 slots on fp16
        # weights run every layer of a decode step as ONE persistent launch (k_persist.hip):
        # its bytes are the layers' weights + the K/V it reads and writes; otherwise the class is
        # the per-projection weight stream (GEMV / skinny GEMM / K-quant GEMV) + the lm_head.
        eng.reset_stats()
        eng.set_profiling((1 << L.K_GEMV) | (1 << L.K_LMHEAD) | (1 << L.K_PERSIST))
        eng.generate(chunks[:min(len(chunks), B)], num_predict=min(args.gen_len, 64), ignore_eos=True)
        eng.set_profiling(0)
        sp = eng.stats()
        bstep = sp["decode_tokens"] / max(sp["decode_steps"], 1)
        n_pk = sp["kernel_launches"][L.K_PERSIST]
        n_lm = sp["kernel_launches"][L.K_LMHEAD]
        launches = sp["kernel_launches"][L.K_GEMV] + n_lm
        if n_pk:
            pk_s = sp["kernel_ms"][L.K_PERSIST] / 1e3
            kv_read = sp["decode_kv_tokens"] * 1.0  # keys attended per layer, summed over steps and rows
            pk_bytes = persist_bytes_per_launch(cfg, bstep, 0) * n_pk + kv_read * cfg.kv_bytes_per_token
            ach = pk_bytes / pk_s / 1e9
            traffic, traffic_src = pmc_traffic(args.weights, B, args.prompt_len, "persist")
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": "decode_step_kernel (persistent: all 28 layers of a decode step in one launch -- "
                              "QKV/O/gate-up/down weights + K/V reads and writes)",
                    "bytes_per_launch": int(pk_bytes / n_pk),
                    "avg_launch_us": round(pk_s / n_pk * 1e6, 2),
                    "method": "hipExtLaunchKernelGGL start/stop events per launch, one extra untimed map step"}
            if n_lm:
                lm_s = sp["kernel_ms"][L.K_LMHEAD] / 1e3
                lm_b = lm_head_bytes_per_step(cfg, bstep, quant) * n_lm
                roof_lm = {"bound": "hbm", "achieved": round(lm_b / lm_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(lm_b / lm_s / 1e9 / HBM_PEAK_GBS, 4),
                           "kernel": "gemv_kernel (lm_head + argmax partials)",
                           "bytes_per_launch": int(lm_b / n_lm), "avg_launch_us": round(lm_s / n_lm * 1e6, 2)}
        elif launches:
            gemv_s = (sp["kernel_ms"][L.K_GEMV] + sp["kernel_ms"][L.K_LMHEAD]) / 1e3
            per_step = (qgemv_bytes_per_step(cfg, bstep) if quant else gemv_bytes_per_step(cfg, bstep)) \
                + lm_head_bytes_per_step(cfg, bstep, quant)
            bytes_total = per_step * sp["decode_steps"]
            ach = bytes_total / gemv_s / 1e9
            traffic, traffic_src = pmc_traffic(args.weights, B, args.prompt_len)
            skinny = not quant and B >= DGEMM_MIN
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": ("qgemv_kernel (Q4_K/Q6_K" if quant else
                               "dgemm_kernel (fp16 skinny GEMM, >= 24 slots:" if skinny else "gemv_kernel (fp16")
                              + " decode weight stream: QKV/O/gate-up/down projections + lm_head)",
                    "bytes_per_launch": int(bytes_total / launches),
                    "avg_launch_us": round(gemv_s / launches * 1e6, 2),
                    "method": "hipExtLaunchKernelGGL start/stop events per launch, one extra untimed map step"}
    # whole-phase rooflines from the timed run's own event-timed prefill / decode passes
    pre_flops = prefill_flops_per_chunk(cfg, args.prompt_len) * n_local * args.steps
    pre_tf = pre_flops / (st["prefill_ms"] / 1e3) / 1e12 if st["prefill_ms"] else None
    kvb = cfg.kv_bytes_per_token
    dec_bytes = (st["decode_steps"] * decode_weight_bytes(cfg, quant) + st["decode_kv_tokens"] * kvb
                 + st["decode_tokens"] * kvb)
    dec_gbs = dec_bytes / (st["decode_ms"] / 1e3) / 1e9 if st["decode_ms"] else None
    roof_pre = {"bound": "mfma", "achieved": round(pre_tf, 1), "peak": F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(pre_tf / F16_PEAK_TFLOPS, 4),
                "flops_per_chunk": prefill_flops_per_chunk(cfg, args.prompt_len),
                "method": "SURVEY.md §8d prefill FLOP / event-timed prefill passes (all kernels)"} if pre_tf else None
    roof_dec = {"bound": "hbm", "achieved": round(dec_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(dec_gbs / HBM_PEAK_GBS, 4),
                "bytes_per_step": round(dec_bytes / max(st["decode_steps"], 1)),
                "method": "weights + KV reads + KV writes (SURVEY.md §8d) / event-timed decode steps "
                          "(all kernels)"} if dec_gbs else None
    out = {
        "metric": METRIC, "value": round(value, 4), "unit": "chunks/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "q4_k_m+f16" if quant else "f16",
        "data": ("synthetic (random Q4_K/Q6_K blocks in the Q4_K_M mix, seed 2, uniform token ids)"
                 if quant else "synthetic (random-init Llama-3.2-3B weights held as fp16, uniform token ids)"),
        "config": {"workload": (f"configs[2]: {args.docs} docs x {CHUNKS_PER_DOC} x {args.prompt_len}-tok "
                                f"chunks over {world} GPU(s) ({n_local} per GPU, <= {B} in flight, "
                                f"continuous batching)" if args.docs else
                                f"{'configs[4]' if quant else 'configs[1]'}: {B} x {args.prompt_len}-tok chunks")
                               + (f" -> {args.gen_len}-tok greedy summaries (ignore_eos)" if ignore_eos else
                                  f" -> greedy summaries of <= {args.gen_len} tok stopping at a synthetic "
                                  f"{args.eos}-id stop set (natural EOS, mean "
                                  f"{np.mean([len(x) for x in outs[0]]):.1f} tok)")
                               + ", batched prefill + decode, summary ids gathered to rank 0",
                   "model": cfg.name, "weights": args.weights, "chunks_per_gpu": n_local, "max_batch": B,
                   "prompt_tokens": args.prompt_len, "summary_tokens": args.gen_len,
                   "global_batch": total_chunks // args.steps,
                   "seq_len": args.prompt_len + args.gen_len, "parallelism": f"chunk-dp{world}"},
        "breakdown": {"prefill_ms_per_step": round(st["prefill_ms"] / args.steps, 2),
                      "decode_ms_per_step": round(st["decode_ms"] / args.steps, 2),
                      "decode_steps": st["decode_steps"],
                      "summary_tokens_per_step": int(sum(len(x) for x in outs[0])),
                      "graphs_built": st["graphs_built"],
                      "persist_steps": st["persist_steps"],
                      "persist_fallbacks": st["persist_fallbacks"],
                      "decode_ms_per_decode_step": round(st["decode_ms"] / max(st["decode_steps"], 1), 4),
                      "gather_ms_per_step": round(gather_s[0] / args.steps * 1e3, 3),
                      "weight_load_s": round(t_load, 3),
                      "weight_bcast_bytes": bcast_bytes,
                      "prefill_tflops": round(pre_tf, 1) if pre_tf else None},
        "roofline": roof,
        "roofline_prefill": roof_pre,
        "roofline_decode": roof_dec,
        "roofline_lm_head": roof_lm,
        "check": check,
        "cpu_baseline": None,
    }
    note(f"timed {args.steps} step(s): {value:.3f} chunks/s")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        eng.close()
        out["cpu_baseline"] = cpu_baseline(cfg, chunks[0], args.gen_len)
    eng.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
