"""TEST / BASELINE INFRASTRUCTURE ONLY -- torch-CPU bf16 restatement of the map call.

BASELINE.md §2's fallback CPU baseline: when Ollama and the fp16 GGUF are absent on the
box (they are -- SURVEY.md §8c), time "the build's CPU restatement (torch-CPU bf16, all
cores) on the same synthetic inputs", labelled "CPU restatement (not Ollama)".  It
runs the same Llama-3.2 map call as ``oracle/llama_ref.py`` (what Ollama does for one
``POST /api/generate`` of ``OllamaLLM._call``, run_full_evaluation_pipeline.py:80-106):
prefill of the prompt ids, then greedy decode with a KV cache.  Weights and
activations are bf16, matmuls go through torch's CPU GEMM (oneDNN) on every thread
``torch.get_num_threads()`` allows, attention is ``scaled_dot_product_attention``.

Only ``bench.py``'s ``cpu_baseline`` leg imports this; it is never on the product path.
"""
from __future__ import annotations

import math
import time

import torch
import torch.nn.functional as F

from . import synth as S
from .llama_ref import rope_inv_freq

_MASK32 = (1 << 32) - 1


def _u64(v: int) -> int:
    """An unsigned 64-bit constant as the int64 with the same bits."""
    return v - (1 << 64) if v >= 1 << 63 else v


def _shr(x, k: int):
    """Logical right shift of int64 tensors holding uint64 bit patterns."""
    return (x >> k) & ((1 << (64 - k)) - 1)


def _splitmix64_(x):
    """In place (int64 arithmetic wraps mod 2^64 like uint64)."""
    x.add_(_u64(0x9E3779B97F4A7C15))
    x.bitwise_xor_(_shr(x, 30)).mul_(_u64(0xBF58476D1CE4E5B9))
    x.bitwise_xor_(_shr(x, 27)).mul_(_u64(0x94D049BB133111EB))
    return x.bitwise_xor_(_shr(x, 31))


def synth_linear(seed: int, kind: int, layer: int, rows: int, cols: int, std: float, dtype=torch.bfloat16):
    """oracle/synth.py ``linear`` in torch (all threads): the engine's counter-based weights,
    bit for bit (tests/test_oracle.py checks against the numpy restatement)."""
    sh = int(S.splitmix64(S.np.uint64(seed)))
    scale = float(S.np.float32(std * S.np.sqrt(3.0) / 65536.0))
    out = torch.empty(rows, cols, dtype=dtype)
    c = torch.arange(cols, dtype=torch.int64)[None, :]
    step = max(1, (1 << 20) // cols)
    for r0 in range(0, rows, step):
        r = torch.arange(r0, min(rows, r0 + step), dtype=torch.int64)[:, None]
        h = ((r << 20) | c).bitwise_or_((kind << 58) | (layer << 50)).bitwise_xor_(_u64(sh))
        _splitmix64_(h)
        lim = (h & 0xFFFF).add_((h >> 16) & 0xFFFF).add_((h >> 32) & 0xFFFF).add_(_shr(h, 48)).sub_(131070)
        out[r0:r0 + r.shape[0]] = lim.to(torch.float32).mul_(scale).to(dtype)  # RNE, as bf16_rne
    return out


def synth_norm(seed: int, kind: int, layer: int, n: int, jitter: float, dtype=torch.bfloat16):
    return torch.from_numpy(S.norm(seed, kind, layer, n, jitter)).to(dtype)


class TorchCpuLlama:
    """The map call on the CPU, over the engine's own synthetic weights (ms_init_synthetic /
    oracle/synth.py: same seed, std, norm jitter -> the same bf16 values)."""

    def __init__(self, cfg, seed: int = 0, std: float = 0.02, jitter: float = 0.0, dtype=torch.bfloat16,
                 progress=None):
        self.cfg, self.dt = cfg, dtype
        H, D, F_ = cfg.hidden, cfg.head_dim, cfg.ffn
        QD, KD = cfg.n_heads * D, cfg.n_kv_heads * D

        def lin(kind, layer, r, c):
            return synth_linear(seed, kind, layer, r, c, std, dtype)
        self.embed = lin(S.EMBED, 0, cfg.vocab, H)
        self.lm_head = self.embed if cfg.tie_embeddings else lin(S.LM_HEAD, 0, cfg.vocab, H)
        self.layers = []
        for l in range(cfg.n_layers):
            self.layers.append({
                "wqkv": torch.cat([lin(S.WQ, l, QD, H), lin(S.WK, l, KD, H), lin(S.WV, l, KD, H)]),
                "wo": lin(S.WO, l, H, QD),
                "wgu": torch.cat([lin(S.WGATE, l, F_, H), lin(S.WUP, l, F_, H)]), "wdown": lin(S.WDOWN, l, H, F_),
                "n1": synth_norm(seed, S.ATTN_NORM, l, H, jitter, dtype),
                "n2": synth_norm(seed, S.FFN_NORM, l, H, jitter, dtype)})
            if progress is not None and (l + 1) % 4 == 0:
                progress(f"weights: {l + 1}/{cfg.n_layers} layers")
        self.final_norm = synth_norm(seed, S.FINAL_NORM, 0, H, jitter, dtype)
        self.inv_freq = torch.tensor(rope_inv_freq(cfg), dtype=torch.float64)

    def _rope(self, x, pos):
        ang = pos.to(torch.float64)[:, None] * self.inv_freq[None, :]
        c, s = ang.cos().to(torch.float32)[:, None, :], ang.sin().to(torch.float32)[:, None, :]
        h = x.shape[-1] // 2
        a, b = x[..., :h].float(), x[..., h:].float()
        return torch.cat([a * c - b * s, b * c + a * s], -1).to(self.dt)

    def _norm(self, x, w):
        """The deferred RMSNorm of the numerics contract (oracle/llama_ref.py): the GEMM input
        bf16(x * w) and the row factor r the projection's output is scaled by."""
        xf = x.float()
        return (xf * w.float()).to(self.dt), torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.cfg.norm_eps)

    def _proj(self, x, w, W):
        xg, r = self._norm(x, w)
        return (xg @ W.T).float() * r

    @torch.inference_mode()
    def forward(self, ids, cache, p0, progress=None):
        """ids [T] after p0 cached tokens; returns the last position's greedy id.  progress(l):
        called after each layer (long CPU prefills report as they go)."""
        cfg = self.cfg
        T = ids.shape[0]
        D, Hq, Hk = cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
        pos = torch.arange(p0, p0 + T)
        x = self.embed[ids].float()
        for l, L in enumerate(self.layers):
            qkv = self._proj(x, L["n1"], L["wqkv"]).to(self.dt)
            q = self._rope(qkv[:, :Hq * D].view(T, Hq, D), pos)
            k = self._rope(qkv[:, Hq * D:(Hq + Hk) * D].view(T, Hk, D), pos)
            v = qkv[:, (Hq + Hk) * D:].view(T, Hk, D)
            kc, vc = cache[l]
            kc[p0:p0 + T], vc[p0:p0 + T] = k, v
            K = kc[:p0 + T].transpose(0, 1)  # [Hk][keys][D]: grouped-query SDPA reads each kv
            V = vc[:p0 + T].transpose(0, 1)  # head for its Hq / Hk query heads (no repeat copy)
            o = F.scaled_dot_product_attention(q.transpose(0, 1), K, V, is_causal=(T > 1 and p0 == 0),
                                               scale=1.0 / math.sqrt(D), enable_gqa=True)
            x = x + (o.transpose(0, 1).reshape(T, Hq * D) @ L["wo"].T).float()
            gu = self._proj(x, L["n2"], L["wgu"])
            h = F.silu(gu[:, :cfg.ffn].float()) * gu[:, cfg.ffn:].float()
            x = x + (h.to(self.dt) @ L["wdown"].T).float()
            if progress is not None:
                progress(l)
        self.last_logits = self._proj(x[-1:], self.final_norm, self.lm_head)[0]
        return int(torch.argmax(self.last_logits))

    def new_cache(self, max_ctx):
        c = self.cfg
        return [(torch.zeros(max_ctx, c.n_kv_heads, c.head_dim, dtype=self.dt),
                 torch.zeros(max_ctx, c.n_kv_heads, c.head_dim, dtype=self.dt)) for _ in range(c.n_layers)]


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def time_chunk(cfg, prompt_ids, gen_len: int, decode_sample: int = 16, seed: int = 0, std: float = 0.02) -> dict:
    """Time one map call on the CPU: the full prefill of ``prompt_ids`` plus
    ``decode_sample`` greedy decode steps, extrapolated to ``gen_len`` generated tokens
    (decode steps at this context length cost the same to within the KV growth).  The weights
    are the engine's (bench.py: ms_init_synthetic(seed 0, std 0.02, jitter 0))."""
    import sys

    def note(msg):  # progress on stderr: a GPU-box run that prints nothing for minutes looks hung
        print(f"[cpu_baseline] {msg}", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    note(f"building weights ({torch.get_num_threads()} threads)")
    m = TorchCpuLlama(cfg, seed=seed, std=std, progress=note)
    note(f"weights built in {time.perf_counter() - t0:.1f} s, {torch.get_num_threads()} threads")
    ids = torch.as_tensor(prompt_ids, dtype=torch.long)
    P = ids.shape[0]
    cache = m.new_cache(P + gen_len)
    t0 = time.perf_counter()
    tok = m.forward(ids, cache, 0, progress=lambda l: (l + 1) % 7 == 0 and note(
        f"prefill layer {l + 1}/{cfg.n_layers}: {time.perf_counter() - t0:.1f} s"))
    t_pre = time.perf_counter() - t0
    note(f"prefill of {P} tokens: {t_pre:.1f} s")
    n = min(decode_sample, gen_len - 1)
    t0 = time.perf_counter()
    for i in range(n):
        tok = m.forward(torch.tensor([tok]), cache, P + i)
        if (i + 1) % 16 == 0:
            note(f"decode step {i + 1}/{n}: {(time.perf_counter() - t0) / (i + 1) * 1e3:.1f} ms/step")
    t_dec = (time.perf_counter() - t0) / max(n, 1)
    chunk_s = t_pre + (gen_len - 1) * t_dec
    return {"prefill_s": t_pre, "decode_step_s": t_dec, "chunk_s": chunk_s,
            "threads": torch.get_num_threads(), "decode_steps_timed": n, "cpu_model": cpu_model()}
