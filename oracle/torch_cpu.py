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

from .llama_ref import rope_inv_freq


class TorchCpuLlama:
    def __init__(self, cfg, seed: int = 0, std: float = 0.02, dtype=torch.bfloat16):
        self.cfg, self.dt = cfg, dtype
        g = torch.Generator().manual_seed(seed)
        H, D, F_ = cfg.hidden, cfg.head_dim, cfg.ffn

        def lin(r, c):
            return (torch.randn(r, c, generator=g, dtype=torch.float32) * std).to(dtype)
        self.embed = lin(cfg.vocab, H)
        self.layers = []
        for _ in range(cfg.n_layers):
            self.layers.append({
                "wqkv": lin((cfg.n_heads + 2 * cfg.n_kv_heads) * D, H), "wo": lin(H, cfg.n_heads * D),
                "wgu": lin(2 * F_, H), "wdown": lin(H, F_),
                "n1": torch.ones(H, dtype=dtype), "n2": torch.ones(H, dtype=dtype)})
        self.final_norm = torch.ones(H, dtype=dtype)
        self.inv_freq = torch.tensor(rope_inv_freq(cfg), dtype=torch.float64)

    def _rope(self, x, pos):
        ang = pos.to(torch.float64)[:, None] * self.inv_freq[None, :]
        c, s = ang.cos().to(torch.float32)[:, None, :], ang.sin().to(torch.float32)[:, None, :]
        h = x.shape[-1] // 2
        a, b = x[..., :h].float(), x[..., h:].float()
        return torch.cat([a * c - b * s, b * c + a * s], -1).to(self.dt)

    def _norm(self, x, w):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.cfg.norm_eps)).to(self.dt) * w

    @torch.inference_mode()
    def forward(self, ids, cache, p0):
        """ids [T] after p0 cached tokens; returns the last position's greedy id."""
        cfg = self.cfg
        T = ids.shape[0]
        D, Hq, Hk = cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
        pos = torch.arange(p0, p0 + T)
        x = self.embed[ids].float()
        for l, L in enumerate(self.layers):
            qkv = self._norm(x, L["n1"]) @ L["wqkv"].T
            q = self._rope(qkv[:, :Hq * D].view(T, Hq, D), pos)
            k = self._rope(qkv[:, Hq * D:(Hq + Hk) * D].view(T, Hk, D), pos)
            v = qkv[:, (Hq + Hk) * D:].view(T, Hk, D)
            kc, vc = cache[l]
            kc[p0:p0 + T], vc[p0:p0 + T] = k, v
            K = kc[:p0 + T].transpose(0, 1).repeat_interleave(Hq // Hk, 0)
            V = vc[:p0 + T].transpose(0, 1).repeat_interleave(Hq // Hk, 0)
            o = F.scaled_dot_product_attention(q.transpose(0, 1), K, V, is_causal=(T > 1 and p0 == 0),
                                               scale=1.0 / math.sqrt(D))
            x = x + (o.transpose(0, 1).reshape(T, Hq * D) @ L["wo"].T).float()
            gu = self._norm(x, L["n2"]) @ L["wgu"].T
            h = F.silu(gu[:, :cfg.ffn].float()) * gu[:, cfg.ffn:].float()
            x = x + (h.to(self.dt) @ L["wdown"].T).float()
        xn = self._norm(x[-1:], self.final_norm)
        return int(torch.argmax((xn @ self.embed.T).float(), -1))

    def new_cache(self, max_ctx):
        c = self.cfg
        return [(torch.zeros(max_ctx, c.n_kv_heads, c.head_dim, dtype=self.dt),
                 torch.zeros(max_ctx, c.n_kv_heads, c.head_dim, dtype=self.dt)) for _ in range(c.n_layers)]


def time_chunk(cfg, prompt_ids, gen_len: int, decode_sample: int = 16, seed: int = 0) -> dict:
    """Time one map call on the CPU: the full prefill of ``prompt_ids`` plus
    ``decode_sample`` greedy decode steps, extrapolated to ``gen_len`` generated tokens
    (decode steps at this context length cost the same to within the KV growth)."""
    m = TorchCpuLlama(cfg, seed=seed)
    ids = torch.as_tensor(prompt_ids, dtype=torch.long)
    P = ids.shape[0]
    cache = m.new_cache(P + gen_len)
    t0 = time.perf_counter()
    tok = m.forward(ids, cache, 0)
    t_pre = time.perf_counter() - t0
    n = min(decode_sample, gen_len - 1)
    t0 = time.perf_counter()
    for i in range(n):
        tok = m.forward(torch.tensor([tok]), cache, P + i)
    t_dec = (time.perf_counter() - t0) / max(n, 1)
    chunk_s = t_pre + (gen_len - 1) * t_dec
    return {"prefill_s": t_pre, "decode_step_s": t_dec, "chunk_s": chunk_s,
            "threads": torch.get_num_threads(), "decode_steps_timed": n}
