"""Model configurations for the map-phase engine.

The reference pins its model only by Ollama tag: ``llama3.2:3b`` (README.md:28-33,
run_full_evaluation_pipeline.py:961); BASELINE.json's oracle is
``llama3.2:3b-instruct-fp16``.  The shapes below are the public Llama-3.2-3B
config (EXT).  ``TINY`` keeps every structural property the
kernels specialise on (head_dim 128, GQA group 3, tied embeddings, llama3 RoPE)
at a size the numpy oracle runs in seconds.
"""
from __future__ import annotations

from dataclasses import dataclass, replace


@dataclass(frozen=True)
class ModelConfig:
    name: str
    n_layers: int
    hidden: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    ffn: int
    vocab: int
    rope_theta: float = 500000.0
    rope_factor: float = 32.0
    rope_low_freq_factor: float = 1.0
    rope_high_freq_factor: float = 4.0
    rope_orig_ctx: int = 8192
    norm_eps: float = 1e-5
    tie_embeddings: bool = True
    bos_id: int = 128000
    eos_ids: tuple = (128001, 128008, 128009)

    def with_(self, **kw) -> "ModelConfig":
        return replace(self, **kw)

    @property
    def weight_bytes(self) -> int:
        """bf16 bytes of the matrices one decode step streams (tied lm_head counted once;
        RMSNorm vectors excluded) -- SURVEY.md §8d W = 6,425,149,440 B for Llama-3.2-3B."""
        H, D = self.hidden, self.head_dim
        per_layer = (H * (self.n_heads + 2 * self.n_kv_heads) * D + self.n_heads * D * H
                     + 3 * H * self.ffn)
        emb = self.vocab * H * (1 if self.tie_embeddings else 2)
        return 2 * (self.n_layers * per_layer + emb)

    @property
    def kv_bytes_per_token(self) -> int:
        return 2 * self.n_layers * self.n_kv_heads * self.head_dim * 2


def llama3_rope_factors(cfg):
    """The per-frequency divisors of llama3 RoPE scaling, float64 [head_dim / 2]: base inverse
    frequency / scaled one -- what llama.cpp's converter stores as the GGUF ``rope_freqs.weight``
    tensor and what the engine's own cos / sin tables apply (engine.cpp rope_tables).  All ones
    without scaling (rope_factor 0)."""
    import math

    import numpy as np
    D = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (np.arange(0, D, 2, dtype=np.float64) / D))
    if not cfg.rope_factor or cfg.rope_factor <= 0:
        return np.ones_like(inv)
    low_wl = cfg.rope_orig_ctx / cfg.rope_low_freq_factor
    high_wl = cfg.rope_orig_ctx / cfg.rope_high_freq_factor
    wl = 2.0 * math.pi / inv
    out = np.where(wl > low_wl, inv / cfg.rope_factor, inv)
    smooth = (cfg.rope_orig_ctx / wl - cfg.rope_low_freq_factor) / (cfg.rope_high_freq_factor - cfg.rope_low_freq_factor)
    smoothed = (1.0 - smooth) * out / cfg.rope_factor + smooth * out
    medium = ~(wl < high_wl) & ~(wl > low_wl)
    return inv / np.where(medium, smoothed, out)


LLAMA32_3B = ModelConfig(name="llama3.2-3b", n_layers=28, hidden=3072, n_heads=24, n_kv_heads=8,
                         head_dim=128, ffn=8192, vocab=128256)

# Tiny test model: same kernel-relevant structure (head_dim 128, GQA 3:1, tied).
TINY = ModelConfig(name="tiny", n_layers=2, hidden=768, n_heads=6, n_kv_heads=2, head_dim=128,
                   ffn=2048, vocab=4096, bos_id=4000, eos_ids=(4001, 4002))

CONFIGS = {c.name: c for c in (LLAMA32_3B, TINY)}
