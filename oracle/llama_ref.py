"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the Llama-3.2 map call.

Restates what happens inside Ollama for one ``POST /api/generate`` made by
``OllamaLLM._call`` (reference ``run_full_evaluation_pipeline.py:80-106``;
runner copies ``runners/run_summarization_ollama_mapreduce.py:37-49``), i.e.
SURVEY.md §8a rows A7-A9: prefill of the prompt ids, then greedy decode up to
``num_predict`` tokens or an end-of-turn id.  The arithmetic itself is EXT
(Ollama / llama.cpp are not vendored); the architecture restated here is the
public Llama-3.2 one (RMSNorm, GQA attention with llama3-scaled rotate-half
RoPE, SwiGLU MLP, tied lm_head) and is pinned against
``transformers.LlamaForCausalLM`` by ``tests/golden/make_golden.py``.

Rounding points (the engine's numerics contract):
  residual stream fp32; every GEMM input bf16, fp32 accumulate; a normalised projection
  (QKV, gate/up, lm_head) multiplies bf16(x * g) by W and scales each output row by the
  RMSNorm factor r = 1/sqrt(mean(x^2) + eps) in fp32 -- r * (bf16(x*g) . W^T), the
  deferred form of W . (x*r*g), so the producer of x can emit the GEMM input without
  knowing the row's norm; Q/K/V, RoPE output, attention output and the SwiGLU product
  rounded to bf16; attention scores/softmax fp32; logits fp32; argmax ties -> lowest id.
The only deliberate difference from the HIP path: softmax here is exact fp32 (the flash
kernels feed P to the P.V MFMAs as hi + lo bf16 halves), which the tests' tolerances cover.
"""
from __future__ import annotations

import math

import numpy as np

from .synth import bf16_rne


def rope_inv_freq(cfg) -> np.ndarray:
    """llama3-scaled inverse frequencies, float64 [head_dim/2] (HF _compute_llama3_parameters)."""
    D = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (np.arange(0, D, 2, dtype=np.float64) / D))
    if cfg.rope_factor and cfg.rope_factor > 0:
        low_wl = cfg.rope_orig_ctx / cfg.rope_low_freq_factor
        high_wl = cfg.rope_orig_ctx / cfg.rope_high_freq_factor
        wl = 2.0 * math.pi / inv
        out = np.where(wl > low_wl, inv / cfg.rope_factor, inv)
        smooth = (cfg.rope_orig_ctx / wl - cfg.rope_low_freq_factor) / (
            cfg.rope_high_freq_factor - cfg.rope_low_freq_factor)
        smoothed = (1.0 - smooth) * out / cfg.rope_factor + smooth * out
        medium = ~(wl < high_wl) & ~(wl > low_wl)
        inv = np.where(medium, smoothed, out)
    return inv


def rope_tables(cfg, positions) -> tuple[np.ndarray, np.ndarray]:
    ang = np.asarray(positions, dtype=np.float64)[:, None] * rope_inv_freq(cfg)[None, :]
    return np.cos(ang).astype(np.float32), np.sin(ang).astype(np.float32)


def _f32(x):
    return np.asarray(x, dtype=np.float32)


def rms_rinv(x: np.ndarray, eps: float) -> np.ndarray:
    """The RMSNorm factor r = 1/sqrt(mean(x^2) + eps) per row, [..., 1] fp32."""
    ms = np.mean(x.astype(np.float32) ** 2, axis=-1, keepdims=True, dtype=np.float32)
    return (np.float32(1.0) / np.sqrt(ms + np.float32(eps))).astype(np.float32)


def norm_input(x: np.ndarray, g: np.ndarray, rnd=bf16_rne) -> np.ndarray:
    """The bf16 GEMM input of a normalised projection: bf16(x * g) (r applied after the GEMM)."""
    return rnd(x * g)


def rmsnorm(x: np.ndarray, g: np.ndarray, eps: float, rnd=bf16_rne) -> np.ndarray:
    """Plain RMSNorm (x * r) * g, rounded: for callers that want the normalised rows."""
    return rnd((x * rms_rinv(x, eps)) * g)


def apply_rope(x: np.ndarray, cos: np.ndarray, sin: np.ndarray, rnd=bf16_rne) -> np.ndarray:
    """x [T, heads, D] (bf16 values); rotate-half convention (HF)."""
    h = x.shape[-1] // 2
    a, b = x[..., :h], x[..., h:]
    c, s = cos[:, None, :], sin[:, None, :]
    return rnd(np.concatenate([a * c - b * s, b * c + a * s], axis=-1))


def silu(x):
    return x / (np.float32(1.0) + np.exp(-x))


class OracleLlama:
    """Greedy Llama-3.2 over bf16-valued float32 weights (oracle.synth.make_weights layout)."""

    def __init__(self, cfg, weights: dict, round_bf16: bool = True):
        """round_bf16=False turns every activation rounding off (pure fp32): the mode
        used to pin this restatement against transformers.LlamaForCausalLM."""
        self.cfg = cfg
        self.w = weights
        self.rnd = bf16_rne if round_bf16 else _f32

    def new_cache(self):
        return {"k": [None] * self.cfg.n_layers, "v": [None] * self.cfg.n_layers, "len": 0}

    def forward(self, ids, cache=None, collect: bool = False, all_logits: bool = False):
        """Run ``ids`` after whatever ``cache`` holds; returns (logits, probes).

        logits: [T, vocab] if all_logits else [vocab] for the last token.
        probes: per-layer residual after each layer (if collect)."""
        cfg, w = self.cfg, self.w
        ids = np.asarray(ids, dtype=np.int64)
        T = ids.shape[0]
        cache = cache if cache is not None else self.new_cache()
        p0 = cache["len"]
        pos = np.arange(p0, p0 + T)
        cos, sin = rope_tables(cfg, pos)
        D, Hq, Hk = cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
        G = Hq // Hk
        scale = np.float32(1.0 / math.sqrt(D))
        rnd = self.rnd
        x = w["embed"][ids].astype(np.float32)
        probes = []
        for l, L in enumerate(w["layers"]):
            xg, r = norm_input(x, L["attn_norm"], rnd), rms_rinv(x, cfg.norm_eps)
            q = rnd(r * (xg @ L["wq"].T)).reshape(T, Hq, D)
            k = rnd(r * (xg @ L["wk"].T)).reshape(T, Hk, D)
            v = rnd(r * (xg @ L["wv"].T)).reshape(T, Hk, D)
            q = apply_rope(q, cos, sin, rnd)
            k = apply_rope(k, cos, sin, rnd)
            if cache["k"][l] is not None:
                k = np.concatenate([cache["k"][l], k], axis=0)
                v = np.concatenate([cache["v"][l], v], axis=0)
            cache["k"][l], cache["v"][l] = k, v
            S = k.shape[0]
            kq = np.repeat(k, G, axis=1)  # [S, Hq, D]
            vq = np.repeat(v, G, axis=1)
            s = np.matmul(q.transpose(1, 0, 2), kq.transpose(1, 2, 0)) * scale  # [Hq, T, S]
            mask = (np.arange(S)[None, :] > (p0 + np.arange(T))[:, None])
            s = np.where(mask[None], np.float32(-np.inf), s)
            s = s - s.max(axis=-1, keepdims=True)
            p = np.exp(s)
            p = p / p.sum(axis=-1, keepdims=True)
            o = rnd(np.matmul(p.astype(np.float32), vq.transpose(1, 0, 2)).transpose(1, 0, 2))  # [T, Hq, D]
            x = x + o.reshape(T, Hq * D) @ L["wo"].T
            xg, r = norm_input(x, L["ffn_norm"], rnd), rms_rinv(x, cfg.norm_eps)
            g = r * (xg @ L["w_gate"].T)
            u = r * (xg @ L["w_up"].T)
            h = rnd(silu(g) * u)
            x = x + h @ L["w_down"].T
            if collect:
                probes.append(x.copy())
        cache["len"] = p0 + T
        xs = x if all_logits else x[-1:]
        xg, r = norm_input(xs, w["final_norm"], rnd), rms_rinv(xs, cfg.norm_eps)
        logits = r * (xg @ w["lm_head"].T)
        return (logits if all_logits else logits[0]), probes

    def generate(self, ids, num_predict: int, eos_ids=(), ignore_eos: bool = False):
        """Greedy decode; returns (tokens, finish) with finish in {"eos", "length"}.
        The EOS id itself is not part of the returned tokens (Ollama drops it from
        ``response``)."""
        cache = self.new_cache()
        logits, _ = self.forward(ids, cache)
        out = []
        while True:
            t = int(np.argmax(logits))
            if not ignore_eos and t in eos_ids:
                return out, "eos"
            out.append(t)
            if len(out) >= num_predict:
                return out, "length"
            logits, _ = self.forward([t], cache)
