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

Rounding points (the engine's numerics contract; mode "engine"):
  weights fp16; residual stream fp32; every GEMM input fp16, fp32 accumulate; a normalised
  projection (QKV, gate/up, lm_head) multiplies f16(x * g) by W and scales each output row by
  the RMSNorm factor r = 1/sqrt(mean(x^2) + eps) in fp32 -- r * (f16(x*g) . W^T), the deferred
  form of W . (x*r*g), so the producer of x can emit the GEMM input without knowing the row's
  norm; Q/K/V, RoPE output, attention output and the SwiGLU product rounded to fp16; attention
  scores/softmax fp32 with the probabilities rounded to fp16 for P.V; logits fp32; argmax
  ties -> lowest id.  The flash kernels' online softmax takes each row's max per tile (and the
  decode split combine per split), so their P rounding is not bit-identical to this one-pass
  softmax; the tests' tolerances cover that.
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


def _f16(x):
    """float32 -> nearest-even fp16 (subnormals included), returned as float32."""
    return np.asarray(x, dtype=np.float32).astype(np.float16).astype(np.float32)


def _f16_weights(w: dict) -> dict:
    """The F16 GGUF of a model: matrices rounded to fp16, norm weights kept fp32 (as
    llama.cpp's converter stores 1-D tensors)."""
    out = {k: v for k, v in w.items() if k != "layers"}
    for k in ("embed", "lm_head"):
        out[k] = _f16(w[k])
    if w["lm_head"] is w["embed"]:
        out["lm_head"] = out["embed"]
    out["layers"] = [{k: (v if k.endswith("norm") else _f16(v)) for k, v in L.items()}
                     for L in w["layers"]]
    return out


def rms_rinv_f64(x: np.ndarray, eps: float) -> np.ndarray:
    """ggml_compute_forward_rms_norm_f32: sum of squares in double, scale = 1/sqrtf(mean + eps)."""
    ms = (np.sum(x.astype(np.float64) ** 2, axis=-1, keepdims=True) / x.shape[-1]).astype(np.float32)
    return (np.float32(1.0) / np.sqrt(ms + np.float32(eps))).astype(np.float32)


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

    MODES = ("engine", "bf16", "fp32", "f16")

    def __init__(self, cfg, weights: dict, mode: str = "engine"):
        """Numerics mode:

        * ``"engine"`` (default) -- the HIP engine's fp16 contract (module docstring, DESIGN.md
          §2): weights held as fp16 (exact for bf16-valued weights), the rounding points below
          with fp16 RNE, and P rounded to fp16 before P.V as the flash kernels do (unnormalised
          p = exp(s - max) rounded, the row sum taken in fp32 before rounding);
        * ``"bf16"`` -- the round-3 contract: the same points with bf16 rounding and exact P
          (kept to show why the engine moved to fp16: tools/parity_modes_cpu.py);
        * ``"fp32"`` -- every activation rounding off: un-rounded Llama,
          the mode pinned against transformers.LlamaForCausalLM;
        * ``"f16"`` -- ggml's CPU graph for an F16 GGUF, the arithmetic Ollama runs for
          ``llama3.2:3b-instruct-fp16`` (EXT llama.cpp ``llm_build_llama`` without flash
          attention, F16 KV cache): weights rounded to fp16 (what the GGUF holds), RMSNorm
          applied in fp32 before the matmul and its output rounded to fp16 (ggml converts
          every F32 ``src1`` to the F16 weight's vec_dot type), K and V rounded to fp16 when
          written to the cache, Q rounded to fp16 for K.Q, the softmax probabilities rounded
          to fp16 for V.P, the attention output and SwiGLU product rounded to fp16 at their
          matmuls; fp32 accumulation, fp32 residual, RMSNorm sum of squares in double."""
        self.cfg = cfg
        self.mode = mode
        assert self.mode in self.MODES, self.mode
        if self.mode in ("f16", "engine"):
            weights = _f16_weights(weights)
        self.w = weights
        self.rnd = {"engine": _f16, "bf16": bf16_rne, "fp32": _f32, "f16": _f16}[self.mode]

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
        f16 = self.mode == "f16"
        eps = cfg.norm_eps

        def normed(x, g):
            """(GEMM input, per-row factor applied after the GEMM)."""
            if f16:  # ggml: rms_norm then mul by g in fp32, the matmul rounds its input
                return _f16((x * rms_rinv_f64(x, eps)) * g), np.float32(1.0)
            if self.mode == "engine":  # kernels.h kXgScale: f16(x g 2^-4), 16 r -- exact scalings
                return rnd((x * g).astype(np.float32) * np.float32(0.0625)), rms_rinv(x, eps) * np.float32(16.0)
            return norm_input(x, g, rnd), rms_rinv(x, eps)

        pre = _f32 if f16 else rnd  # Q/K/V before RoPE: ggml keeps them fp32
        x = w["embed"][ids].astype(np.float32)
        probes = []
        for l, L in enumerate(w["layers"]):
            xg, r = normed(x, L["attn_norm"])
            q = pre(r * (xg @ L["wq"].T)).reshape(T, Hq, D)
            k = pre(r * (xg @ L["wk"].T)).reshape(T, Hk, D)
            v = rnd(r * (xg @ L["wv"].T)).reshape(T, Hk, D)
            q = apply_rope(q, cos, sin, rnd)  # f16: Q rounded for K.Q, K for the F16 cache
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
            den = p.sum(axis=-1, keepdims=True)
            if self.mode == "engine":  # flash kernels: fp16(p) . V, then / the fp32 row sum
                pv = np.matmul(_f16(p), vq.transpose(1, 0, 2)) / den
            else:
                p = p / den
                if f16:  # V.P: ggml rounds the fp32 probabilities to the F16 V's vec_dot type
                    p = _f16(p)
                pv = np.matmul(p.astype(np.float32), vq.transpose(1, 0, 2))
            o = rnd(pv.transpose(1, 0, 2))  # [T, Hq, D]
            x = x + o.reshape(T, Hq * D) @ L["wo"].T
            xg, r = normed(x, L["ffn_norm"])
            g = r * (xg @ L["w_gate"].T)
            u = r * (xg @ L["w_up"].T)
            h = rnd(silu(g) * u)
            x = x + h @ L["w_down"].T
            if collect:
                probes.append(x.copy())
        cache["len"] = p0 + T
        xs = x if all_logits else x[-1:]
        xg, r = normed(xs, w["final_norm"])
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
