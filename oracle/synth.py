"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the engine's synthetic weights.

The engine generates synthetic Llama weights on the device (``ms_init_synthetic``,
csrc/k_misc.hip ``synth_weight_kernel``) so that a 6.4 GB random-init model needs
no host->device copy.  This file restates the same counter-based generator so the
oracle can rebuild bit-identical bf16 weights for small configs.

Generator (integer-only up to one fp32 multiply, so host and device agree bit for bit):
    key  = kind<<58 | layer<<50 | row<<20 | col
    h    = splitmix64(key ^ splitmix64(seed))
    s    = sum of the four 16-bit limbs of h                  (Irwin-Hall(4), mean 131070)
    w    = bf16_rne( float32(s - 131070) * float32(std*sqrt(3)/65536) )     linear weights
    g    = bf16_rne( 1 + float32(s - 131070) * float32(jitter/131070) )     norm weights
The sum of four uniforms has the variance of ``std**2`` (N(0, 0.02)
weights, RMSNorm weights 1; ``jitter`` > 0 only in tests so a norm bug is visible).
"""
from __future__ import annotations

import numpy as np

EMBED, ATTN_NORM, WQ, WK, WV, WO, FFN_NORM, WGATE, WUP, WDOWN, FINAL_NORM, LM_HEAD = range(12)

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def bf16_rne(x: np.ndarray) -> np.ndarray:
    """float32 -> nearest-even bf16, returned as float32 holding the bf16 value."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) & np.uint32(0xFFFF0000)
    return r.view(np.float32)


def to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """float32 (already bf16-valued) -> uint16 bit pattern."""
    return (np.ascontiguousarray(x, dtype=np.float32).view(np.uint32) >> np.uint32(16)).astype(np.uint16)


def from_bf16_bits(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def _limb_sum(seed: int, kind: int, layer: int, rows: int, cols: int, row0: int = 0) -> np.ndarray:
    r = np.arange(row0, row0 + rows, dtype=np.uint64)[:, None]
    c = np.arange(cols, dtype=np.uint64)[None, :]
    key = (np.uint64(kind) << np.uint64(58)) | (np.uint64(layer) << np.uint64(50)) | (r << np.uint64(20)) | c
    h = splitmix64(key ^ splitmix64(np.uint64(seed)))
    m = np.uint64(0xFFFF)
    s = (h & m) + ((h >> np.uint64(16)) & m) + ((h >> np.uint64(32)) & m) + ((h >> np.uint64(48)) & m)
    return s.astype(np.int64) - 131070


def linear(seed: int, kind: int, layer: int, rows: int, cols: int, std: float) -> np.ndarray:
    scale = np.float32(std * np.sqrt(3.0) / 65536.0)
    out = np.empty((rows, cols), np.float32)
    step = max(1, (1 << 22) // cols)  # row blocks: uint64 temporaries stay ~32 MB each
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        v = _limb_sum(seed, kind, layer, r1 - r0, cols, row0=r0).astype(np.float32) * scale
        out[r0:r1] = bf16_rne(v)
    return out


def norm(seed: int, kind: int, layer: int, n: int, jitter: float) -> np.ndarray:
    scale = np.float32(jitter / 131070.0)
    v = _limb_sum(seed, kind, layer, 1, n)[0].astype(np.float32) * scale
    return bf16_rne(np.float32(1.0) + v)


def make_weights(cfg, seed: int, std: float = 0.02, jitter: float = 0.0) -> dict:
    """Logical (unfused) weights, float32 arrays holding bf16 values.

    Layout follows HF ``nn.Linear`` ([out, in]); the engine fuses Q|K|V and
    interleaves gate/up at 16-row granularity on upload (see mapsum/weights.py)."""
    H, D = cfg.hidden, cfg.head_dim
    w = {"embed": linear(seed, EMBED, 0, cfg.vocab, H, std),
         "final_norm": norm(seed, FINAL_NORM, 0, H, jitter), "layers": []}
    for l in range(cfg.n_layers):
        w["layers"].append({
            "attn_norm": norm(seed, ATTN_NORM, l, H, jitter),
            "wq": linear(seed, WQ, l, cfg.n_heads * D, H, std),
            "wk": linear(seed, WK, l, cfg.n_kv_heads * D, H, std),
            "wv": linear(seed, WV, l, cfg.n_kv_heads * D, H, std),
            "wo": linear(seed, WO, l, H, cfg.n_heads * D, std),
            "ffn_norm": norm(seed, FFN_NORM, l, H, jitter),
            "w_gate": linear(seed, WGATE, l, cfg.ffn, H, std),
            "w_up": linear(seed, WUP, l, cfg.ffn, H, std),
            "w_down": linear(seed, WDOWN, l, H, cfg.ffn, std),
        })
    w["lm_head"] = w["embed"] if cfg.tie_embeddings else linear(seed, LM_HEAD, 0, cfg.vocab, H, std)
    return w


def f16_rne(x: np.ndarray) -> np.ndarray:
    """float32 -> nearest-even IEEE fp16 (the engine's 16-bit type), returned as float32."""
    return np.asarray(x, dtype=np.float32).astype(np.float16).astype(np.float32)
