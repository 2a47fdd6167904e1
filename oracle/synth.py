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


# ----------------------------------------------------------------- synthetic K-quant blocks
# Restates csrc/k_qgemv.hip synth_qblocks_kernel and engine.cpp ms_init_synthetic_q (the
# configs[4] bench weights, seed 2): block i of a tensor = the bytes of successive splitmix64
# states h_{j+1} = smix(h_j), h_0 = smix(i ^ smix(seed ^ tensor << 56 ^ layer << 48)), little
# endian, 8 per state; then u = 0.5 + (smix(h_last) >> 40) 2^-24 and the fp16 scale fields
# (Q4_K: d = f16(u scale / 270), dmin = f16(d 7.5); Q6_K: the 16 int8 scales folded into
# [-64, 63], d = f16(u scale / 680)).
Q4_K, Q6_K = 12, 14
_QBYTES = {Q4_K: 144, Q6_K: 210}


def synth_qblocks(qtype: int, n_blocks: int, seed: int, tensor: int, layer: int, scale: float = 0.02) -> np.ndarray:
    """uint8 [n_blocks, block_bytes]: the device generator's blocks of one tensor, bit for bit."""
    braw = _QBYTES[qtype]
    seed_h = splitmix64(np.uint64((seed ^ (tensor << 56) ^ (layer << 48)) & 0xFFFFFFFFFFFFFFFF))
    out = np.empty((n_blocks, braw), np.uint8)
    step = 1 << 20
    for b0 in range(0, n_blocks, step):
        b1 = min(n_blocks, b0 + step)
        h = splitmix64(np.arange(b0, b1, dtype=np.uint64) ^ seed_h)
        for k in range(0, braw, 8):
            h = splitmix64(h)
            nb = min(8, braw - k)
            out[b0:b1, k:k + nb] = h.view(np.uint8).reshape(-1, 8)[:, :nb]
        u = np.float32(0.5) + (splitmix64(h) >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        blk = out[b0:b1]
        if qtype == Q4_K:
            d = ((u * np.float32(scale)) / np.float32(270.0)).astype(np.float16)
            dm = (d.astype(np.float32) * np.float32(7.5)).astype(np.float16)
            blk[:, 0:2] = d.view(np.uint8).reshape(-1, 2)
            blk[:, 2:4] = dm.view(np.uint8).reshape(-1, 2)
        else:
            blk[:, 192:208] = ((blk[:, 192:208].astype(np.int32) & 0x7F) - 64).astype(np.int8).view(np.uint8)
            d = ((u * np.float32(scale)) / np.float32(680.0)).astype(np.float16)
            blk[:, 208:210] = d.view(np.uint8).reshape(-1, 2)
    return out


def make_q4km_blocks(cfg, seed: int = 2, scale: float = 0.02) -> dict:
    """{name or (layer, name): (ggml type, blocks)} of ms_init_synthetic_q's Q4_K_M model
    (tied embedding = lm_head; per-tensor mix oracle/quants.py q4_k_m_type)."""
    from oracle.quants import q4_k_m_type
    H, D = cfg.hidden, cfg.head_dim
    shapes = {"wq": (WQ, cfg.n_heads * D, H), "wk": (WK, cfg.n_kv_heads * D, H), "wv": (WV, cfg.n_kv_heads * D, H),
              "wo": (WO, H, cfg.n_heads * D), "w_gate": (WGATE, cfg.ffn, H), "w_up": (WUP, cfg.ffn, H),
              "w_down": (WDOWN, H, cfg.ffn)}
    qt = q4_k_m_type("embed", 0, cfg.n_layers)
    qw = {"embed": (qt, synth_qblocks(qt, cfg.vocab * H // 256, seed, EMBED, 0, scale))}
    for l in range(cfg.n_layers):
        for name, (kind, r, c) in shapes.items():
            qt = q4_k_m_type(name, l, cfg.n_layers)
            qw[(l, name)] = (qt, synth_qblocks(qt, r * c // 256, seed, kind, l, scale))
    return qw


def q4km_weights(cfg, qw: dict, seed: int = 2, jitter: float = 0.0, dequant=None) -> dict:
    """Logical float32 weights of a Q4_K_M block set: the EXACT fp32 dequantisation (ggml's
    dequantize_row_*, oracle/ggml_quants.c) -- not rounded to fp16."""
    if dequant is None:
        from oracle.quants import c_dequant as dequant
    H = cfg.hidden
    qt, eb = qw["embed"]
    w = {"embed": dequant(eb, qt).reshape(cfg.vocab, H), "final_norm": norm(seed, FINAL_NORM, 0, H, jitter),
         "layers": []}
    w["lm_head"] = w["embed"]
    for l in range(cfg.n_layers):
        ly = {"attn_norm": norm(seed, ATTN_NORM, l, H, jitter), "ffn_norm": norm(seed, FFN_NORM, l, H, jitter)}
        for name in ("wq", "wk", "wv", "wo", "w_gate", "w_up", "w_down"):
            qt, b = qw[(l, name)]
            r = {"wo": H, "w_down": H}.get(name)
            ly[name] = dequant(b, qt).reshape(r if r else -1, -1 if r else H)
        w["layers"].append(ly)
    return w
