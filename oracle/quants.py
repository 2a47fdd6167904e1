"""TEST INFRASTRUCTURE ONLY -- ggml K-quant restatements for the parity tests.

Two independent restatements of llama.cpp's dequantize_row_q4_K / dequantize_row_q6_K
(EXT: ggml-quants.c, not vendored, version unpinned):
  * ``oracle/ggml_quants.c`` (C, -ffp-contract=off), loaded through ctypes, and
  * the numpy functions below (float32 arithmetic, one rounding per operation),
which must agree bit for bit; the HIP dequant kernel is then checked against them.

Also: seeded random Q4_K / Q6_K blocks (BASELINE.json config 5 "synthetic: random
Q4_K/Q6_K blocks, seed 2") and the Q4_K_M per-tensor type mix (EXT).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

QK_K = 256
Q4_K_BYTES = 144
Q6_K_BYTES = 210
GGML_TYPE_Q4_K = 12  # ggml type ids (EXT: ggml.h enum ggml_type)
GGML_TYPE_Q6_K = 14

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libggml_quants.so")


def c_lib():
    """ctypes handle on the C restatement (built by `make -C oracle`)."""
    if not os.path.exists(_LIB):
        raise RuntimeError(f"{_LIB} missing: run `make -C oracle`")
    lib = ctypes.CDLL(_LIB)
    for n in ("ms_dequantize_row_q4_K", "ms_dequantize_row_q6_K"):
        f = getattr(lib, n)
        f.restype = None
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    lib.ms_fp16_to_fp32.restype = ctypes.c_float
    lib.ms_fp16_to_fp32.argtypes = [ctypes.c_uint16]
    return lib


def c_dequant(blocks: np.ndarray, qtype: int) -> np.ndarray:
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    bs = Q4_K_BYTES if qtype == GGML_TYPE_Q4_K else Q6_K_BYTES
    nb = blocks.size // bs
    out = np.empty(nb * QK_K, np.float32)
    lib = c_lib()
    fn = lib.ms_dequantize_row_q4_K if qtype == GGML_TYPE_Q4_K else lib.ms_dequantize_row_q6_K
    fn(blocks.ctypes.data, out.ctypes.data, nb * QK_K)
    return out


def _f16(u16: np.ndarray) -> np.ndarray:
    return np.asarray(u16, dtype=np.uint16).view(np.float16).astype(np.float32)


def _scale_min_k4(sc: np.ndarray, j: int):
    """get_scale_min_k4 over a batch: sc [nb, 12] uint8 -> (scale, min) int [nb]."""
    sc = sc.astype(np.int32)
    if j < 4:
        return sc[:, j] & 63, sc[:, j + 4] & 63
    d = (sc[:, j + 4] & 0xF) | ((sc[:, j - 4] >> 6) << 4)
    m = (sc[:, j + 4] >> 4) | ((sc[:, j] >> 6) << 4)
    return d, m


def dequant_q4_K(blocks: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, Q4_K_BYTES)
    nb = b.shape[0]
    d = _f16(b[:, 0:2].copy().view(np.uint16)[:, 0])
    dmin = _f16(b[:, 2:4].copy().view(np.uint16)[:, 0])
    sc = b[:, 4:16]
    qs = b[:, 16:144].astype(np.int32)
    y = np.empty((nb, QK_K), np.float32)
    for c in range(4):  # 64-weight chunks
        s1, m1 = _scale_min_k4(sc, 2 * c)
        s2, m2 = _scale_min_k4(sc, 2 * c + 1)
        d1 = (d * s1.astype(np.float32)).astype(np.float32)
        mm1 = (dmin * m1.astype(np.float32)).astype(np.float32)
        d2 = (d * s2.astype(np.float32)).astype(np.float32)
        mm2 = (dmin * m2.astype(np.float32)).astype(np.float32)
        q = qs[:, 32 * c:32 * c + 32]
        lo = (q & 0xF).astype(np.float32)
        hi = (q >> 4).astype(np.float32)
        y[:, 64 * c:64 * c + 32] = (d1[:, None] * lo).astype(np.float32) - mm1[:, None]
        y[:, 64 * c + 32:64 * c + 64] = (d2[:, None] * hi).astype(np.float32) - mm2[:, None]
    return y.reshape(-1)


def dequant_q6_K(blocks: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, Q6_K_BYTES)
    nb = b.shape[0]
    ql = b[:, 0:128].astype(np.int32)
    qh = b[:, 128:192].astype(np.int32)
    sc = b[:, 192:208].view(np.int8).astype(np.float32)
    d = _f16(b[:, 208:210].copy().view(np.uint16)[:, 0])
    y = np.empty((nb, QK_K), np.float32)
    for n in range(2):  # 128-weight halves
        L = ql[:, 64 * n:64 * n + 64]
        H = qh[:, 32 * n:32 * n + 32]
        S = sc[:, 8 * n:8 * n + 8]
        for l0 in (0, 16):
            l = slice(l0, l0 + 16)
            is_ = l0 // 16
            q1 = (L[:, l] & 0xF) | (((H[:, l] >> 0) & 3) << 4)
            q2 = (L[:, l0 + 32:l0 + 48] & 0xF) | (((H[:, l] >> 2) & 3) << 4)
            q3 = (L[:, l] >> 4) | (((H[:, l] >> 4) & 3) << 4)
            q4 = (L[:, l0 + 32:l0 + 48] >> 4) | (((H[:, l] >> 6) & 3) << 4)
            base = 128 * n
            for k, (q, off) in enumerate(((q1, 0), (q2, 32), (q3, 64), (q4, 96))):
                ds = (d * S[:, is_ + 2 * k]).astype(np.float32)
                y[:, base + off + l0:base + off + l0 + 16] = (ds[:, None] * (q - 32).astype(np.float32)).astype(np.float32)
    return y.reshape(-1)


def dequant(blocks: np.ndarray, qtype: int) -> np.ndarray:
    return dequant_q4_K(blocks) if qtype == GGML_TYPE_Q4_K else dequant_q6_K(blocks)


def random_blocks(qtype: int, n_blocks: int, seed: int, scale: float = 0.02) -> np.ndarray:
    """Seeded random K-quant blocks whose dequantised weights have std ~``scale`` and mean
    ~0: uniform 6-bit scales/mins and quants, fp16 d ~ scale/270 with dmin = 7.5 d (Q4_K,
    centres d*s*q - dmin*m), d ~ scale/680 (Q6_K).  Returns uint8 [n_blocks, block_bytes]."""
    rng = np.random.default_rng(seed)
    if qtype == GGML_TYPE_Q4_K:
        b = rng.integers(0, 256, size=(n_blocks, Q4_K_BYTES), dtype=np.uint8)
        d = (rng.uniform(0.5, 1.5, n_blocks) * scale / 270).astype(np.float16)
        dmin = (d.astype(np.float32) * 7.5).astype(np.float16)
        b[:, 0:2] = d.view(np.uint8).reshape(-1, 2)
        b[:, 2:4] = dmin.view(np.uint8).reshape(-1, 2)
        return b
    b = rng.integers(0, 256, size=(n_blocks, Q6_K_BYTES), dtype=np.uint8)
    b[:, 192:208] = rng.integers(-64, 64, size=(n_blocks, 16), dtype=np.int8).view(np.uint8)
    d = (rng.uniform(0.5, 1.5, n_blocks) * scale / 680).astype(np.float16)
    b[:, 208:210] = d.view(np.uint8).reshape(-1, 2)
    return b


def q4_k_m_type(tensor: str, layer: int, n_layers: int) -> int:
    """Per-tensor type of a Q4_K_M file (EXT: llama.cpp llama_tensor_get_type; approximated:
    Q6_K for token_embd/output and for attn_v / ffn_down of the 'use_more_bits' layers)."""
    if tensor in ("embed", "lm_head"):
        return GGML_TYPE_Q6_K
    if tensor in ("wv", "w_down"):
        more = layer < n_layers // 8 or layer >= 7 * n_layers // 8 or (layer - n_layers // 8) % 3 == 2
        return GGML_TYPE_Q6_K if more else GGML_TYPE_Q4_K
    return GGML_TYPE_Q4_K
