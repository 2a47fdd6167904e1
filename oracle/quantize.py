"""TEST INFRASTRUCTURE ONLY -- float -> ggml Q4_K / Q6_K blocks (numpy).

The Q4_K_M parity fixtures need K-quant weights with a prescribed structure (the copy head of
tests/golden/sharp_model.py): those are quantised here and then, like every other K-quant weight
of the tests, DEQUANTISED exactly (oracle/quants.py, oracle/ggml_quants.c) for the oracle, while
the engine runs the blocks through its dequant-fused GEMVs.  So this quantiser only has to write
VALID blocks of the layouts ggml's dequantize_row_q4_K / dequantize_row_q6_K read (restated in
oracle/quants.py, which the round trip test pins); it is a plain min/max quantiser, not
llama.cpp's error-minimising search (EXT quantize_row_q4_K_ref): the engine is checked against
the dequantisation of these exact bytes, whichever bytes they are.
"""
from __future__ import annotations

import numpy as np

from oracle.quants import GGML_TYPE_Q4_K, GGML_TYPE_Q6_K, Q4_K_BYTES, Q6_K_BYTES, QK_K


def quantize_q4_K(x: np.ndarray) -> np.ndarray:
    """x float [n * 256] -> uint8 [n, 144]: 8 sub-blocks of 32, value = d*s_j*q - dmin*m_j."""
    x = np.asarray(x, np.float32).reshape(-1, 8, 32)
    n = x.shape[0]
    mn = np.maximum(-x.min(axis=2), 0.0)                     # m_j * dmin (>= 0)
    rng = x.max(axis=2) + mn                                 # span above -mn
    scf = rng / 15.0                                         # d * s_j
    d = (scf.max(axis=1) / 63.0).astype(np.float16)
    dmin = (mn.max(axis=1) / 63.0).astype(np.float16)
    d32, dm32 = d.astype(np.float32), dmin.astype(np.float32)
    s = np.where(d32[:, None] > 0, np.rint(scf / np.where(d32 > 0, d32, 1)[:, None]), 0).clip(0, 63).astype(np.int32)
    m = np.where(dm32[:, None] > 0, np.rint(mn / np.where(dm32 > 0, dm32, 1)[:, None]), 0).clip(0, 63).astype(np.int32)
    ds = d32[:, None] * s
    q = np.where(ds[:, :, None] > 0,
                 np.rint((x + (dm32[:, None] * m)[:, :, None]) / np.where(ds > 0, ds, 1)[:, :, None]), 0)
    q = q.clip(0, 15).astype(np.uint8)
    b = np.zeros((n, Q4_K_BYTES), np.uint8)
    b[:, 0:2] = d.view(np.uint8).reshape(-1, 2)
    b[:, 2:4] = dmin.view(np.uint8).reshape(-1, 2)
    sc = np.zeros((n, 12), np.int32)  # get_scale_min_k4's packing
    for j in range(4):
        sc[:, j] = s[:, j] | ((s[:, j + 4] >> 4) << 6)
        sc[:, j + 4] = m[:, j] | ((m[:, j + 4] >> 4) << 6)
        sc[:, j + 8] = (s[:, j + 4] & 0xF) | ((m[:, j + 4] & 0xF) << 4)
    b[:, 4:16] = sc.astype(np.uint8)
    for c in range(4):  # 64-weight chunk c: low nibbles sub-block 2c, high nibbles 2c + 1
        b[:, 16 + 32 * c:16 + 32 * c + 32] = q[:, 2 * c] | (q[:, 2 * c + 1] << 4)
    return b


def quantize_q6_K(x: np.ndarray) -> np.ndarray:
    """x float [n * 256] -> uint8 [n, 210]: 16 sub-blocks of 16, value = d*s_j*(q - 32)."""
    x = np.asarray(x, np.float32).reshape(-1, 16, 16)
    n = x.shape[0]
    amax = np.abs(x).max(axis=2)
    scf = amax / 31.0                                        # d * s_j
    d = (scf.max(axis=1) / 127.0).astype(np.float16)
    d32 = d.astype(np.float32)
    s = np.where(d32[:, None] > 0, np.rint(scf / np.where(d32 > 0, d32, 1)[:, None]), 0).clip(-128, 127).astype(np.int32)
    ds = d32[:, None] * s
    q = np.where(ds[:, :, None] != 0, np.rint(x / np.where(ds != 0, ds, 1)[:, :, None]), 0) + 32
    q = q.clip(0, 63).astype(np.int32).reshape(n, QK_K)
    b = np.zeros((n, Q6_K_BYTES), np.uint8)
    for h in range(2):  # 128-weight halves (dequant_q6_K's n)
        qa, qb, qc, qd = (q[:, 128 * h + 32 * k:128 * h + 32 * k + 32] for k in range(4))
        b[:, 64 * h:64 * h + 32] = ((qa & 0xF) | ((qc & 0xF) << 4)).astype(np.uint8)
        b[:, 64 * h + 32:64 * h + 64] = ((qb & 0xF) | ((qd & 0xF) << 4)).astype(np.uint8)
        b[:, 128 + 32 * h:128 + 32 * h + 32] = ((qa >> 4) | ((qb >> 4) << 2) | ((qc >> 4) << 4)
                                                | ((qd >> 4) << 6)).astype(np.uint8)
    b[:, 192:208] = s.astype(np.int8).view(np.uint8)
    b[:, 208:210] = d.view(np.uint8).reshape(-1, 2)
    return b


def quantize(x: np.ndarray, qtype: int, chunk: int = 1 << 20) -> np.ndarray:
    """Row-major float weights (K % 256 == 0) -> blocks, in pieces of `chunk` blocks (memory)."""
    f = quantize_q4_K if qtype == GGML_TYPE_Q4_K else quantize_q6_K
    flat = np.asarray(x, np.float32).reshape(-1, QK_K)
    return np.concatenate([f(flat[i:i + chunk]) for i in range(0, flat.shape[0], chunk)])


__all__ = ["quantize_q4_K", "quantize_q6_K", "quantize", "GGML_TYPE_Q4_K", "GGML_TYPE_Q6_K"]
