"""CPU tests: the K-quant dequant oracle.

The C restatement (oracle/ggml_quants.c) and the numpy restatement (oracle/quants.py)
must agree bit for bit, and both must reproduce hand-computed known answers for blocks
built field by field from the published Q4_K / Q6_K layouts (llama.cpp is not available
here, so these KATs -- not llama.cpp dumps -- pin the format).
"""
import subprocess

import numpy as np
import pytest

from oracle import quants as Q

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", f"{ROOT}/oracle"], check=True)


def f16bits(x):
    return int(np.array([x], np.float16).view(np.uint16)[0])


def q4k_block(d, dmin, sc, mn, qs):
    """Pack one Q4_K block: sc/mn = 8 six-bit (scale, min) pairs, qs = 128 bytes."""
    b = np.zeros(144, np.uint8)
    b[0:2] = np.array([d], np.uint16).view(np.uint8)
    b[2:4] = np.array([dmin], np.uint16).view(np.uint8)
    s = np.zeros(12, np.int64)
    for j in range(4):
        s[j] = (sc[j] & 63) | ((sc[j + 4] >> 4) << 6)
        s[j + 4] = (mn[j] & 63) | ((mn[j + 4] >> 4) << 6)
        s[j + 8] = (sc[j + 4] & 15) | ((mn[j + 4] & 15) << 4)
    b[4:16] = s.astype(np.uint8)
    b[16:144] = qs
    return b


def test_q4k_known_answers():
    sc = [5, 7, 63, 0, 33, 17, 48, 1]
    mn = [3, 0, 63, 12, 20, 63, 0, 9]
    qs = np.zeros(128, np.uint8)
    qs[0] = 0x2F          # weight 0 -> low nibble 15, weight 32 -> high nibble 2
    qs[32 * 2 + 5] = 0xF0  # chunk 2: weight 128+5 -> 0, weight 128+32+5 -> 15
    b = q4k_block(f16bits(1.0), f16bits(0.5), sc, mn, qs)
    y_c = Q.c_dequant(b, Q.GGML_TYPE_Q4_K)
    y_n = Q.dequant_q4_K(b)
    assert np.array_equal(y_c.view(np.uint32), y_n.view(np.uint32))
    assert y_c[0] == 1.0 * 5 * 15 - 0.5 * 3        # sub-block 0
    assert y_c[32] == 1.0 * 7 * 2 - 0.5 * 0        # sub-block 1 (high nibbles of chunk 0)
    assert y_c[1] == -0.5 * 3                      # q = 0
    assert y_c[128 + 5] == 33 * 0 - 0.5 * 20       # sub-block 4: scale/min from the packed j>=4 form
    assert y_c[128 + 32 + 5] == 17 * 15 - 0.5 * 63  # sub-block 5
    assert y_c[255] == 1 * 0 - 0.5 * 9             # sub-block 7


def test_q6k_known_answers():
    b = np.zeros(210, np.uint8)
    b[208:210] = np.array([f16bits(0.25)], np.uint16).view(np.uint8)
    sc = np.array([2, -3, 4, 5, -6, 7, 8, -9, 10, 11, 12, 13, 14, 15, 16, -128], np.int8)
    b[192:208] = sc.view(np.uint8)
    b[0] = 0x21            # ql[0]: low 1 (weight 0), high 2 (weight 64)
    b[128] = 0b11100100    # qh[0]: bits for weights 0 / 32 / 64 / 96
    b[32] = 0x0F           # ql[32]: weight 32 low 15, weight 96 high 0
    y_c = Q.c_dequant(b, Q.GGML_TYPE_Q6_K)
    y_n = Q.dequant_q6_K(b)
    assert np.array_equal(y_c.view(np.uint32), y_n.view(np.uint32))
    assert y_c[0] == 0.25 * 2 * ((1 | (0 << 4)) - 32)
    assert y_c[32] == 0.25 * 4 * ((15 | (1 << 4)) - 32)
    assert y_c[64] == 0.25 * -6 * ((2 | (2 << 4)) - 32)
    assert y_c[96] == 0.25 * 8 * ((0 | (3 << 4)) - 32)
    assert y_c[16] == 0.25 * -3 * (0 - 32)   # is = 1 for l >= 16
    assert y_c[128 + 127] == 0.25 * -128 * (0 - 32)  # last sub-block, scale -128


@pytest.mark.parametrize("qtype", [Q.GGML_TYPE_Q4_K, Q.GGML_TYPE_Q6_K])
def test_c_and_numpy_agree_bitwise_random(qtype):
    b = Q.random_blocks(qtype, 300, seed=2)
    # edge cases: subnormal / zero / negative scales in the first blocks
    if qtype == Q.GGML_TYPE_Q4_K:
        b[0, 0:2] = [0x01, 0x00]   # d = smallest subnormal
        b[1, 2:4] = [0x00, 0x80]   # dmin = -0
        b[2, 4:16] = 0xFF          # every 6-bit scale/min = 63
        b[3, 16:] = 0xFF           # all nibbles 15
    else:
        b[0, 208:210] = [0x01, 0x00]
        b[1, 192:208] = 0x80       # scales = -128
    y_c = Q.c_dequant(b, qtype)
    y_n = Q.dequant(b, qtype)
    assert np.array_equal(y_c.view(np.uint32), y_n.view(np.uint32))
    assert np.all(np.isfinite(y_c))


def test_random_blocks_statistics_and_mix():
    for qt in (Q.GGML_TYPE_Q4_K, Q.GGML_TYPE_Q6_K):
        y = Q.dequant(Q.random_blocks(qt, 256, seed=2, scale=0.02), qt)
        assert 0.012 < float(y.std()) < 0.03 and abs(float(y.mean())) < 0.002
    types = [Q.q4_k_m_type("wv", i, 28) for i in range(28)]
    assert types.count(Q.GGML_TYPE_Q6_K) >= 8 and types.count(Q.GGML_TYPE_Q4_K) >= 8
    assert Q.q4_k_m_type("embed", 0, 28) == Q.GGML_TYPE_Q6_K


@pytest.mark.parametrize("qtype,tol", [(Q.GGML_TYPE_Q4_K, 0.10), (Q.GGML_TYPE_Q6_K, 0.03)])
def test_quantizer_writes_blocks_the_dequantiser_reads(qtype, tol):
    """oracle/quantize.py (the K-quant fixtures' writer): its blocks dequantise (ggml's C
    restatement) back to the input within the format's error, and re-quantising the
    dequantised weights reproduces them (a fixed point of quantize o dequant)."""
    from oracle.quantize import quantize
    x = np.random.default_rng(3).standard_normal(64 * 256).astype(np.float32) * 0.02
    b = quantize(x, qtype)
    y = Q.c_dequant(b, qtype)
    assert np.array_equal(y, Q.dequant(b, qtype))
    assert np.linalg.norm(y - x) / np.linalg.norm(x) < tol
    y2 = Q.c_dequant(quantize(y, qtype), qtype)
    assert np.linalg.norm(y2 - y) / np.linalg.norm(y) < tol / 4
