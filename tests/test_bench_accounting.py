"""bench.py's algorithmic work figures against SURVEY.md §8d (the roofline numerators)."""
import importlib.util
import os

from mapsum.config import LLAMA32_3B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(bench)


def test_prefill_flops_match_survey():
    # §8d: 1.1546e13 (linear) + 7.22e11 (attention) + lm_head on the last token ~= 1.2268e13
    f = bench.prefill_flops_per_chunk(LLAMA32_3B, 2048)
    assert abs(f - 1.2268e13) / 1.2268e13 < 1e-3


def test_decode_weight_bytes_match_survey():
    # §8d: W = 6,425,149,440 B of bf16 weights per decode step incl. the tied lm_head
    cfg, B = LLAMA32_3B, 8
    act = bench.gemv_bytes_per_step(cfg, B) - bench.gemv_bytes_per_step(cfg, 0)
    w = bench.gemv_bytes_per_step(cfg, 0) + cfg.vocab * cfg.hidden * 2
    assert w == 6_425_149_440
    assert 0 < act < 1e-2 * w  # activations are ~0.4 % of the weight stream at B = 8
    lm = bench.lm_head_bytes_per_step(cfg, B)
    assert lm == cfg.vocab * cfg.hidden * 2 + 2 * B * cfg.hidden + 4 * B * cfg.vocab


def test_q4_k_m_bytes_between_4_5_and_6_6_bits():
    cfg = LLAMA32_3B
    q = bench.qgemv_bytes_per_step(cfg, 0)
    n = bench.gemv_bytes_per_step(cfg, 0) / 2  # weights
    assert 144 / 256 <= q / n <= 224 / 256
