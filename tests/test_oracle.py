"""CPU tests: the oracle pinned against its golden vectors (no GPU).

tests/golden/hf_tiny_llama.npz holds transformers.LlamaForCausalLM outputs on the
oracle's own seeded weights (tests/golden/make_golden.py).  In fp32 mode the oracle
must reproduce them to fp32 round-off; in its bf16-rounding mode (the engine's
numerics contract) within the north-star tolerance.
"""
import os

import numpy as np
import pytest

from mapsum.config import LLAMA32_3B, TINY
from oracle import synth
from oracle.llama_ref import OracleLlama, rope_inv_freq

GOLD = os.path.join(os.path.dirname(__file__), "golden", "hf_tiny_llama.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


@pytest.fixture(scope="module")
def weights(gold):
    return synth.make_weights(TINY, int(gold["seed"]), std=float(gold["std"]), jitter=float(gold["jitter"]))


def test_oracle_fp32_matches_transformers(gold, weights):
    o = OracleLlama(TINY, weights, mode="fp32")
    ids = gold["ids"]
    lg, probes = o.forward(ids, collect=True, all_logits=True)
    top_idx, top_val = gold["top16_idx"], gold["top16_val"]
    mine = np.take_along_axis(lg, top_idx, 1)
    assert np.allclose(mine, top_val, rtol=1e-4, atol=1e-4)
    assert np.array_equal(np.argmax(lg, 1), top_idx[:, 0])
    assert np.allclose(lg[-1], gold["last_logits"], rtol=1e-4, atol=1e-4)
    for l in range(TINY.n_layers):
        assert np.allclose(probes[l][:, :32], gold["hidden_head"][l], rtol=1e-4, atol=1e-4)
        assert np.allclose(np.linalg.norm(probes[l], axis=1), gold["hidden_norm"][l], rtol=1e-5)


def test_oracle_fp32_greedy_matches_transformers(gold, weights):
    o = OracleLlama(TINY, weights, mode="fp32")
    toks, fin = o.generate(gold["ids"], len(gold["greedy"]), ignore_eos=True)
    assert toks == gold["greedy"].tolist() and fin == "length"


@pytest.mark.parametrize("mode,tol", [("engine", 2e-3), ("f16", 2e-3), ("bf16", 2e-2)])
def test_oracle_rounded_modes_within_tolerance(gold, weights, mode, tol):
    """The fp16 rounding points the HIP path implements ("engine") and ggml's F16 graph stay
    within 2e-3 of fp32 Llama on TINY; the round-3 bf16 contract within 2e-2."""
    o = OracleLlama(TINY, weights, mode=mode)
    lg, _ = o.forward(gold["ids"])
    ref = gold["last_logits"]
    err = np.linalg.norm(lg - ref) / np.linalg.norm(ref)
    print(f"{mode}: last-token logits rel err vs transformers fp32 {err:.2e}")
    assert err < tol


def test_llama3_rope_frequencies():
    """Llama-3.2 rope_scaling: factor 32, low/high 1/4, original ctx 8192 (EXT config)."""
    inv = rope_inv_freq(LLAMA32_3B)
    base = 1.0 / (500000.0 ** (np.arange(0, 128, 2) / 128))
    wl = 2 * np.pi / base
    assert np.allclose(inv[wl < 2048], base[wl < 2048])          # high-frequency: untouched
    assert np.allclose(inv[wl > 8192], base[wl > 8192] / 32.0)   # low-frequency: / factor
    mid = (wl >= 2048) & (wl <= 8192)
    assert np.all((inv[mid] <= base[mid]) & (inv[mid] >= base[mid] / 32.0))


def test_synth_generator_known_answers():
    """Pins the counter-based generator the engine restates on the device."""
    assert int(synth.splitmix64(np.uint64(0))) == 0xE220A8397B1DCDAF  # published splitmix64(0)
    w = synth.linear(0, synth.WQ, 3, 4, 8, 0.02)
    assert w.dtype == np.float32 and w.shape == (4, 8)
    assert np.array_equal(synth.bf16_rne(w), w)                  # already bf16 values
    big = synth.linear(1, synth.EMBED, 0, 256, 256, 0.02)
    assert abs(float(big.std()) - 0.02) < 0.001 and abs(float(big.mean())) < 0.001
    g = synth.norm(1, synth.ATTN_NORM, 0, 1024, 0.0)
    assert np.all(g == 1.0)


def test_bf16_rounding_is_nearest_even():
    x = np.array([1.0, 1.00390625, 1.01171875, -2.5, 3.0e38], np.float32)
    r = synth.bf16_rne(x)
    assert r.tolist()[:4] == [1.0, 1.0, 1.015625, -2.5]
    bits = synth.to_bf16_bits(r)
    assert np.array_equal(synth.from_bf16_bits(bits), r)


def test_torch_cpu_baseline_is_the_same_model():
    """bench.py's cpu_baseline (oracle/torch_cpu.py) runs the engine's own synthetic weights:
    the torch generator is bit-exact with oracle/synth.py, and on TINY its last-position logits
    follow the numpy oracle's (bf16 torch arithmetic vs the oracle's rounding points)."""
    import torch
    from mapsum.config import TINY
    from oracle import synth as S
    from oracle.llama_ref import OracleLlama
    from oracle.torch_cpu import TorchCpuLlama, synth_linear
    assert np.array_equal(synth_linear(5, S.WUP, 1, 64, 768, 0.05).float().numpy(), S.linear(5, S.WUP, 1, 64, 768, 0.05))
    seed, std, jit = 3, 0.05, 0.1
    m = TorchCpuLlama(TINY, seed=seed, std=std, jitter=jit)
    o = OracleLlama(TINY, S.make_weights(TINY, seed, std=std, jitter=jit))
    ids = np.random.default_rng(1).integers(0, 4000, size=80)
    cache = m.new_cache(96)
    m.forward(torch.as_tensor(ids), cache, 0)
    ref, _ = o.forward(ids)
    got = m.last_logits.numpy()
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 3e-2
    # the decode path (one new token over the grouped-query KV cache) continues the prefill
    cache = m.new_cache(96)
    m.forward(torch.as_tensor(ids[:-1]), cache, 0)
    m.forward(torch.as_tensor(ids[-1:]), cache, len(ids) - 1)
    dec = m.last_logits.numpy()
    assert np.linalg.norm(dec - got) / np.linalg.norm(got) < 3e-2
