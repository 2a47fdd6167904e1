"""The committed 28-layer fixtures (tests/golden/make_fullshape_golden.py) are what they claim
to be -- CPU only; the GPU comparison is tests/test_gpu_golden28.py."""
import importlib.util
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(HERE), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


FIXTURES = [("flat", "fp32"), ("flat", "f16"), ("flat", "engine"), ("sharp", "fp32"), ("sharp", "engine"),
            ("q4km", "fp32")]


@pytest.mark.parametrize("which,mode", FIXTURES)
def test_fixture_layout_and_prompts(which, mode):
    from mapsum.config import LLAMA32_3B as C
    d = np.load(os.path.join(GOLD, f"fullshape_{which}_{mode}.npz"))
    meta = json.loads(bytes(d["meta"]).decode())
    assert meta["which"] == which and meta["mode"] == mode
    assert meta["n_layers"] == C.n_layers == 28 and meta["prompt_len"] == 2048
    if which == "flat":  # the bench's exact weights (bench.py init_synthetic(seed=0, std=0.02, norm_jitter=0))
        assert (meta["seed"], meta["std"], meta["jitter"]) == (0, 0.02, 0.0)
    if which == "q4km":  # bench.py --weights q4_k_m: init_synthetic_q(seed=2, scale=0.02, norm_jitter=0)
        assert (meta["seed"], meta["std"], meta["jitter"]) == (2, 0.02, 0.0)
    chunks = _bench().synthetic_chunks(8, 2048, doc=0, vocab=C.vocab, bos=C.bos_id)
    for ci in meta["chunks"]:
        k = f"c{ci}_"
        assert np.array_equal(d[k + "prompt"], chunks[ci])  # configs[1]'s own chunks
        assert d[k + "hid_rows"].shape == (28, 3, C.hidden) and d[k + "hid_norm"].shape == (28, 2048)
        assert d[k + "hid_sketch"].shape == (28, 512, 8)
        assert d[k + "gen_ids"].shape == (meta["gen"],) and meta["gen"] >= 128
        tv = d[k + "gen_top_vals"]
        assert np.all(np.diff(tv, axis=1) <= 0)  # top-16 sorted
        assert np.array_equal(d[k + "gen_ids"], d[k + "gen_top_ids"][:, 0])  # greedy = top-1
        # the residual grows through the stack (the sketch is not all zeros / NaN)
        assert np.all(np.isfinite(d[k + "hid_norm"])) and np.all(d[k + "hid_norm"][-1] > 0)


@pytest.mark.parametrize("mode", ["fp32", "engine"])
def test_sharp_fixture_is_decisive_and_copies(mode):
    """The sharp model's oracle continuation is the copy head's (token(p+1) = token(p-36)) with
    top-2 gaps far above any fp16 logit noise; the flat one has near-ties (why it exists)."""
    import sharp_model
    d = np.load(os.path.join(GOLD, f"fullshape_sharp_{mode}.npz"))
    meta = json.loads(bytes(d["meta"]).decode())
    assert meta["copy_offset"] == sharp_model.COPY_OFFSET
    assert meta["copy_layer"] == sharp_model.COPY_LAYER >= 20  # a late layer (round-3 review)
    for ci in meta["chunks"]:
        k = f"c{ci}_"
        n = len(d[k + "gen_ids"])
        assert list(d[k + "gen_ids"]) == sharp_model.expected_continuation(d[k + "prompt"], n)
        gap = d[k + "gen_top_vals"][:, 0] - d[k + "gen_top_vals"][:, 1]
        # >> the engine's logit noise (~4e-3 of the logits' rms against fp32, tools/parity_modes_cpu.py)
        assert gap.min() > 0.1 * float(np.mean(d[k + "lg_rms"]))
    f = np.load(os.path.join(GOLD, "fullshape_flat_fp32.npz"))
    gap = f["c0_gen_top_vals"][:, 0] - f["c0_gen_top_vals"][:, 1]
    assert gap.min() < 0.01  # flat logits: near-ties exist


def test_q4km_block_generator_matches_a_c_restatement():
    """oracle/synth.py synth_qblocks (the fixture's weights) restates csrc/k_qgemv.hip
    synth_qblocks_kernel: spot blocks of a Q4_K and a Q6_K tensor against hashes computed
    once from a C restatement of the kernel body (clang, _Float16; values recorded here)."""
    from oracle.synth import synth_qblocks

    def h(r):
        s = 0
        for x in r:
            s = (s * 131 + int(x)) % (1 << 64)
        return s
    got = [h(r) for r in synth_qblocks(12, 3, 2, 5, 3)] + [h(r) for r in synth_qblocks(14, 3, 2, 0, 0)]
    assert got == [8019031135127078327, 9551836282545629676, 12036773794748307063,
                   10111947276205690581, 16656358883380273260, 9763757120072924146]


def test_q4km_fixture_is_exact_dequant():
    """The Q4_K_M fixture's oracle ran on the EXACT fp32 dequantisation: the weights it
    describes are not fp16-valued (the Q4_K d * q - m products need more than 11 bits)."""
    from mapsum.config import LLAMA32_3B as C
    from oracle.quants import dequant, q4_k_m_type
    from oracle.synth import WO, synth_qblocks
    qt = q4_k_m_type("wo", 0, C.n_layers)
    w = dequant(synth_qblocks(qt, 64, 2, WO, 0, 0.02), qt)
    assert np.any(w.astype(np.float16).astype(np.float32) != w)
