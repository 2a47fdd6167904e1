"""The persistent decode step (k_persist.hip) against the per-layer launches it replaces (needs a GPU).

Engines of <= 8 slots on fp16 Llama-3.2-3B weights run every layer of a decode step as ONE
launch: a loader wave per CU streams weights and K/V pages into an LDS ring ahead of every
dependency, three consumer waves compute, and phases hand off through write-through stores and
arrival counters.  The kernel restates the launches' arithmetic exactly (the split-6 QKV GEMV,
decode attention v2 + its split combine, the residual-fused O / down GEMVs, the gate/up SwiGLU
GEMV), so the bar here is BIT-EXACTNESS, not a tolerance: the same greedy ids, the same K/V
cache bytes of every layer (every step's new K/V row is written by the kernel), the same lm_head
partials of the last step and the same residual, at the benchmarked widths.  The 28-layer
parity against the oracle (tests/test_gpu_golden28*.py) runs through the persistent step by
default at 8 slots, so it inherits those bars too.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from mapsum import _lib as L  # noqa: E402
from mapsum.config import LLAMA32_3B  # noqa: E402
from mapsum.engine import Engine  # noqa: E402

SEED, STD, JIT = 77, 0.02, 0.1
P, NCHUNK = 2048, 8


def _chunks(n=NCHUNK, p=P, doc=0):
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench.synthetic_chunks(n, p, doc=doc, vocab=LLAMA32_3B.vocab, bos=LLAMA32_3B.bos_id)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def chunks():
    return _chunks()


def _run(cfg, prompts, gen, persist, slots=NCHUNK, ctx=P + 64, state=True):
    e = Engine(cfg, device=0, max_batch=slots, max_ctx=ctx, max_prefill_tokens=NCHUNK * P)
    try:
        ok = e.set_persist(persist)
        e.init_synthetic(SEED, STD, JIT)
        res = e.generate(list(prompts), num_predict=gen, ignore_eos=True)
        st = e.stats()
        out = {"ids": [r.ids for r in res], "ok": ok, "steps": st["persist_steps"],
               "fallbacks": st["persist_fallbacks"]}
        if state:
            H, V = cfg.hidden, cfg.vocab
            pages = (ctx + 63) // 64
            kv_layer = slots * pages * cfg.n_kv_heads * 64 * cfg.head_dim * 2
            out["k"] = e.debug_read(L.MS_DBG_KPOOL, 0, kv_layer * cfg.n_layers)
            out["v"] = e.debug_read(L.MS_DBG_VPOOL, 0, kv_layer * cfg.n_layers)
            # the last decode step's lm_head partials {max, id} of every row, and the residual
            out["lm"] = e.debug_read(L.MS_DBG_DECODE_LOGITS, 0, len(prompts) * (V // 16) * 8)
            out["x"] = e.debug_read(L.MS_DBG_DECODE_X, 0, len(prompts) * H * 4)
        return out
    finally:
        e.close()


def _same(a, b, cfg):
    assert a["ok"] and a["steps"] > 0 and a["fallbacks"] == 0, (a["ok"], a["steps"], a["fallbacks"])
    assert b["steps"] == 0
    assert a["ids"] == b["ids"]
    for key in ("k", "v"):
        if not np.array_equal(a[key], b[key]):
            per = a[key].size // cfg.n_layers
            bad = [l for l in range(cfg.n_layers) if not np.array_equal(a[key][l * per:(l + 1) * per],
                                                                           b[key][l * per:(l + 1) * per])]
            raise AssertionError(f"{key} cache differs in layers {bad}")
    assert np.array_equal(a["lm"], b["lm"]), "lm_head partials differ"
    assert np.array_equal(a["x"], b["x"]), "residual differs"


def test_persist_bit_exact_bench_widths(dev, chunks):
    """configs[1]'s batch (8 x 2048-token chunks, 8 slots) at the full widths, 2 layers: the
    persistent step and the launches give the same ids, K/V caches, lm_head partials, residual."""
    cfg = LLAMA32_3B.with_(n_layers=2)
    a = _run(cfg, chunks, 40, True)
    b = _run(cfg, chunks, 40, False)
    _same(a, b, cfg)


def test_persist_bit_exact_ragged(dev, chunks):
    """Ragged prompts: 1 .. 33 pages, splits with fewer pages than ppb, a new token on a page
    boundary (64, 65), fewer sequences than slots (attention items on fewer CUs)."""
    cfg = LLAMA32_3B.with_(n_layers=2)
    prompts = [chunks[i][:n] for i, n in enumerate((5, 63, 64, 65, 700, 1500, 2047))]
    a = _run(cfg, prompts, 40, True)
    b = _run(cfg, prompts, 40, False)
    _same(a, b, cfg)


@pytest.mark.parametrize("slots,n", [(1, 1), (3, 3), (8, 5)])
def test_persist_bit_exact_slots(dev, chunks, slots, n):
    """Engines of 1 / 3 / 8 slots with n sequences (rows of the MFMA tiles padded by duplicating
    the last row, as the GEMVs do)."""
    cfg = LLAMA32_3B.with_(n_layers=2)
    prompts = [chunks[i][: 300 + 97 * i] for i in range(n)]
    a = _run(cfg, prompts, 24, True, slots=slots, ctx=1024)
    b = _run(cfg, prompts, 24, False, slots=slots, ctx=1024)
    _same(a, b, cfg)


def test_persist_bit_exact_28_layers(dev, chunks):
    """The benchmarked model itself: all 28 layers, 8 x 2048-token chunks."""
    cfg = LLAMA32_3B
    a = _run(cfg, chunks, 24, True)
    b = _run(cfg, chunks, 24, False)
    _same(a, b, cfg)


def test_persist_timeout_recovers(dev, chunks, monkeypatch):
    """A hand-off that gives up (forced: MS_PK_SPIN=0 makes every poll that is not ready at once
    time out) never hangs or fails the step: the run is recomputed with the launches, the engine
    turns the persistent step off, and the ids are the launches' own."""
    cfg = LLAMA32_3B.with_(n_layers=2)
    want = _run(cfg, chunks[:4], 24, False, state=False)
    monkeypatch.setenv("MS_PK_SPIN", "0")
    got = _run(cfg, chunks[:4], 24, True, state=False)
    assert got["ids"] == want["ids"]
    assert got["fallbacks"] == 1 and got["steps"] == 0, (got["fallbacks"], got["steps"])
