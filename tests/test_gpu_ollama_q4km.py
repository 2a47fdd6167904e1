"""The reference's own model tag on K-quant weights, end to end.

``ollama pull llama3.2:3b`` installs a Q4_K_M GGUF (Q4_K matrices, Q6_K for the tied
token_embd and for half of attn_v / ffn_down -- llama.cpp's LLAMA_FTYPE_MOSTLY_Q4_K_M mix,
restated in oracle/quants.py q4_k_m_type), and the reference reaches it through
``OllamaLLM("http://localhost:11434", "llama3.2:3b")`` (run_full_evaluation_pipeline.py:961).
No such file exists offline, so this test writes one of the same structure at the TINY
shapes: float weights quantised by oracle/quantize.py at each tensor's Q4_K_M type, Q/K rows
permuted as llama.cpp's converter does, F32 norms, rope_freqs, the trained byte-level BPE of
tests/test_ollama_gguf.py in the metadata, and an Ollama-layout manifest with a Llama-3
template layer.  The GPU test then runs the drop-in class with only OLLAMA_MODELS set and
checks its engine against the oracle run on the EXACT dequantisation of the same blocks
(oracle/ggml_quants.c), by the bar of tests/test_gpu_parity.py's quantised-engine test:
logits within 2e-2, every greedy token the oracle's argmax except at an oracle near-tie."""
import asyncio
import os

import numpy as np
import pytest

from mapsum import _lib as L
from mapsum import compat, gguf, ollama_store, template
from mapsum.config import TINY
from oracle import quants as Q
from oracle.quantize import quantize
from oracle.synth import make_weights
from test_gguf import META, _NAMES, rope_freqs, write_gguf
from test_ollama_gguf import LLAMA3_LIKE, PARAMS, RecordingEngine, ollama_store_with, trained  # noqa: F401

_T = {"wq": L.MS_T_WQ, "wk": L.MS_T_WK, "wv": L.MS_T_WV, "wo": L.MS_T_WO,
      "w_gate": L.MS_T_WGATE, "w_up": L.MS_T_WUP, "w_down": L.MS_T_WDOWN}
PROMPTS = ["Chương 1. Nội dung chính của văn bản.",
           "Hà Nội, ngày 15 tháng 8 năm 2024 -- báo cáo tổng kết. Phần II. Điều 7: kết luận và kiến nghị.",
           "Tóm tắt nội dung văn bản tiếng Việt."]
N_GEN = 40


def q4km_model(seed=21):
    """(qw: {name | (layer, name): (type, un-permuted blocks [rows, bytes])}, logical float weights
    of the GGUF = exact dequantisation, the float weights that were quantised)."""
    w = make_weights(TINY, seed, std=0.05, jitter=0.1)
    qt = Q.q4_k_m_type("embed", 0, TINY.n_layers)
    qw = {"embed": (qt, quantize(w["embed"], qt).reshape(TINY.vocab, -1))}
    dq = {"embed": Q.c_dequant(qw["embed"][1], qt).reshape(TINY.vocab, TINY.hidden),
          "final_norm": w["final_norm"], "layers": []}
    dq["lm_head"] = dq["embed"]
    for i, ly in enumerate(w["layers"]):
        d = {"attn_norm": ly["attn_norm"], "ffn_norm": ly["ffn_norm"]}
        for n in _NAMES:
            qt = Q.q4_k_m_type(n, i, TINY.n_layers)
            a = np.asarray(ly[n], np.float32)
            qw[(i, n)] = (qt, quantize(a, qt).reshape(a.shape[0], -1))
            d[n] = Q.c_dequant(qw[(i, n)][1], qt).reshape(a.shape)
        dq["layers"].append(d)
    return qw, dq, w


def q4km_gguf(path, qw, w, tok_meta):
    f = lambda a: np.asarray(a, np.float32).tobytes()  # noqa: E731
    qt, eb = qw["embed"]
    ts = [("token_embd.weight", qt, [TINY.hidden, TINY.vocab], eb.tobytes()),
          ("output_norm.weight", gguf.GGML_F32, [TINY.hidden], f(w["final_norm"])), rope_freqs()]
    heads = {"wq": TINY.n_heads, "wk": TINY.n_kv_heads}
    for i, ly in enumerate(w["layers"]):
        for n in ("attn_norm", "ffn_norm"):
            ts.append((f"blk.{i}.{n}.weight", gguf.GGML_F32, [TINY.hidden], f(ly[n])))
        for n, g in _NAMES.items():
            qt, b = qw[(i, n)]
            a = gguf.permute_rows(b, heads[n]) if n in heads else b
            rows, cols = np.asarray(ly[n]).shape
            ts.append((f"blk.{i}.{g}.weight", qt, [cols, rows], a.tobytes()))
    meta = dict(META, **{"llama.feed_forward_length": TINY.ffn, "llama.rope.freq_base": TINY.rope_theta,
                         "llama.attention.layer_norm_rms_epsilon": TINY.norm_eps,
                         "general.file_type": 15}, **tok_meta)  # 15 = LLAMA_FTYPE_MOSTLY_Q4_K_M
    write_gguf(path, meta, ts)


@pytest.fixture(scope="module")
def q4km_store(trained, tmp_path_factory):  # noqa: F811
    _, tok_meta = trained
    root = tmp_path_factory.mktemp("ollama_q4km")
    qw, dq, w = q4km_model()
    g = str(root / "model.gguf")
    q4km_gguf(g, qw, w, tok_meta)
    ollama_store_with(str(root), "llama3.2:3b", g, PARAMS, template=LLAMA3_LIKE)
    os.remove(g)
    return str(root), qw, dq


def test_q4km_store_uploads_the_blocks(q4km_store, monkeypatch):
    """CPU: the store route uploads every matrix as its raw K-quant blocks (Q/K un-permuted),
    both types of the mix occur, and the tied Q6_K embedding is the lm head."""
    root, qw, _ = q4km_store
    assert {qt for qt, _ in qw.values()} == {Q.GGML_TYPE_Q4_K, Q.GGML_TYPE_Q6_K}
    m = ollama_store.resolve("llama3.2:3b", root)
    assert m.template == LLAMA3_LIKE
    eng = RecordingEngine(TINY)
    gguf.load_gguf(eng, m.gguf)
    assert eng.q[(L.MS_T_EMBED, 0)][0] == Q.GGML_TYPE_Q6_K
    assert np.array_equal(eng.q[(L.MS_T_EMBED, 0)][1], qw["embed"][1].reshape(-1))
    for i in range(TINY.n_layers):
        for n in _NAMES:
            qt, b = qw[(i, n)]
            got_t, got = eng.q[(_T[n], i)]
            assert got_t == qt and np.array_equal(got, b.reshape(-1)), (i, n)


def _agreement(oracle, prompt, gen):
    """Teacher-forced: the oracle's argmax after prompt + gen[:i] vs gen[i]; returns the
    positions that differ with the oracle's top-2 gap there."""
    ids = np.concatenate([np.asarray(prompt, np.int32), np.asarray(gen[:-1], np.int32)])
    lg, _ = oracle.forward(ids, all_logits=True)
    lg = lg[len(prompt) - 1:]
    srt = np.sort(lg, 1)
    return [(i, float(srt[i, -1] - lg[i, gen[i]]), float(srt[i, -1]))
            for i in range(len(gen)) if int(np.argmax(lg[i])) != gen[i]], lg


@pytest.mark.gpu
def test_ollamallm_q4km_store_vs_oracle(q4km_store, monkeypatch):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.llama_ref import OracleLlama
    root, _, dq = q4km_store
    for k, v in (("OLLAMA_MODELS", root), ("MAPSUM_MAX_BATCH", "8"), ("MAPSUM_MAX_CTX", "1024"),
                 ("MAPSUM_MAX_PREFILL", "4096")):
        monkeypatch.setenv(k, v)
    for k in ("MAPSUM_MODEL_DIR", "MAPSUM_GGUF", "MAPSUM_ALLOW_TEMPLATE"):
        monkeypatch.delenv(k, raising=False)
    compat._BACKENDS.pop("llama3.2:3b", None)
    try:
        llm = compat.OllamaLLM("http://localhost:11434", "llama3.2:3b", max_new_tokens=N_GEN, clean="none")
        prompts = [template.map_prompt("mapreduce", t) for t in PROMPTS]
        first = llm._call(prompts[0])

        async def fan_out():
            return await asyncio.gather(*[llm._acall(p) for p in prompts])
        outs = asyncio.run(fan_out())
        assert outs[0] == first  # batched == alone (the decode arithmetic is fixed per engine)
        be = compat.get_backend("llama3.2:3b")
        assert be.engine.cfg.vocab == TINY.vocab and be.engine.cfg.tie_embeddings
        ids = [be.encode_prompt(p) for p in prompts]
        free = be.engine.generate(ids, num_predict=N_GEN, ignore_eos=True)
        stopped = be.generate_ids(ids, N_GEN)
        oracle = OracleLlama(TINY, dq)
        agree = total = 0
        for k, (p, r, s) in enumerate(zip(ids, free, stopped)):
            # the call's text is the decode of the greedy ids up to the first stop id
            assert r.ids[:len(s.ids)] == s.ids
            assert outs[k] == compat.CLEANERS["none"](be.tok.decode(s.ids))
            flips, lg = _agreement(oracle, p, r.ids)
            print(f"prompt {k}: {len(p)} tokens, {N_GEN - len(flips)}/{N_GEN} greedy tokens = oracle argmax"
                  f", flips {[(i, round(g, 4)) for i, g, _ in flips]}, stop after {len(s.ids)}")
            for pos, gap, top in flips:  # only at a near-tie of the oracle's own logits
                assert gap <= 1e-2 * (abs(top) + 1.0), (k, pos, gap, top)
            agree += N_GEN - len(flips)
            total += N_GEN
        assert agree / total >= 0.97, (agree, total)
        _, lg = be.engine.forward(ids[1], hidden=False, logits=True)
        ref_lg, _ = oracle.forward(ids[1], all_logits=True)
        err = float(np.linalg.norm(lg - ref_lg) / np.linalg.norm(ref_lg))
        print(f"prefill logits rel err {err:.2e}")
        assert err < 2e-2
    finally:
        b = compat._BACKENDS.pop("llama3.2:3b", None)
        if b is not None:
            b.engine.close()
