"""GGUF reader/loader (mapsum/gguf.py).  No GGUF ships with the reference or this image,
so the files are written here by a minimal GGUF v3 writer (format as published by ggml)
with llama.cpp's Q/K row permutation applied; parity against a real Ollama blob is
unpinned.  CPU tests use a recording engine; the GPU test runs a real engine from a GGUF
against the oracle."""
import struct

import numpy as np
import pytest

from mapsum import _lib as L
from mapsum import gguf
from mapsum.config import TINY
from mapsum.weights import f32_to_f16_bits
from oracle import quants as Q
from oracle.synth import make_weights


def _s(x: str) -> bytes:
    b = x.encode()
    return struct.pack("<Q", len(b)) + b


def write_gguf(path, meta: dict, tensors: list, align=32):
    """tensors: [(name, ggml_type, dims innermost-first, raw bytes)]."""
    out = bytearray(b"GGUF" + struct.pack("<IQQ", 3, len(tensors), len(meta)))
    for k, v in meta.items():
        out += _s(k)
        if isinstance(v, bool):
            out += struct.pack("<IB", 7, int(v))
        elif isinstance(v, str):
            out += struct.pack("<I", 8) + _s(v)
        elif isinstance(v, float):
            out += struct.pack("<If", 6, v)
        elif isinstance(v, (list, tuple)):  # arrays: of strings (type 8) or of int32 (type 5)
            if v and isinstance(v[0], str):
                out += struct.pack("<IIQ", 9, 8, len(v)) + b"".join(_s(x) for x in v)
            else:
                out += struct.pack("<IIQ", 9, 5, len(v)) + b"".join(struct.pack("<i", int(x)) for x in v)
        else:
            out += struct.pack("<II", 4, v)
    off, datas = 0, []
    for name, t, dims, raw in tensors:
        out += _s(name) + struct.pack("<I", len(dims)) + b"".join(struct.pack("<Q", d) for d in dims)
        out += struct.pack("<IQ", t, off)
        pad = (-len(raw)) % align
        datas.append(raw + b"\0" * pad)
        off += len(raw) + pad
    out += b"\0" * ((-len(out)) % align)
    out += b"".join(datas)
    open(path, "wb").write(bytes(out))


META = {"general.architecture": "llama", "llama.block_count": TINY.n_layers,
        "llama.embedding_length": TINY.hidden, "llama.attention.head_count": TINY.n_heads,
        "llama.attention.head_count_kv": TINY.n_kv_heads, "general.name": "tiny-test"}
_NAMES = {"wq": "attn_q", "wk": "attn_k", "wv": "attn_v", "wo": "attn_output", "w_gate": "ffn_gate",
          "w_up": "ffn_up", "w_down": "ffn_down"}


def rope_freqs(cfg=TINY):
    """llama.cpp's rope_freqs.weight for a llama3-scaled config (the converter's divisors)."""
    from mapsum.config import llama3_rope_factors
    f = llama3_rope_factors(cfg).astype(np.float32)
    return ("rope_freqs.weight", gguf.GGML_F32, [f.size], f.tobytes())


def float_gguf(path, w, dtype=np.float32):
    t = gguf.GGML_F32 if dtype == np.float32 else gguf.GGML_F16
    f = lambda a: a.astype(dtype).tobytes()  # noqa: E731
    ts = [("token_embd.weight", t, [TINY.hidden, TINY.vocab], f(w["embed"])),
          ("output_norm.weight", gguf.GGML_F32, [TINY.hidden], w["final_norm"].astype(np.float32).tobytes()),
          rope_freqs()]
    heads = {"wq": TINY.n_heads, "wk": TINY.n_kv_heads}
    for i, ly in enumerate(w["layers"]):
        for n in ("attn_norm", "ffn_norm"):
            ts.append((f"blk.{i}.{n}.weight", gguf.GGML_F32, [TINY.hidden], ly[n].astype(np.float32).tobytes()))
        for n, g in _NAMES.items():
            a = gguf.permute_rows(ly[n], heads[n]) if n in heads else ly[n]
            ts.append((f"blk.{i}.{g}.weight", t, [a.shape[1], a.shape[0]], f(a)))
    write_gguf(path, META, ts)


class Recorder:
    cfg = TINY

    def __init__(self):
        self.f16, self.q = {}, {}

    def load_tensor(self, tensor, layer, bits):
        self.f16[(tensor, layer)] = np.asarray(bits)

    def load_tensor_q(self, tensor, layer, qt, blocks):
        self.q[(tensor, layer)] = (qt, np.asarray(blocks))


_T = {"wq": L.MS_T_WQ, "wk": L.MS_T_WK, "wv": L.MS_T_WV, "wo": L.MS_T_WO, "w_gate": L.MS_T_WGATE,
      "w_up": L.MS_T_WUP, "w_down": L.MS_T_WDOWN}


def test_permute_roundtrip():
    a = np.arange(6 * 128 * 3).reshape(6 * 128, 3)
    p = gguf.permute_rows(a, 6)
    assert not np.array_equal(p, a)
    assert np.array_equal(p[1], a[64]) and np.array_equal(p[2], a[1])  # rotary pairs adjacent
    assert np.array_equal(gguf.unpermute_rows(p, 6), a)


def test_float_gguf_loads_logical_weights(tmp_path):
    w = make_weights(TINY, 5, std=0.05, jitter=0.1)
    path = str(tmp_path / "tiny-f32.gguf")
    float_gguf(path, w)
    meta, ts = gguf.read_gguf(path)
    assert meta["general.name"] == "tiny-test" and len(ts) == 3 + 9 * TINY.n_layers
    eng = Recorder()
    gguf.load_gguf(eng, path)
    assert np.array_equal(eng.f16[(L.MS_T_EMBED, 0)], f32_to_f16_bits(w["embed"]))
    for i, ly in enumerate(w["layers"]):
        for n, t in _T.items():
            assert np.array_equal(eng.f16[(t, i)], f32_to_f16_bits(ly[n])), (i, n)
        assert np.array_equal(eng.f16[(L.MS_T_ATTN_NORM, i)], f32_to_f16_bits(ly["attn_norm"]))


def test_quant_gguf_loads_unpermuted_blocks(tmp_path):
    rng = np.random.default_rng(0)
    ts, want = [], {}
    heads = {"wq": TINY.n_heads, "wk": TINY.n_kv_heads}
    shapes = {"wq": (TINY.n_heads * 128, TINY.hidden), "wk": (TINY.n_kv_heads * 128, TINY.hidden),
              "wv": (TINY.n_kv_heads * 128, TINY.hidden), "wo": (TINY.hidden, TINY.n_heads * 128),
              "w_gate": (TINY.ffn, TINY.hidden), "w_up": (TINY.ffn, TINY.hidden), "w_down": (TINY.hidden, TINY.ffn)}
    emb = Q.random_blocks(Q.GGML_TYPE_Q6_K, TINY.vocab * TINY.hidden // 256, seed=1).reshape(TINY.vocab, -1)
    ts.append(("token_embd.weight", gguf.GGML_Q6_K, [TINY.hidden, TINY.vocab], emb.tobytes()))
    ts.append(("output_norm.weight", gguf.GGML_F32, [TINY.hidden], np.ones(TINY.hidden, np.float32).tobytes()))
    ts.append(rope_freqs())
    for i in range(TINY.n_layers):
        for n in ("attn_norm", "ffn_norm"):
            ts.append((f"blk.{i}.{n}.weight", gguf.GGML_F32, [TINY.hidden],
                       rng.standard_normal(TINY.hidden).astype(np.float32).tobytes()))
        for n, g in _NAMES.items():
            qt = Q.GGML_TYPE_Q6_K if n == "wv" else Q.GGML_TYPE_Q4_K
            r, k = shapes[n]
            b = Q.random_blocks(qt, r * k // 256, seed=10 * i + len(n)).reshape(r, -1)
            want[(i, n)] = (qt, b)
            a = gguf.permute_rows(b, heads[n]) if n in heads else b
            ts.append((f"blk.{i}.{g}.weight", qt, [k, r], a.tobytes()))
    path = str(tmp_path / "tiny-q4km.gguf")
    write_gguf(path, META, ts)
    eng = Recorder()
    gguf.load_gguf(eng, path)
    assert np.array_equal(eng.q[(L.MS_T_EMBED, 0)][1], emb.reshape(-1))
    for (i, n), (qt, b) in want.items():
        got_t, got = eng.q[(_T[n], i)]
        assert got_t == qt and np.array_equal(got, b.reshape(-1)), (i, n)


def test_errors(tmp_path):
    p = tmp_path / "bad.gguf"
    p.write_bytes(b"GGML" + b"\0" * 64)
    with pytest.raises(gguf.GGUFError):
        gguf.read_gguf(str(p))
    write_gguf(str(p), dict(META, **{"llama.block_count": 3}), [])
    with pytest.raises(gguf.GGUFError, match="block_count"):
        gguf.load_gguf(Recorder(), str(p))
    write_gguf(str(p), META, [("token_embd.weight", 2, [32, 4], b"\0" * 72)])  # Q4_0
    with pytest.raises(gguf.GGUFError, match="not supported"):
        gguf.read_gguf(str(p))


def test_rope_freqs_must_match_the_engine(tmp_path):
    """the engine builds its cos / sin tables from its config, so a GGUF whose
    rope_freqs.weight holds other llama3 divisors (here: another scaling factor), or none at all
    for a scaled config, is refused instead of silently running with the wrong RoPE."""
    w = make_weights(TINY, 5, std=0.05, jitter=0.1)
    good = str(tmp_path / "good.gguf")
    float_gguf(good, w)
    gguf.load_gguf(Recorder(), good)
    meta, ts = gguf.read_gguf(good)
    other = rope_freqs(TINY.with_(rope_factor=8.0))
    for name, entries in (("other", [other]), ("missing", [])):
        p = str(tmp_path / f"{name}.gguf")
        keep = [(n, t, d, bytes(raw)) for n, (t, d, raw) in ts.items() if n != "rope_freqs.weight"]
        write_gguf(p, META, keep + entries)
        with pytest.raises(gguf.GGUFError, match="rope_freqs"):
            gguf.load_gguf(Recorder(), p)
    # an unscaled config needs no table
    class Unscaled(Recorder):
        cfg = TINY.with_(rope_factor=0.0)
    p = str(tmp_path / "missing.gguf")
    gguf.load_gguf(Unscaled(), p)


@pytest.mark.gpu
def test_engine_from_gguf_vs_oracle(tmp_path):
    """A real engine loaded from an F32 GGUF (permuted Q/K rows) reproduces the oracle."""
    from mapsum.engine import Engine
    from oracle.llama_ref import OracleLlama
    w = make_weights(TINY, 9, std=0.05, jitter=0.1)
    path = str(tmp_path / "tiny.gguf")
    float_gguf(path, w)
    ids = np.random.default_rng(4).integers(0, 4000, size=80).astype(np.int32)
    with Engine(TINY, device=0, max_batch=2, max_ctx=256, max_prefill_tokens=256) as e:
        gguf.load_gguf(e, path)
        _, lg = e.forward(ids, hidden=False, logits=True)
        got = e.generate([ids], num_predict=8, ignore_eos=True)[0].ids
    oracle = OracleLlama(TINY, w)
    ref_lg, _ = oracle.forward(ids, all_logits=True)
    assert float(np.linalg.norm(lg - ref_lg) / np.linalg.norm(ref_lg)) < 2e-2
    ref, _ = oracle.generate(ids, 8, ignore_eos=True)
    assert got == ref
