"""The drop-in's route to the reference's own model tag.

The reference constructs ``OllamaLLM("http://localhost:11434", "llama3.2:3b")``
(run_full_evaluation_pipeline.py:961, runners/run_summarization_ollama_mapreduce.py:206);
Ollama serves that tag from a GGUF blob named by a manifest under ~/.ollama/models, and
tokenises with the vocabulary stored in the GGUF's own metadata (there is no tokenizer.json
in an Ollama install).  No Ollama store, GGUF or Llama-3 vocabulary exists offline, so the
files here are synthetic: a byte-level BPE trained on the reference's own Vietnamese map
prompt (mapsum/template.py) with Llama-3's pre-tokenizer, written into GGUF metadata the way
llama.cpp's converter writes it (tokenizer.ggml.model "gpt2", .pre "llama-bpe", tokens,
token_type, merges, bos/eos ids), TINY weights with llama.cpp's Q/K row permutation, and an
Ollama-layout manifest + content-addressed blobs.  Parity of the tokenizer against the real
Llama-3.2 vocabulary is unpinned (the vocabulary is not available here)."""
import hashlib
import json
import os
import shutil

import numpy as np
import pytest

from mapsum import compat, gguf, ollama_store, template
from mapsum.config import TINY
from mapsum.engine import RequestQueue, Result
from mapsum.tokenizer import PRE_TOKENIZERS, Tokenizer, gguf_stop_ids, tokenizer_from_gguf
from oracle.synth import make_weights
from test_gguf import META, _NAMES, rope_freqs, write_gguf

SPECIALS = {4000: "<|begin_of_text|>", 4001: "<|end_of_text|>", 4002: "<|eot_id|>",
            4003: "<|start_header_id|>", 4004: "<|end_header_id|>", 4005: "<|eom_id|>"}
CORPUS = [template.MAP_PROMPT_MAPREDUCE, "Tóm tắt nội dung văn bản tiếng Việt. Chương 12: Kết luận!",
          "Hà Nội, ngày 15 tháng 8 năm 2024 -- báo cáo 3,141 trang.\n\nPhần II.\tĐiều 7"] * 3
SAMPLES = ["Văn bản dài: 12345 ký tự, 'quoted' và \"double\"...\n\n  thụt lề",
           "Đây là bản tóm tắt ngắn gọn.\r\nDòng mới", "mixed English words, CAPS and café",
           template.map_prompt("mapreduce", "Chương 1. Nội dung chính.")]


@pytest.fixture(scope="module")
def trained():
    """(reference tokenizer object, GGUF tokenizer metadata) of a 4096-entry vocabulary."""
    from tokenizers import Regex, decoders, models, pre_tokenizers, trainers
    from tokenizers import Tokenizer as T
    pat, _ = PRE_TOKENIZERS["llama-bpe"]
    tk = T(models.BPE(ignore_merges=True))
    tk.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(pat), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, trim_offsets=False, use_regex=False)])
    tk.decoder = decoders.ByteLevel()
    tk.train_from_iterator(CORPUS, trainers.BpeTrainer(vocab_size=700, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                                        show_progress=False))
    model = json.loads(tk.to_str())["model"]
    vocab = model["vocab"]
    merges = [m if isinstance(m, str) else " ".join(m) for m in model["merges"]]
    tokens = [None] * TINY.vocab
    for t, i in vocab.items():
        tokens[i] = t
    types = [1] * TINY.vocab
    for i in range(TINY.vocab):
        if tokens[i] is None:
            tokens[i] = SPECIALS.get(i, f"<|reserved_special_token_{i}|>")
            types[i] = 3
    meta = {"tokenizer.ggml.model": "gpt2", "tokenizer.ggml.pre": "llama-bpe", "tokenizer.ggml.tokens": tokens,
            "tokenizer.ggml.token_type": types, "tokenizer.ggml.merges": merges,
            "tokenizer.ggml.bos_token_id": 4000, "tokenizer.ggml.eos_token_id": 4002,
            "tokenizer.ggml.add_bos_token": True}
    return tk, meta


def test_gguf_tokenizer_equals_the_trained_one(trained):
    tk, meta = trained
    g = tokenizer_from_gguf(meta)
    for s in CORPUS + SAMPLES:
        assert g.encode(s, add_bos=False) == tk.encode(s).ids, s[:40]
        assert g.decode(g.encode(s)) == s  # byte-level: lossless, BOS skipped as special
    assert g.bos_id == 4000
    full = template.render_llama32("Xin chào")
    ids = g.encode(full, add_bos=False)
    assert ids[:2] == [4000, 4003] and 4002 in ids and 4004 in ids  # template specials are one id each
    assert gguf_stop_ids(meta) == (4002, 4005, 4001)


def test_gguf_tokenizer_rejects_other_families(trained):
    _, meta = trained
    with pytest.raises(ValueError, match="byte-level"):
        tokenizer_from_gguf(dict(meta, **{"tokenizer.ggml.model": "llama"}))
    with pytest.raises(ValueError, match="pre-tokenizer"):
        tokenizer_from_gguf(dict(meta, **{"tokenizer.ggml.pre": "qwen2"}))


@pytest.mark.parametrize("tag,want", [
    ("llama3.2:3b", ("registry.ollama.ai", "library", "llama3.2", "3b")),
    ("llama3.2", ("registry.ollama.ai", "library", "llama3.2", "latest")),
    ("me/summ:q4", ("registry.ollama.ai", "me", "summ", "q4")),
    ("hf.co/org/model:Q4_K_M", ("hf.co", "org", "model", "Q4_K_M")),
])
def test_parse_tag(tag, want):
    assert ollama_store.parse_tag(tag) == want


@pytest.mark.parametrize("bad", ["", " x", "a/b/c/d:t", "m:"])
def test_parse_tag_rejects(bad):
    with pytest.raises(ValueError):
        ollama_store.parse_tag(bad)


def tiny_gguf(path, w, tok_meta):
    """TINY weights (F32, Q/K rows permuted as llama.cpp's converter does) + tokenizer metadata."""
    f = lambda a: np.asarray(a, np.float32).tobytes()  # noqa: E731
    ts = [("token_embd.weight", gguf.GGML_F32, [TINY.hidden, TINY.vocab], f(w["embed"])),
          ("output_norm.weight", gguf.GGML_F32, [TINY.hidden], f(w["final_norm"])), rope_freqs()]
    heads = {"wq": TINY.n_heads, "wk": TINY.n_kv_heads}
    for i, ly in enumerate(w["layers"]):
        for n in ("attn_norm", "ffn_norm"):
            ts.append((f"blk.{i}.{n}.weight", gguf.GGML_F32, [TINY.hidden], f(ly[n])))
        for n, g in _NAMES.items():
            a = gguf.permute_rows(ly[n], heads[n]) if n in heads else ly[n]
            ts.append((f"blk.{i}.{g}.weight", gguf.GGML_F32, [a.shape[1], a.shape[0]], f(a)))
    meta = dict(META, **{"llama.feed_forward_length": TINY.ffn, "llama.rope.freq_base": TINY.rope_theta,
                         "llama.attention.layer_norm_rms_epsilon": TINY.norm_eps}, **tok_meta)
    write_gguf(path, meta, ts)


def ollama_store_with(root, tag, gguf_path, params, template=None):
    """An Ollama models dir holding one pulled model: manifest + sha256-named blobs."""
    host, ns, model, t = ollama_store.parse_tag(tag)
    os.makedirs(os.path.join(root, "blobs"), exist_ok=True)
    layers = []
    items = [(ollama_store.MODEL_MEDIA, open(gguf_path, "rb").read()),
             (ollama_store.PARAMS_MEDIA, json.dumps(params).encode())]
    if template is not None:
        items.append((ollama_store.TEMPLATE_MEDIA, template.encode()))
    for media, data in items:
        dg = hashlib.sha256(data).hexdigest()
        open(os.path.join(root, "blobs", f"sha256-{dg}"), "wb").write(data)
        layers.append({"mediaType": media, "digest": f"sha256:{dg}", "size": len(data)})
    mdir = os.path.join(root, "manifests", host, ns, model)
    os.makedirs(mdir, exist_ok=True)
    with open(os.path.join(mdir, t), "w") as fh:
        json.dump({"schemaVersion": 2, "layers": layers}, fh)


PARAMS = {"stop": ["<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>"]}


@pytest.fixture(scope="module")
def store(trained, tmp_path_factory):
    _, tok_meta = trained
    root = tmp_path_factory.mktemp("ollama_models")
    w = make_weights(TINY, 21, std=0.05, jitter=0.1)
    g = str(root / "model.gguf")
    tiny_gguf(g, w, tok_meta)
    ollama_store_with(str(root), "llama3.2:3b", g, PARAMS)
    os.remove(g)  # only the content-addressed blob remains, as in a real store
    return str(root), w


# Ollama's llama3.2 chat template source is EXT (not offline): a llama3-family stand-in with the
# same structure (Go template actions, Llama-3 header / end-of-turn markers), and a ChatML one
LLAMA3_LIKE = ("{{- range .Messages }}<|start_header_id|>{{ .Role }}<|end_header_id|>\n\n{{ .Content }}"
               "<|eot_id|>{{ end }}<|start_header_id|>assistant<|end_header_id|>\n\n")
CHATML = "{{- range .Messages }}<|im_start|>{{ .Role }}\n{{ .Content }}<|im_end|>\n{{ end }}<|im_start|>assistant\n"


def test_resolve_checks_the_template(tmp_path, store):
    """the manifest's template layer is read and checked -- a llama3-family
    template resolves, any other family is refused (the engine renders Llama-3.2's template
    itself, mapsum/template.py), unless explicitly allowed."""
    root, _ = store
    blob = ollama_store.resolve("llama3.2:3b", root).gguf
    for tag, tmpl in (("llama3.2:ok", LLAMA3_LIKE), ("llama3.2:chatml", CHATML)):
        ollama_store_with(root, tag, blob, PARAMS, template=tmpl)
    assert ollama_store.template_problems(LLAMA3_LIKE) == []
    m = ollama_store.resolve("llama3.2:ok", root)
    assert m.template == LLAMA3_LIKE
    with pytest.raises(ollama_store.OllamaStoreError, match="template is not Llama-3"):
        ollama_store.resolve("llama3.2:chatml", root)
    assert ollama_store.resolve("llama3.2:chatml", root, allow_foreign_template=True).template == CHATML


def test_gguf_add_bos_token_false(trained):
    """tokenizer.ggml.add_bos_token = false really disables BOS (it used to fall back
    to looking <|begin_of_text|> up)."""
    _, tok_meta = trained
    with_bos = tokenizer_from_gguf(tok_meta)
    no_bos = tokenizer_from_gguf(dict(tok_meta, **{"tokenizer.ggml.add_bos_token": False}))
    text = "xin chao the gioi"
    assert no_bos.bos_id is None
    assert no_bos.encode(text) == with_bos.encode(text, add_bos=False)
    if with_bos.bos_id is not None:
        assert with_bos.encode(text)[0] == with_bos.bos_id


def test_resolve_and_config(store):
    root, _ = store
    m = ollama_store.resolve("llama3.2:3b", root)
    assert os.path.basename(m.gguf).startswith("sha256-") and m.params == PARAMS
    meta, ts = gguf.read_gguf(m.gguf)
    cfg = ollama_store.config_from_gguf(meta)
    assert (cfg.n_layers, cfg.hidden, cfg.n_heads, cfg.n_kv_heads, cfg.ffn, cfg.vocab) == \
        (TINY.n_layers, TINY.hidden, TINY.n_heads, TINY.n_kv_heads, TINY.ffn, TINY.vocab)
    assert cfg.bos_id == 4000 and cfg.eos_ids[0] == 4002 and cfg.head_dim == 128
    with pytest.raises(ollama_store.OllamaStoreError, match="not found"):
        ollama_store.resolve("llama3.2:1b", root)


class RecordingEngine(RequestQueue):
    """CPU double of mapsum.engine.Engine for the factory: records the config, the stop set
    and every uploaded tensor; a chunk's 'summary' is its prompt ids reversed."""
    made = []

    def __init__(self, cfg, eos_ids=None, **kw):
        self.cfg, self.eos_ids, self.kw = cfg, eos_ids, kw
        self.f16, self.q, self.pending_, self.done = {}, {}, {}, []
        self._mailbox, self._tag = {}, 1
        RecordingEngine.made.append(self)

    def load_tensor(self, tensor, layer, bits):
        self.f16[(tensor, layer)] = np.asarray(bits)

    def load_tensor_q(self, tensor, layer, qt, blocks):
        self.q[(tensor, layer)] = (qt, np.asarray(blocks))

    def submit(self, ids, n, ignore_eos=False, tag=None):
        if tag is None:
            tag, self._tag = self._tag, self._tag + 1
        self.pending_[tag] = (list(ids), n)
        return tag

    def step(self):
        for tag, (ids, n) in self.pending_.items():
            self.done.append(Result(tag, ids[::-1][:n], "length", len(ids)))
        self.pending_ = {}
        return 0

    def poll(self, cap=256):
        out, self.done = self.done[:cap], self.done[cap:]
        return out


def test_ollamallm_tag_resolves_through_the_store(store, trained, monkeypatch):
    """OllamaLLM(url, 'llama3.2:3b') -> manifest -> GGUF blob -> config, tokenizer and weights
    from the file -> one map call, with no MAPSUM_MODEL_DIR / MAPSUM_GGUF set."""
    root, w = store
    monkeypatch.setenv("OLLAMA_MODELS", root)
    monkeypatch.delenv("MAPSUM_MODEL_DIR", raising=False)
    monkeypatch.delenv("MAPSUM_GGUF", raising=False)
    import mapsum.engine
    monkeypatch.setattr(mapsum.engine, "Engine", RecordingEngine)
    compat._BACKENDS.pop("llama3.2:3b", None)
    RecordingEngine.made.clear()
    try:
        llm = compat.OllamaLLM("http://localhost:11434", "llama3.2:3b", max_new_tokens=40)
        prompt = template.map_prompt("mapreduce", "Chương 1. Nội dung chính.")
        out = llm._call(prompt)
        eng = RecordingEngine.made[0]
        # the stop set: the GGUF's eos/eot/eom ids + the params layer's single-token stops
        assert eng.eos_ids[:3] == (4002, 4005, 4001) and 4003 in eng.eos_ids and 4004 in eng.eos_ids
        assert eng.cfg.vocab == TINY.vocab and eng.cfg.tie_embeddings
        from mapsum import _lib as L
        from mapsum.weights import f32_to_f16_bits
        assert np.array_equal(eng.f16[(L.MS_T_EMBED, 0)], f32_to_f16_bits(w["embed"]))
        assert np.array_equal(eng.f16[(L.MS_T_WQ, 1)], f32_to_f16_bits(w["layers"][1]["wq"]))  # un-permuted
        tok = tokenizer_from_gguf(trained[1])
        ids = tok.encode(template.render_llama32(prompt, add_bos=False), add_bos=True)
        assert ids[0] == 4000
        assert out == compat.CLEANERS["pipeline"](tok.decode(ids[::-1][:40]))
    finally:
        compat._BACKENDS.pop("llama3.2:3b", None)


@pytest.mark.gpu
def test_map_call_through_the_ollama_store_on_gpu(store, monkeypatch):
    """One map call on the GPU through the same route: OllamaLLM('llama3.2:3b') with only
    OLLAMA_MODELS set equals the same prompt ids run on an engine loaded directly from the
    weights (identical greedy ids -> identical text)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mapsum.engine import Engine
    from mapsum.weights import load_logical
    root, w = store
    for k, v in (("OLLAMA_MODELS", root), ("MAPSUM_MAX_BATCH", "4"), ("MAPSUM_MAX_CTX", "2048"),
                 ("MAPSUM_MAX_PREFILL", "4096")):
        monkeypatch.setenv(k, v)
    monkeypatch.delenv("MAPSUM_MODEL_DIR", raising=False)
    monkeypatch.delenv("MAPSUM_GGUF", raising=False)
    compat._BACKENDS.pop("llama3.2:3b", None)
    try:
        llm = compat.OllamaLLM("http://localhost:11434", "llama3.2:3b", max_new_tokens=24, clean="none")
        prompt = template.map_prompt("mapreduce", "Chương 1. Nội dung chính của văn bản.")
        out = llm._call(prompt)
        be = compat.get_backend("llama3.2:3b")
        ids = be.encode_prompt(prompt)
        with Engine(be.engine.cfg, device=0, max_batch=4, max_ctx=2048, max_prefill_tokens=4096,
                    eos_ids=tuple(be.engine.cfg.eos_ids)) as e:
            load_logical(e, w)
            want = e.generate([ids], num_predict=24, ignore_eos=True)[0].ids
        got = be.engine.generate([ids], num_predict=24, ignore_eos=True)[0].ids
        assert got == want
        assert isinstance(out, str)
    finally:
        b = compat._BACKENDS.pop("llama3.2:3b", None)
        if b is not None:
            b.engine.close()
