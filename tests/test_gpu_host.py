"""The host paths end to end on the GPU (needs a GPU): the reference's call sites through
the drop-in ``OllamaLLM`` -> ``MapBackend`` -> libmapsum on cuda:0, with a toy byte-level
BPE whose vocabulary is the model's (the Llama-3.2 tokenizer is not available offline).

Reference call sites restated: ``generate_summary``'s ``await llm.ainvoke(prompt)``
fan-out (runners/run_summarization_ollama_mapreduce.py:103-112), the pipeline's
``OllamaLLM._call`` (run_full_evaluation_pipeline.py:80-106), the hierarchical runner's
sequential map (runners/run_summarization_ollama_mapreduce_hierarchical.py:128-141) and
the Ollama wire (`/api/generate`, pipeline.py:81-94).  The bar: what the batched paths
return is byte-identical to the reference's one-call-at-a-time order on the same engine.
"""
import asyncio
import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from mapsum import compat, template  # noqa: E402
from mapsum import hierarchical as hz  # noqa: E402
from mapsum.config import TINY  # noqa: E402
from mapsum.engine import Engine  # noqa: E402
from mapsum.mapreduce import reduce_prompt, run_map_reduce  # noqa: E402

NPRED = 24


@pytest.fixture(scope="module")
def toy():
    """Byte-level BPE padded with placeholder tokens to a multiple of 16 entries, so every
    id the model can emit decodes; its <|eot_id|> is the engine's EOS."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from mapsum.tokenizer import Tokenizer as MT
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    specials = ["<|begin_of_text|>", "<|eot_id|>", "<|start_header_id|>", "<|end_header_id|>"]
    tr = trainers.BpeTrainer(vocab_size=900, special_tokens=specials,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    corpus = [template.MAP_PROMPT_MAPREDUCE, template.MAP_PROMPT_HIERARCHICAL, hz.REDUCE_TEMPLATE_HIERARCHICAL,
              "Văn bản tiếng Việt về kinh tế, xã hội và lịch sử của đất nước."] * 4
    tk.train_from_iterator(corpus, tr)
    n = tk.get_vocab_size()
    tk.add_tokens([f"<x{i}>" for i in range((-n) % 16 + 16)])
    return MT.from_object(tk)


@pytest.fixture(scope="module")
def backend(toy):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = TINY.with_(vocab=toy.tk.get_vocab_size(), bos_id=toy.bos_id,
                     eos_ids=(toy.tk.token_to_id("<|eot_id|>"),))
    eng = Engine(cfg, device=0, max_batch=16, max_ctx=2048, max_prefill_tokens=8192)
    eng.init_synthetic(11, 0.05, 0.1)
    be = compat.MapBackend(eng, toy)
    compat.register_backend("mapsum:tiny", be)
    yield be
    compat._BACKENDS.pop("mapsum:tiny", None)
    eng.close()


def _llm(clean="pipeline"):
    return compat.OllamaLLM("http://localhost:11434", "mapsum:tiny", max_new_tokens=NPRED, clean=clean)


def _chunk(i, words=60):
    rng = np.random.default_rng(i)
    vocab = ["kinh", "tế", "xã", "hội", "lịch", "sử", "đất", "nước", "văn", "bản", "Việt", "Nam", "năm"]
    return " ".join(vocab[j] for j in rng.integers(0, len(vocab), size=words))


def test_call_is_engine_generate(backend, toy):
    """_call = template -> BPE -> libmapsum greedy -> detokenize -> clean_thinking_tokens."""
    from mapsum.postprocess import clean_thinking_tokens
    prompt = template.map_prompt("mapreduce", _chunk(0))
    ids = toy.encode(template.render_llama32(prompt, add_bos=False), add_bos=True)
    r = backend.engine.generate([ids], NPRED)[0]
    assert r.finish in ("eos", "length") and len(r.ids) <= NPRED
    assert _llm()._call(prompt) == clean_thinking_tokens(toy.decode(r.ids))


def test_async_fanout_equals_sequential_calls(backend):
    """The Send fan-out's concurrent ainvoke calls (one continuous batch on the GPU) return
    exactly what one-at-a-time _call returns (the reference's serialized order)."""
    m = _llm()
    prompts = [template.map_prompt("mapreduce", _chunk(i, 20 + 13 * i)) for i in range(7)]

    async def fan_out():
        return await asyncio.gather(*[m.ainvoke(p) for p in prompts])
    batched = asyncio.run(fan_out())
    assert batched == [m._call(p) for p in prompts]


def test_map_reduce_graph_on_gpu_equals_sequential(backend):
    """run_map_reduce (map fan-out, collapse, final reduce: mapreduce.py:75-181) through the
    GPU engine == the reference's node order with one call at a time."""
    m = _llm()
    contents = [_chunk(100 + i) for i in range(6)]
    tr = run_map_reduce(m, contents, token_max=40)
    sums = [m._call(template.map_prompt("mapreduce", c)) for c in contents]
    assert tr.summaries == sums
    collapsed = sums
    from mapsum.mapreduce import split_list_of_docs

    def length(docs):
        return sum(m.get_num_tokens(d) for d in docs)
    while length(collapsed) > 40:
        collapsed = [m._call(reduce_prompt(g)) for g in split_list_of_docs(collapsed, length, 40)]
    assert tr.final_summary == m._call(reduce_prompt(collapsed))


def test_hierarchical_on_gpu_equals_sequential(backend):
    """hierarchical_summarize_document (level-synchronous batches) through the GPU engine ==
    the hierarchical runner's strictly sequential order (:168-315), same cleaner."""
    m = _llm("hierarchical")

    def para(i):
        return {"type": "Paragraph", "text": _chunk(200 + i, 30 + 11 * i)}
    root = {"type": "Document", "text": "", "children": [
        {"type": "Header", "text": "Chương 1", "children": [para(0), {"type": "Header", "text": "1.1",
                                                                     "children": [para(1), para(2)]}]},
        {"type": "Header", "text": "Chương 2", "children": [para(3)]}]}
    a, b = copy.deepcopy(root), copy.deepcopy(root)
    got = asyncio.run(hz.hierarchical_summarize_document(a, max_depth=2, llm=m, chunk_size=50,
                                                         chunk_overlap=10))

    def summarize(text):
        sp = hz.RecursiveCharacterTextSplitter(50, 10, m.get_num_tokens, hz.SEPARATORS)
        sums = [m._call(template.map_prompt("mapreduce_hierarchical", c)) for c in sp.split_text(text)]
        return m._call(hz.reduce_prompt_text("\n\n".join(sums)))
    for d in range(min(2, hz.tree_depth(b)), 0, -1):
        for t in hz.collect_nodes_at_depth(b, d):
            title = t.get("text", "").strip()
            body = hz.extract_descendant_paragraph_text(t)
            if not body.strip():
                hz.replace_node_with_paragraph(t, title)
                continue
            s = summarize(f"{title}\n\n{body}" if title else body)
            hz.replace_node_with_paragraph(t, f"{title}:\n{s}" if title else s)
    want = m._call(hz.review_prompt_text(summarize(hz.extract_descendant_paragraph_text(b))))
    assert got == want and a == b


def test_ollama_wire_on_gpu(backend):
    """The reference's own request (pipeline.py:83-94) against the shim on the GPU engine;
    done_reason reports 'length' when num_predict cut the summary."""
    import requests
    from mapsum.server import OllamaShim
    prompt = template.map_prompt("mapreduce", _chunk(7))
    with OllamaShim({"mapsum:tiny": backend}, port=0) as s:
        payload = {"model": "mapsum:tiny", "prompt": prompt, "stream": False,
                   "options": {"num_predict": NPRED}}
        resp = requests.post(f"http://127.0.0.1:{s.port}/api/generate", json=payload, timeout=120)
        resp.raise_for_status()
        body = resp.json()
    from mapsum.postprocess import clean_thinking_tokens
    assert clean_thinking_tokens(body["response"]) == _llm()._call(prompt)
    r = backend.engine.generate([backend.encode_prompt(prompt)], NPRED)[0]
    assert body["done_reason"] == ("length" if r.finish == "length" else "stop")


def test_failed_chunk_is_isolated_and_requeued(toy):
    """SURVEY.md §5 failure row on the GPU: a chunk whose activations go non-finite (a NaN
    embedding row for one of its tokens) finishes MS_FINISH_ERROR on its own; the batch
    companions' summaries are unchanged, and the host re-queues the failed chunk once."""
    from mapsum import _lib as L
    from mapsum.weights import f32_to_f16_bits
    from oracle.synth import make_weights
    cfg = TINY.with_(vocab=toy.tk.get_vocab_size(), bos_id=toy.bos_id, eos_ids=())
    e = Engine(cfg, device=0, max_batch=4, max_ctx=512, max_prefill_tokens=2048)
    try:
        e.init_synthetic(11, 0.05, 0.1)
        rng = np.random.default_rng(3)
        good = [rng.integers(0, 300, size=n).astype(np.int32) for n in (40, 90, 70)]
        bad = np.concatenate([good[0][:20], [333], good[0][20:]]).astype(np.int32)
        before = e.generate(good, 8, ignore_eos=True)
        emb = make_weights(cfg.with_(n_layers=1), 11, std=0.05, jitter=0.1)["embed"].copy()
        emb[333] = np.nan
        e.load_tensor(L.MS_T_EMBED, 0, f32_to_f16_bits(emb))
        res = e.generate(good + [bad], 8, ignore_eos=True, retries=0)
        assert [r.ids for r in res[:3]] == [r.ids for r in before]
        assert res[3].finish == "error" and res[3].ids == []
        # with one retry the chunk is re-run once and fails again (the NaN row is permanent)
        st0 = e.stats()["finished"]
        res = e.generate([bad], 8, ignore_eos=True, retries=1)
        assert res[0].finish == "error" and e.stats()["finished"] - st0 == 2
    finally:
        e.close()
