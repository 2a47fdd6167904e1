"""CPU tests of the map -> collapse -> reduce driver (mapsum/mapreduce.py, SURVEY.md §8f
row 1) against a sequential restatement of the reference graph
(runners/run_summarization_ollama_mapreduce.py:75-181)."""
import asyncio
import hashlib
import json
import os

import pytest

from mapsum import compat, template
from mapsum.mapreduce import (GraphRecursionError, REDUCE_PROMPT_MAPREDUCE, reduce_prompt,
                              run_map_reduce, split_list_of_docs)

HERE = os.path.dirname(os.path.abspath(__file__))


class ToyLLM:
    """Deterministic async LLM: the 'summary' of a prompt is the first ``k`` words of the
    text between the prompt's last blank line pair, tagged by a digest of the prompt.
    Records every prompt and the peak number of calls in flight."""

    def __init__(self, k=6):
        self.k, self.prompts, self.inflight, self.peak = k, [], 0, 0

    def get_num_tokens(self, text):  # pipeline.py:115-117, verbatim semantics
        return len(text.split())

    def _answer(self, prompt):
        words = prompt.split()
        h = hashlib.sha256(prompt.encode()).hexdigest()[:6]
        return " ".join([h] + words[len(words) // 3: len(words) // 3 + self.k - 1])

    async def ainvoke(self, prompt):
        self.prompts.append(prompt)
        self.inflight += 1
        self.peak = max(self.peak, self.inflight)
        await asyncio.sleep(0)
        self.inflight -= 1
        return self._answer(prompt)


def reference_sequential(llm, contents, token_max):
    """The reference's node order, one call at a time (mapreduce.py:103-165), with the
    published langchain split_list_of_docs / acollapse_docs semantics."""
    def length(docs):
        return sum(llm.get_num_tokens(d) for d in docs)

    def reduce(docs):
        return llm._answer(REDUCE_PROMPT_MAPREDUCE.format(docs="\n\n".join(docs)))

    summaries = [llm._answer(template.map_prompt("mapreduce", c)) for c in contents]
    collapsed = summaries
    while length(collapsed) > token_max:
        groups, cur = [], []
        for d in collapsed:
            cur.append(d)
            if length(cur) > token_max:
                groups.append(cur[:-1])
                cur = cur[-1:]
        groups.append(cur)
        collapsed = [reduce(g) for g in groups]
    return reduce(collapsed)


def _doc(n_chunks, words=40):
    return [" ".join(f"từ{i}_{j}" for j in range(words)) for i in range(n_chunks)]


def test_reduce_prompt_bytes_pinned():
    fx = json.load(open(os.path.join(HERE, "golden", "prompts.json"), encoding="utf-8"))["reduce_mapreduce"]
    assert len(REDUCE_PROMPT_MAPREDUCE) == fx["n_chars"]
    assert hashlib.sha256(REDUCE_PROMPT_MAPREDUCE.encode()).hexdigest() == fx["sha256"]
    p = reduce_prompt(["a", "b"])
    assert "a\n\nb" in p and "{docs}" not in p


def test_split_list_of_docs_grouping():
    n = lambda docs: sum(len(d.split()) for d in docs)  # noqa: E731
    docs = ["a b c", "d e", "f g h i", "j"]
    assert split_list_of_docs(docs, n, 5) == [["a b c", "d e"], ["f g h i", "j"]]
    assert split_list_of_docs(docs, n, 100) == [docs]
    assert split_list_of_docs([], n, 5) == [[]]
    with pytest.raises(ValueError):
        split_list_of_docs(["a b c d e f"], n, 5)


@pytest.mark.parametrize("n_chunks,token_max", [(1, 1000), (8, 1000), (8, 20), (16, 14)])
def test_map_reduce_matches_sequential_reference(n_chunks, token_max):
    contents = _doc(n_chunks)
    llm = ToyLLM()
    tr = run_map_reduce(llm, contents, token_max=token_max)
    assert tr.final_summary == reference_sequential(ToyLLM(), contents, token_max)
    assert len(tr.summaries) == n_chunks
    # the whole Send fan-out is in flight at once (one engine batch)
    assert llm.peak >= n_chunks
    if token_max < 6 * n_chunks:
        assert tr.collapses, "expected at least one collapse round"


def test_recursion_limit():
    # summaries never shrink below the limit -> LangGraph would stop at recursion_limit
    class Wordy(ToyLLM):
        def _answer(self, prompt):
            return " ".join(["x"] * 12)
    with pytest.raises((GraphRecursionError, ValueError)):
        run_map_reduce(Wordy(), _doc(4), token_max=20, recursion_limit=10)


def test_map_reduce_through_ollamallm_batches(toy_tokenizer_mr):
    """Through the drop-in OllamaLLM + MapBackend: the map fan-out reaches the engine as
    one batch of all chunks."""
    from test_host import FakeEngine
    eng = FakeEngine()
    compat.register_backend("fake:mr", compat.MapBackend(eng, toy_tokenizer_mr))
    try:
        m = compat.OllamaLLM("http://localhost:11434", "fake:mr", max_new_tokens=64)
        tr = run_map_reduce(m, _doc(8, words=10), token_max=10_000)
        assert eng.batches[0] == 8 and len(tr.summaries) == 8
        assert isinstance(tr.final_summary, str)
    finally:
        compat._BACKENDS.pop("fake:mr", None)


@pytest.fixture(scope="module")
def toy_tokenizer_mr():
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    specials = ["<|begin_of_text|>", "<|eot_id|>", "<|start_header_id|>", "<|end_header_id|>"]
    tr = trainers.BpeTrainer(vocab_size=300, special_tokens=specials,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator([template.MAP_PROMPT_MAPREDUCE, REDUCE_PROMPT_MAPREDUCE] * 4, tr)
    from mapsum.tokenizer import Tokenizer as MT
    return MT.from_object(tk)
