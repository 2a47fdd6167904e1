"""CPU tests of the level-synchronous hierarchical driver (mapsum/hierarchical.py, SURVEY.md
§8f row 2) against a sequential restatement of
runners/run_summarization_ollama_mapreduce_hierarchical.py:168-315.

The text splitter restates langchain_text_splitters (absent here, version unpinned by the
reference): its known answers below are derived by hand from the published algorithm, so
splitter parity with the real library is unpinned."""
import asyncio
import copy
import hashlib
import json
import os

import pytest

from mapsum import hierarchical as hz
from mapsum.template import map_prompt
from test_mapreduce import ToyLLM

HERE = os.path.dirname(os.path.abspath(__file__))


def test_prompts_bytes_pinned():
    fx = json.load(open(os.path.join(HERE, "golden", "prompts.json"), encoding="utf-8"))
    for key, s in (("reduce_hierarchical", hz.REDUCE_TEMPLATE_HIERARCHICAL),
                   ("review_hierarchical", hz.REVIEW_TEMPLATE_HIERARCHICAL)):
        assert len(s) == fx[key]["n_chars"], key
        assert hashlib.sha256(s.encode()).hexdigest() == fx[key]["sha256"], key


@pytest.mark.parametrize("text,size,overlap,want", [
    ("abc def ghi jkl", 10, 0, ["abc def", "ghi jkl"]),
    ("abc def ghi jkl", 10, 4, ["abc def", "def ghi", "ghi jkl"]),
    ("abcdefghijkl mn", 5, 0, ["abcde", "fghij", "kl", "mn"]),
    ("a\n\nb c\n\nd", 100, 0, ["a\n\nb c\n\nd"]),
    ("", 10, 0, []),
])
def test_splitter_known_answers(text, size, overlap, want):
    sp = hz.RecursiveCharacterTextSplitter(size, overlap, len, ["\n\n", "\n", " ", ""])
    assert sp.split_text(text) == want


def test_splitter_word_length_properties():
    words = [f"từ{i}" for i in range(5000)]
    text = "\n\n".join(" ".join(words[i:i + 37]) + "." for i in range(0, 5000, 37))
    n = lambda s: len(s.split())  # noqa: E731  (pipeline.py:115-117)
    sp = hz.RecursiveCharacterTextSplitter(600, 50, n, hz.SEPARATORS)
    chunks = sp.split_text(text)
    assert len(chunks) > 1 and all(n(c) <= 600 for c in chunks)
    # every word is covered, in order; consecutive chunks overlap
    seen = [w for c in chunks for w in c.replace(".", " ").split()]
    assert sorted(set(seen), key=lambda w: int(w[2:])) == words
    assert any(set(a.split()) & set(b.split()) for a, b in zip(chunks, chunks[1:]))
    with pytest.raises(ValueError):
        hz.RecursiveCharacterTextSplitter(10, 20)


def _tree(seed=0):
    import random
    rnd = random.Random(seed)

    def para():
        return {"type": "Paragraph", "text": " ".join(f"w{rnd.randrange(10**6)}" for _ in range(rnd.randrange(20, 200)))}

    def header(title, depth):
        kids = [para() for _ in range(rnd.randrange(1, 4))]
        if depth < 2:
            kids += [header(f"{title}.{j}", depth + 1) for j in range(rnd.randrange(1, 3))]
        return {"type": "Header", "text": title, "children": kids}

    return {"type": "Document", "text": "", "children": [header(f"Chương {i}", 1) for i in range(3)]
            + [{"type": "Header", "text": "Rỗng", "children": []}]}


def reference_sequential(llm, root, max_depth, chunk_size, overlap):
    """:168-315 in the reference's order: targets one after another, chunks one after
    another (answers come from the same deterministic ToyLLM function)."""
    def summarize(text):
        sp = hz.RecursiveCharacterTextSplitter(min(chunk_size, int(16384 * 0.75)), overlap,
                                               llm.get_num_tokens, hz.SEPARATORS)
        sums = [llm._answer(map_prompt("mapreduce_hierarchical", c)) for c in sp.split_text(text)]
        return llm._answer(hz.reduce_prompt_text("\n\n".join(sums)))

    for d in range(min(max_depth, hz.tree_depth(root)), 0, -1):
        for t in hz.collect_nodes_at_depth(root, d):
            title = t.get("text", "").strip()
            body = hz.extract_descendant_paragraph_text(t)
            if not body.strip():
                hz.replace_node_with_paragraph(t, title)
                continue
            s = summarize(f"{title}\n\n{body}" if title else body)
            hz.replace_node_with_paragraph(t, f"{title}:\n{s}" if title else s)
    final = summarize(hz.extract_descendant_paragraph_text(root))
    return llm._answer(hz.review_prompt_text(final))


@pytest.mark.parametrize("max_depth,chunk_size", [(2, 12000), (2, 60), (1, 80), (5, 45)])
def test_level_synchronous_matches_sequential(max_depth, chunk_size):
    root_a, root_b = _tree(1), _tree(1)
    llm = ToyLLM()
    got = asyncio.run(hz.hierarchical_summarize_document(root_a, max_depth=max_depth, llm=llm,
                                                         chunk_size=chunk_size, chunk_overlap=10))
    want = reference_sequential(ToyLLM(), root_b, max_depth, chunk_size, 10)
    assert got == want
    assert root_a == root_b  # the collapsed trees are identical too
    if chunk_size < 100:
        assert llm.peak > 3, "a level's map prompts should be in flight together"


def test_empty_section_keeps_title():
    root = {"type": "Document", "children": [{"type": "Header", "text": " Mục ", "children": []},
                                             {"type": "Header", "text": "B", "children": [
                                                 {"type": "Paragraph", "text": "một hai ba"}]}]}
    r = copy.deepcopy(root)
    asyncio.run(hz.collapse_level(r, 1, ToyLLM()))
    assert r["children"][0] == {"type": "Paragraph", "text": "Mục"}
    assert r["children"][1]["type"] == "Paragraph" and r["children"][1]["text"].startswith("B:\n")
