"""Checkpoint / resume: the reference's per-document file contract
(run_full_evaluation_pipeline.py:422-431, 568-570) and the per-call journal that lets a
crashed map phase resume without re-running finished chunks."""
import asyncio
import hashlib
import os

import pytest

from mapsum import mapreduce as mr
from mapsum.resume import CallJournal, JournaledLLM, call_key, summarize_dir


class FakeLLM:
    """Deterministic stand-in for OllamaLLM: a summary is a digest of its prompt; can be
    told to die after n calls (a crash in the middle of a map phase)."""
    model_name, clean, max_new_tokens = "fake:1b", "pipeline", 64

    def __init__(self, die_after=None):
        self.calls = []
        self.die_after = die_after

    def _gen(self, prompt):
        if self.die_after is not None and len(self.calls) >= self.die_after:
            raise RuntimeError("engine died")
        self.calls.append(prompt)
        return "tóm tắt " + hashlib.sha1(prompt.encode()).hexdigest()[:8]

    def invoke(self, prompt):
        return self._gen(prompt)

    async def ainvoke(self, prompt):
        await asyncio.sleep(0)
        return self._gen(prompt)

    def get_num_tokens(self, text):
        return len(text.split())


def _contents(n=12):
    return [f"đoạn văn số {i} " + "kinh tế xã hội " * (5 + i % 4) for i in range(n)]


def test_call_key_separates_fields():
    assert call_key("m", 8, "a", "bc") != call_key("m", 8, "ab", "c")
    assert call_key("m", 8, "a", "b") != call_key("m", 9, "a", "b")
    assert call_key("m", 8, "a", "b") == call_key("m", 8, "a", "b")


def test_journal_roundtrip_and_torn_line(tmp_path):
    p = tmp_path / "j" / "calls.jsonl"
    with CallJournal(str(p)) as j:
        j.put("k1", "d", "một")
        j.put("k2", "d", "hai")
        j.put("k1", "d", "ignored: first write wins")
    with open(p, "a", encoding="utf-8") as f:
        f.write('{"k": "k3", "doc": "d", "te')  # crash mid-write
    j = CallJournal(str(p))
    assert len(j) == 2 and j.get("k1") == "một" and j.get("k2") == "hai"
    assert j.torn_lines == 1 and "k3" not in j
    # a write after the torn line must survive the next reload (the fragment was cut away)
    j.put("k4", "d", "bốn")
    j.close()
    j = CallJournal(str(p))
    assert len(j) == 3 and j.get("k4") == "bốn" and j.torn_lines == 0
    j.close()


def test_journal_keeps_unicode_line_separators(tmp_path):
    """json.dumps(ensure_ascii=False) writes U+2028 / U+2029 / U+0085 unescaped: a record that
    holds one is still one record on reload (str.splitlines() tore it)."""
    p = tmp_path / "calls.jsonl"
    text = "dòng một\u2028dòng hai\u2029ba\x85bốn"
    with CallJournal(str(p)) as j:
        j.put("k1", "d", text)
        j.put("k2", "d", "hai")
    j = CallJournal(str(p))
    assert len(j) == 2 and j.get("k1") == text and j.torn_lines == 0
    j.close()


def test_crashed_map_phase_resumes_to_the_same_result(tmp_path):
    contents = _contents()
    want = mr.run_map_reduce(FakeLLM(), contents, token_max=40)
    path = str(tmp_path / "calls.jsonl")
    # first run dies after 7 of the 12 map calls
    with CallJournal(path) as j:
        with pytest.raises(RuntimeError):
            mr.run_map_reduce(JournaledLLM(FakeLLM(die_after=7), j, "doc1"), contents, token_max=40)
    with CallJournal(path) as j:
        assert len(j) == 7
        inner = FakeLLM()
        m = JournaledLLM(inner, j, "doc1")
        got = mr.run_map_reduce(m, contents, token_max=40)
    assert got.summaries == want.summaries and got.final_summary == want.final_summary
    assert m.hits == 7 and len(inner.calls) == m.misses
    # the engine saw only the calls the crashed run had not finished: 5 map calls + reduces
    from mapsum.template import map_prompt
    maps = [map_prompt("mapreduce", c) for c in contents]
    assert [c for c in inner.calls if c in maps] == [p for p in maps if p not in maps[:7]]
    # a third run is all hits
    with CallJournal(path) as j:
        inner = FakeLLM()
        m = JournaledLLM(inner, j, "doc1")
        again = mr.run_map_reduce(m, contents, token_max=40)
    assert again.final_summary == want.final_summary and inner.calls == [] and m.misses == 0


def test_journal_keys_are_per_doc_and_per_model(tmp_path):
    with CallJournal(str(tmp_path / "c.jsonl")) as j:
        a = JournaledLLM(FakeLLM(), j, "doc-a")
        a.invoke("cùng một prompt")
        b_inner = FakeLLM()
        b = JournaledLLM(b_inner, j, "doc-b")
        b.invoke("cùng một prompt")
        assert b.misses == 1  # another document's call is not reused
        other = FakeLLM()
        other.clean = "hierarchical"
        c = JournaledLLM(other, j, "doc-a")
        c.invoke("cùng một prompt")
        assert c.misses == 1  # another cleaner returns another string


def test_summarize_dir_file_contract(tmp_path):
    docs, refs, out = tmp_path / "docs", tmp_path / "refs", tmp_path / "out"
    for d in (docs, refs, out):
        d.mkdir()
    for name in ("a.txt", "b.txt", "c.txt", "d.txt"):
        (docs / name).write_text("văn bản " + name * 30, encoding="utf-8")
    for name in ("a.txt", "b.txt", "c.txt"):
        (refs / name).write_text("ref", encoding="utf-8")
    (out / "b.txt").write_text("đã có", encoding="utf-8")  # finished in an earlier run
    seen = []

    async def summarize(text, llm):
        seen.append(text[:20])
        return (await llm.ainvoke(text))

    res = summarize_dir(str(docs), str(out), summarize, journal_path=str(tmp_path / "j.jsonl"),
                        llm=FakeLLM(), refs_dir=str(refs))
    assert sorted(res) == ["a.txt", "b.txt", "c.txt"]  # d has no reference: skipped (:433-436)
    assert res["b.txt"] == "đã có" and len(seen) == 2  # b loaded, not re-run
    assert (out / "a.txt").read_text(encoding="utf-8") == res["a.txt"]
    assert not any(n.endswith(".tmp") for n in os.listdir(out))
    # rerun: everything loads from the files
    seen.clear()
    res2 = summarize_dir(str(docs), str(out), summarize, llm=FakeLLM(), refs_dir=str(refs))
    assert res2 == res and seen == []
