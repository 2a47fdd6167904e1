"""Checkpoint / resume for the map phase (SURVEY.md §5 'Checkpoint / resume' row).

The reference resumes per document: a summary file is written as soon as a document is
done, and documents whose output file exists are loaded instead of re-run
(run_full_evaluation_pipeline.py:422-431, written at :568-570; the map-reduce runner's
:240-250, 268-271).  ``summarize_dir`` keeps that file contract.

Below it, ``CallJournal`` adds what SURVEY.md §5 asks for at map-phase scale: every
generate call's output is appended to a JSONL journal the moment it returns, keyed by
(model, num_predict, doc id, prompt), so a run killed in the middle of a 4096-chunk map
phase re-issues only the calls that had not finished.  ``JournaledLLM`` wraps the drop-in
``OllamaLLM`` (or anything with ``ainvoke``/``invoke``/``get_num_tokens``): journaled
prompts return their stored text without touching the engine, the rest go through the
wrapped LLM as one batch exactly as before.  Greedy decoding is deterministic and
batch-invariant, so a resumed run returns the strings an uninterrupted run
would have returned.

The journal is append-only; a torn last line (a crash mid-write) is ignored on load.
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import os


def call_key(model: str, num_predict: int, doc_id: str, prompt: str) -> str:
    h = hashlib.sha256()
    for part in (model, str(int(num_predict)), doc_id, prompt):
        b = part.encode("utf-8")
        h.update(len(b).to_bytes(8, "little"))
        h.update(b)
    return h.hexdigest()


class CallJournal:
    """Append-only JSONL journal of finished generate calls: one line
    ``{"k": key, "doc": doc_id, "text": output}`` per call."""

    def __init__(self, path: str, fsync: bool = False):
        self.path = path
        self.fsync = fsync
        self._done: dict = {}
        self.torn_lines = 0
        if os.path.exists(path):
            # a crash mid-write leaves a torn last line with no newline: cut the file back to
            # the last complete record so the next put() starts on a fresh line (appending onto
            # the fragment would tear that record too); the torn call is simply re-run
            with open(path, "rb+") as f:
                data = f.read()
                keep = data.rfind(b"\n") + 1
                if keep < len(data):
                    f.truncate(keep)
                    self.torn_lines += 1
                    data = data[:keep]
            # records end in b"\n" only: str.splitlines() would also split on U+2028/U+2029/
            # U+0085, which json.dumps(ensure_ascii=False) writes unescaped inside a summary
            for raw in data.split(b"\n"):
                if not raw:
                    continue
                try:
                    rec = json.loads(raw.decode("utf-8", errors="replace"))
                    self._done[rec["k"]] = rec["text"]
                except (json.JSONDecodeError, KeyError, TypeError):
                    self.torn_lines += 1
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._f = open(path, "a", encoding="utf-8")

    def __len__(self) -> int:
        return len(self._done)

    def __contains__(self, key: str) -> bool:
        return key in self._done

    def get(self, key: str):
        return self._done.get(key)

    def put(self, key: str, doc_id: str, text: str) -> None:
        if key in self._done:
            return
        self._f.write(json.dumps({"k": key, "doc": doc_id, "text": text}, ensure_ascii=False) + "\n")
        self._f.flush()
        if self.fsync:
            os.fsync(self._f.fileno())
        self._done[key] = text

    def close(self) -> None:
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class JournaledLLM:
    """``llm`` with every call journaled under ``doc_id`` (one wrapper per document)."""

    def __init__(self, llm, journal: CallJournal, doc_id: str, model: str | None = None,
                 num_predict: int | None = None):
        self.llm = llm
        self.journal = journal
        self.doc_id = doc_id
        # the cleaner is part of what a call returns (compat.OllamaLLM.clean)
        self.model = model if model is not None else f"{getattr(llm, 'model_name', '')}|{getattr(llm, 'clean', '')}"
        self.num_predict = int(num_predict if num_predict is not None else getattr(llm, "max_new_tokens", 0))
        self.hits = 0
        self.misses = 0

    def _key(self, prompt: str) -> str:
        return call_key(self.model, self.num_predict, self.doc_id, prompt)

    def get_num_tokens(self, text: str) -> int:
        return self.llm.get_num_tokens(text)

    async def ainvoke(self, prompt: str, **kw) -> str:
        k = self._key(prompt)
        got = self.journal.get(k)
        if got is not None:
            self.hits += 1
            return got
        self.misses += 1
        text = await self.llm.ainvoke(prompt, **kw)
        self.journal.put(k, self.doc_id, text)
        return text

    def invoke(self, prompt: str, **kw) -> str:
        k = self._key(prompt)
        got = self.journal.get(k)
        if got is not None:
            self.hits += 1
            return got
        self.misses += 1
        text = self.llm.invoke(prompt, **kw)
        self.journal.put(k, self.doc_id, text)
        return text

    __call__ = invoke


def summarize_dir(docs_dir: str, out_dir: str, summarize, journal_path: str | None = None,
                  llm=None, refs_dir: str | None = None) -> dict:
    """The reference's document loop with its resume contract (pipeline.py:417-431, 568-570):
    documents in sorted file order; an existing output file is loaded, not re-run; a
    document without a reference summary (when ``refs_dir`` is given) is skipped; every
    new summary is written as soon as it is done.

    ``summarize(text, llm) -> str`` (or a coroutine function) produces one document's
    summary, e.g. ``lambda t, m: mapreduce.asummarize_document_mapreduce(t, m, splitter)``.
    With ``journal_path`` every call of ``llm`` is journaled per document (``JournaledLLM``),
    so a document interrupted half-way resumes at call granularity.

    Returns {file name: summary} for every document with an output."""
    os.makedirs(out_dir, exist_ok=True)
    journal = CallJournal(journal_path) if journal_path else None
    out = {}
    try:
        for fname in sorted(os.listdir(docs_dir)):
            src, dst = os.path.join(docs_dir, fname), os.path.join(out_dir, fname)
            if not os.path.isfile(src):
                continue
            if os.path.isfile(dst):  # :422-431
                with open(dst, "r", encoding="utf-8") as f:
                    out[fname] = f.read()
                continue
            if refs_dir is not None and not os.path.isfile(os.path.join(refs_dir, fname)):
                continue
            with open(src, "r", encoding="utf-8") as f:
                text = f.read()
            m = JournaledLLM(llm, journal, fname) if (journal is not None and llm is not None) else llm
            s = summarize(text, m)
            if asyncio.iscoroutine(s):
                s = asyncio.run(s)
            tmp = dst + ".tmp"
            with open(tmp, "w", encoding="utf-8") as f:  # :568-570, atomically
                f.write(s)
            os.replace(tmp, dst)
            out[fname] = s
    finally:
        if journal is not None:
            journal.close()
    return out
