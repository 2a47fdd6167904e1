"""Host-side chunking of the map phase.

The pipeline splits every document with
    RecursiveCharacterTextSplitter(chunk_size=12000, chunk_overlap=200,
        length_function=lambda t: len(tokenizer.encode(t)),
        separators=["\\n\\n", "\\n", ".", "!", "?", ";", " ", ""])
(run_full_evaluation_pipeline.py:344-361; chunk_size/overlap from its config :994-998),
tokenizer = the HF Llama-3.2 tokenizer.  ``encode`` adds BOS by default, so a piece's
length is its token count + 1, and the splitter calls the length function once per
candidate piece at every recursion level -- one Python -> Rust round trip per piece.  At
the GPU's 100+ chunks/s that serial host loop would become the bottleneck.

``TokenLength`` keeps the exact semantics (same tokenizer, same +1) but measures the
pieces of one recursion level in ONE ``encode_batch`` call (HF tokenizers: Rust, all
cores, GIL released) and memoises them; the splitter (mapsum.hierarchical's restatement of
the published LangChain algorithm) asks it to ``prime`` each level.  Same chunks, fewer
round trips: tests/test_splitter.py checks equality with the unbatched function,
tools/bench_splitter.py measures the throughput.
"""
from __future__ import annotations

from .hierarchical import SEPARATORS, RecursiveCharacterTextSplitter

PIPELINE_CHUNK_SIZE = 12000    # run_full_evaluation_pipeline.py:994-998
PIPELINE_CHUNK_OVERLAP = 200


class TokenLength:
    """``len(tokenizer.encode(text))`` of the pipeline, memoised and batchable.

    tokenizer: mapsum.tokenizer.Tokenizer (encode / encode_batch with add_bos)."""

    def __init__(self, tokenizer, add_special_tokens: bool = True, max_cache: int = 1 << 20):
        self.tok = tokenizer
        self.add = add_special_tokens
        self.cache: dict = {}
        self.max_cache = max_cache
        self.calls = self.batches = 0

    def __call__(self, text: str) -> int:
        n = self.cache.get(text)
        if n is None:
            self.calls += 1
            n = len(self.tok.encode(text, add_bos=self.add))
            self._put(text, n)
        return n

    def prime(self, texts) -> None:
        todo = list(dict.fromkeys(t for t in texts if t not in self.cache))
        if not todo:
            return
        self.batches += 1
        for t, ids in zip(todo, self.tok.encode_batch(todo, add_bos=self.add)):
            self._put(t, len(ids))

    def _put(self, text, n):
        if len(self.cache) >= self.max_cache:
            self.cache.clear()
        self.cache[text] = n


def pipeline_splitter(tokenizer, chunk_size: int = PIPELINE_CHUNK_SIZE,
                      chunk_overlap: int = PIPELINE_CHUNK_OVERLAP) -> RecursiveCharacterTextSplitter:
    """The map-reduce pipeline's token-length splitter (run_full_evaluation_pipeline.py:356-361)."""
    return RecursiveCharacterTextSplitter(chunk_size, chunk_overlap, TokenLength(tokenizer), SEPARATORS)


def split_documents(texts, tokenizer, chunk_size: int = PIPELINE_CHUNK_SIZE,
                    chunk_overlap: int = PIPELINE_CHUNK_OVERLAP) -> list:
    """Chunks of many documents with one shared length cache (text_splitter.split_documents
    applied per document, as summarize_document_mapreduce does at mapreduce.py:187-188)."""
    sp = pipeline_splitter(tokenizer, chunk_size, chunk_overlap)
    return [sp.split_text(t) for t in texts]
