"""Post-processing of the model response -- the summary string the runners see.

Two variants exist in the reference:
  * pipeline / critique / iterative runners (run_full_evaluation_pipeline.py:34-63):
    drop <think>/<thinking>/<thought>/<reasoning>/<analysis> blocks (DOTALL,
    IGNORECASE), fold runs of 3+ newline-separated blank lines to one blank line, strip;
  * hierarchical runner (runners/run_summarization_ollama_mapreduce_hierarchical.py:20-40):
    the same tag removal, then every whitespace run becomes one space.
"""
from __future__ import annotations

import re

_TAGS = ("think", "thinking", "thought", "reasoning", "analysis")
_TAG_RES = [re.compile(rf"<{t}>.*?</{t}>", re.DOTALL | re.IGNORECASE) for t in _TAGS]
_BLANKS = re.compile(r"\n\s*\n\s*\n")
_WS = re.compile(r"\s+")


def _drop_tags(text: str) -> str:
    for rx in _TAG_RES:  # applied in the reference's order, one pattern after another
        text = rx.sub("", text)
    return text


def clean_thinking_tokens(text: str) -> str:
    if not text:
        return text
    return _BLANKS.sub("\n\n", _drop_tags(text)).strip()


def clean_thinking_tokens_hierarchical(text: str) -> str:
    if not text:
        return text
    return _WS.sub(" ", _drop_tags(text)).strip()


CLEANERS = {"pipeline": clean_thinking_tokens, "hierarchical": clean_thinking_tokens_hierarchical,
            "none": lambda t: t}
