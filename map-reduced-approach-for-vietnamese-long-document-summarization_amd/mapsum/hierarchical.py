"""Hierarchical summarisation with level-synchronous batching.

Follows runners/run_summarization_ollama_mapreduce_hierarchical.py:
  collapse_level (:242-274)            every non-Paragraph node at one depth is summarised
                                       and replaced by a Paragraph "title:\\nsummary"
  summarize_text_mapreduce (:168-199)  split (RecursiveCharacterTextSplitter, word-count
                                       length, :178-186) -> map each chunk -> one reduce
  hierarchical_summarize_document (:277-315)  depths deepest..1, then the whole document,
                                       then one review/polish call

The reference awaits every target, and every chunk inside a target, one after another
(:132-141, :248-274).  All of them are independent, so here one depth is one batch: every
map prompt of every target at that depth is issued together, then every reduce prompt.
The engine is greedy and batch-invariant (one decode arithmetic per engine,
whatever the number of sequences in flight), so each call returns the string it would have
returned alone, and the tree ends up identical.
"""
from __future__ import annotations

import asyncio
import re

from .template import map_prompt

# :104-112 (the commented line is dropped by implicit concatenation, as in the reference)
REDUCE_TEMPLATE_HIERARCHICAL = (
    "Sau đây là một tập hợp các bản tóm tắt:\n<docs>\n{docs}\n</docs>\n\n"
    "Hãy tổng hợp và chắt lọc chúng thành một bản tóm tắt cuối cùng bằng **tiếng Việt**\n"
    "Lưu ý bao gồm đầy đủ các chi tiết quan trọng như sự kiện hay nhân vật, các chủ đề chính. "
    "Không bỏ sót thông tin quan trọng."
    "Chỉ viết nội dung tóm tắt. Không giải thích, không xin lỗi, không nói về quy trình."
    "Không sử dụng dấu đầu dòng; hãy viết thành các câu hoàn chỉnh theo đoạn văn."
    "Tóm tắt mới:"
)

# :297-311, a system message sent as ``.messages[0].content`` (bare text, :313)
REVIEW_TEMPLATE_HIERARCHICAL = (
    "Bạn là một biên tập viên chuyên nghiệp.\n"
    "Dưới đây là bản tóm tắt của một tài liệu:\n"
    "<summary>\n"
    "{summary}"
    "</summary>\n"
    "Hãy rà soát để sửa lỗi ngữ pháp và đảm bảo văn phong mạch lạc, rõ ràng. "
    "Không bỏ sót thông tin quan trọng.\n"
    "không cần giải thích, không cần xin lỗi, không cần nói về quy trình.\n"
    "Tóm tắt mới:\n"
)

SEPARATORS = ["\n\n", "\n", ".", "!", "?", ";", " ", ""]  # :183


def reduce_prompt_text(joined: str) -> str:
    """``REDUCE_PROMPT | llm`` (:128, :145-146): a human message rendered with its role
    prefix (EXT LangChain get_buffer_string), like the map prompt's "System: "."""
    return "Human: " + REDUCE_TEMPLATE_HIERARCHICAL.replace("{docs}", joined)


def review_prompt_text(summary: str) -> str:
    return REVIEW_TEMPLATE_HIERARCHICAL.replace("{summary}", summary)


# ---------------------------------------------------------------- text splitter
class RecursiveCharacterTextSplitter:
    """EXT langchain_text_splitters.RecursiveCharacterTextSplitter as published (unpinned:
    requirements.txt:10 pins no version), with the defaults the runner relies on:
    keep_separator=True (separator kept at the start of the next piece),
    is_separator_regex=False, strip_whitespace=True."""

    def __init__(self, chunk_size: int, chunk_overlap: int, length_function=len, separators=None):
        if chunk_overlap > chunk_size:
            raise ValueError("chunk_overlap larger than chunk_size")
        self.chunk_size, self.chunk_overlap = chunk_size, chunk_overlap
        self.length = length_function
        self.separators = list(separators or ["\n\n", "\n", " ", ""])

    @staticmethod
    def _split_keep(text: str, sep: str) -> list:
        if not sep:
            return [c for c in text]
        parts = re.split(f"({re.escape(sep)})", text)
        pieces = [parts[i] + parts[i + 1] for i in range(1, len(parts), 2)]
        if len(parts) % 2 == 0:
            pieces += parts[-1:]
        pieces = [parts[0]] + pieces
        return [p for p in pieces if p != ""]

    def _join(self, docs: list, sep: str):
        t = sep.join(docs).strip()
        return t or None

    def _merge(self, splits: list, sep: str) -> list:
        # the current window is splits[lo:hi] (LangChain keeps it as a list it pops from the
        # front; an index pair gives the same windows without the quadratic copies)
        sep_len = self.length(sep)
        docs, lo, hi, total = [], 0, 0, 0
        for d in splits:
            n = self.length(d)
            if total + n + (sep_len if hi > lo else 0) > self.chunk_size:
                if hi > lo:
                    doc = self._join(splits[lo:hi], sep)
                    if doc is not None:
                        docs.append(doc)
                    while total > self.chunk_overlap or (
                            total + n + (sep_len if hi > lo else 0) > self.chunk_size and total > 0):
                        total -= self.length(splits[lo]) + (sep_len if hi - lo > 1 else 0)
                        lo += 1
            hi += 1
            total += n + (sep_len if hi - lo > 1 else 0)
        doc = self._join(splits[lo:hi], sep)
        if doc is not None:
            docs.append(doc)
        return docs

    def _split(self, text: str, separators: list) -> list:
        out = []
        sep, rest = separators[-1], []
        for i, s in enumerate(separators):
            if s == "":
                sep = s
                break
            if re.search(re.escape(s), text):
                sep, rest = s, separators[i + 1:]
                break
        good = []
        pieces = self._split_keep(text, sep)
        prime = getattr(self.length, "prime", None)
        if prime is not None:  # a batched length function measures every piece in one call
            prime(pieces + [""])
        for piece in pieces:
            if self.length(piece) < self.chunk_size:
                good.append(piece)
                continue
            if good:
                out.extend(self._merge(good, ""))
                good = []
            out.extend(self._split(piece, rest) if rest else [piece])
        if good:
            out.extend(self._merge(good, ""))
        return out

    def split_text(self, text: str) -> list:
        return self._split(text, self.separators)


# ---------------------------------------------------------------- tree helpers (:202-240)
def depth_first_traverse(node: dict, callback, depth: int = 0, parent=None):
    callback(node, depth, parent)
    for child in node.get("children", []):
        depth_first_traverse(child, callback, depth + 1, node)


def collect_nodes_at_depth(root: dict, target_depth: int) -> list:
    nodes = []
    depth_first_traverse(root, lambda n, d, _p: nodes.append(n)
                         if d == target_depth and n.get("type") != "Paragraph" else None)
    return nodes


def extract_descendant_paragraph_text(node: dict) -> str:
    texts = []
    depth_first_traverse(node, lambda n, _d, _p: texts.append(n.get("text", ""))
                         if n.get("type") == "Paragraph" else None)
    return "\n\n".join(texts)


def replace_node_with_paragraph(node: dict, text: str):
    node.clear()
    node["type"] = "Paragraph"
    node["text"] = text


def tree_depth(n: dict, depth: int = 0) -> int:
    if not n.get("children"):
        return depth
    return max(tree_depth(c, depth + 1) for c in n["children"])


# ---------------------------------------------------------------- batched drivers
def _splitter(llm, chunk_size: int, chunk_overlap: int, max_context: int = 16384):
    size = min(chunk_size, int(max_context * 0.75))  # :176-177
    return RecursiveCharacterTextSplitter(size, chunk_overlap, llm.get_num_tokens, SEPARATORS)


async def summarize_texts_mapreduce(texts: list, llm, *, chunk_size: int = 12000,
                                    chunk_overlap: int = 200, max_context: int = 16384) -> list:
    """summarize_text_mapreduce (:168-199) for many texts at once: every map prompt of every
    text in one batch, then every reduce prompt in one batch."""
    sp = _splitter(llm, chunk_size, chunk_overlap, max_context)
    chunks = [sp.split_text(t) for t in texts]
    flat = [c for cs in chunks for c in cs]
    maps = await asyncio.gather(*(llm.ainvoke(map_prompt("mapreduce_hierarchical", c)) for c in flat))
    it = iter(maps)
    joined = ["\n\n".join(next(it) for _ in cs) for cs in chunks]
    return list(await asyncio.gather(*(llm.ainvoke(reduce_prompt_text(j)) for j in joined)))


async def collapse_level(root: dict, depth_level: int, llm, chunk_size: int = 12000,
                         chunk_overlap: int = 200) -> int:
    """:242-274 with the targets of one depth summarised as one batch."""
    targets = collect_nodes_at_depth(root, depth_level)
    work = []
    for t in targets:
        title = t.get("text", "").strip()
        body = extract_descendant_paragraph_text(t)
        if not body.strip():
            replace_node_with_paragraph(t, title)
            continue
        work.append((t, title, f"{title}\n\n{body}" if title else body))
    sums = await summarize_texts_mapreduce([w[2] for w in work], llm, chunk_size=chunk_size,
                                           chunk_overlap=chunk_overlap)
    for (t, title, _), s in zip(work, sums):
        replace_node_with_paragraph(t, f"{title}:\n{s}" if title else s)
    return len(targets)


async def hierarchical_summarize_document(document_node: dict, *, max_depth: int, llm,
                                          chunk_size: int = 12000, chunk_overlap: int = 200) -> str:
    """:277-315: collapse deepest..1, summarise the document, then one review call."""
    for d in range(min(max_depth, tree_depth(document_node)), 0, -1):
        await collapse_level(document_node, d, llm, chunk_size, chunk_overlap)
    final_text = extract_descendant_paragraph_text(document_node)
    (final,) = await summarize_texts_mapreduce([final_text], llm, chunk_size=chunk_size,
                                               chunk_overlap=chunk_overlap)
    return await llm.ainvoke(review_prompt_text(final))
