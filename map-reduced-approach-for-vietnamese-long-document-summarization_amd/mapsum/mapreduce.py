"""Map -> collect -> collapse* -> reduce for one document, driven on the engine.

Mirrors the LangGraph in runners/run_summarization_ollama_mapreduce.py:75-181 (SURVEY.md
§8f row 1) without LangGraph/LangChain, which are not installed here:

  generate_summary (map node, :103-106)      one map prompt per chunk via ``llm.ainvoke``
  map_summaries (Send fan-out, :109-112)     all chunks issued at once -> one engine batch
  collect_summaries (:114-117)               summaries in chunk order
  should_collapse (:146-154)                 whitespace-word count (``get_num_tokens``) > token_max
  collapse_summaries (:130-144)              split_list_of_docs groups, one reduce call each
  generate_final_summary (:157-165)          reduce prompt over the collapsed summaries

Differences that do not change any string the reference produces:
- The reference awaits collapse groups one after another (:134-135).  Each group's
  reduce call depends only on its own group, and the engine is greedy and batch-invariant
  (DESIGN.md §5), so the groups are issued together and land in one batch.
- ``acollapse_docs`` also merges Document metadata; the map path carries none, so only
  the page_content survives here.
"""
from __future__ import annotations

import asyncio
from dataclasses import dataclass, field

# runners/run_summarization_ollama_mapreduce.py:88-94 -- the human message of reduce_prompt;
# ``prompt.messages[0].content`` after formatting {docs} is what reaches the LLM (:124-125).
REDUCE_PROMPT_MAPREDUCE = (
    "\n"
    "Sau đây là một tập hợp các bản tóm tắt:\n"
    "{docs}\n"
    "\n"
    "Hãy tổng hợp và chắt lọc chúng thành một bản tóm tắt cuối cùng, toàn diện về các chủ đề "
    "chính bằng tiếng Việt.\n"
    "Không sử dụng dấu đầu dòng, hãy viết bằng câu đầy đủ và theo đoạn văn.\n"
)


def reduce_prompt(docs: list) -> str:
    """:119-125: summaries joined by a blank line, substituted into the reduce template."""
    return REDUCE_PROMPT_MAPREDUCE.replace("{docs}", "\n\n".join(docs))


def split_list_of_docs(docs: list, length_func, token_max: int) -> list:
    """EXT langchain ``split_list_of_docs`` (called at :131-133), as published: grow a
    group until adding the next doc pushes ``length_func(group)`` past token_max, then
    start a new group with that doc.  A single doc over the limit is an error."""
    groups, cur = [], []
    for d in docs:
        cur.append(d)
        if length_func(cur) > token_max:
            if len(cur) == 1:
                raise ValueError("A single document was longer than the context length,"
                                 " we cannot handle this.")
            groups.append(cur[:-1])
            cur = cur[-1:]
    groups.append(cur)
    return groups


class GraphRecursionError(RuntimeError):
    """Raised where LangGraph would stop the run for exceeding ``recursion_limit``
    (summarize_document_mapreduce passes 10, :196)."""


@dataclass
class MapReduceTrace:
    """What each node produced, for tests and logging."""
    summaries: list = field(default_factory=list)
    collapses: list = field(default_factory=list)  # list of group sizes per collapse round
    final_summary: str = ""
    supersteps: int = 0


async def arun_map_reduce(llm, contents: list, token_max: int = 1000, recursion_limit: int = 10,
                          map_prompt=None) -> MapReduceTrace:
    """The graph of create_map_reduce_graph(llm, token_max) (:75-181) over ``contents``.

    ``llm`` is anything with ``ainvoke(str) -> str`` and ``get_num_tokens(str)`` -- the
    drop-in ``mapsum.compat.OllamaLLM`` in production.  ``map_prompt(chunk) -> str`` defaults
    to the mapreduce runner's prompt (:79-86, template.MAP_PROMPT_MAPREDUCE)."""
    if map_prompt is None:
        from .template import map_prompt as _mp
        map_prompt = lambda c: _mp("mapreduce", c)  # noqa: E731

    def length_function(docs):  # :98-100
        return sum(llm.get_num_tokens(d) for d in docs)

    tr = MapReduceTrace()

    def tick():
        tr.supersteps += 1
        if tr.supersteps > recursion_limit:
            raise GraphRecursionError(f"Recursion limit of {recursion_limit} reached")

    # superstep: every generate_summary node (the Send fan-out) runs concurrently
    tick()
    tr.summaries = list(await asyncio.gather(*(llm.ainvoke(map_prompt(c)) for c in contents)))
    tick()  # collect_summaries
    collapsed = list(tr.summaries)
    while length_function(collapsed) > token_max:
        tick()  # collapse_summaries
        groups = split_list_of_docs(collapsed, length_function, token_max)
        tr.collapses.append([len(g) for g in groups])
        collapsed = list(await asyncio.gather(*(llm.ainvoke(reduce_prompt(g)) for g in groups)))
    tick()  # generate_final_summary
    tr.final_summary = str(await llm.ainvoke(reduce_prompt(collapsed)))
    return tr


def run_map_reduce(llm, contents: list, token_max: int = 1000, recursion_limit: int = 10,
                   map_prompt=None) -> MapReduceTrace:
    """Synchronous entry (a fresh event loop), like ``asyncio.run(summarize_document_mapreduce)``."""
    return asyncio.run(arun_map_reduce(llm, contents, token_max, recursion_limit, map_prompt))


async def asummarize_document_mapreduce(doc_text: str, llm, text_splitter, token_max: int = 1000,
                                        recursion_limit: int = 10) -> str:
    """summarize_document_mapreduce (runners/run_summarization_ollama_mapreduce.py:183-201):
    split the document (``text_splitter.split_documents`` of one Document == split_text of
    its text), then the map-reduce graph; returns the final summary."""
    contents = text_splitter.split_text(doc_text)
    tr = await arun_map_reduce(llm, contents, token_max=token_max, recursion_limit=recursion_limit)
    return tr.final_summary
