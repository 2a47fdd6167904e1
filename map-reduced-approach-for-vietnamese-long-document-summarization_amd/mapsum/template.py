"""Prompt strings of the map call, byte for byte.

Two layers produce the text that reaches the model:
  1. the runner's map prompt around one chunk (reference, quoted verbatim below), and
  2. Ollama's chat template for llama3.2 around that prompt (EXT: Ollama's
     ``llama3.2`` TEMPLATE; not vendored, not pinned -- SURVEY.md §7 hard part 2).
Greedy parity with Ollama needs both to be exact, so they live here as data.
"""
from __future__ import annotations

# runners/run_summarization_ollama_mapreduce.py:79-86 -- sent as prompt.messages[0].content
# (the bare system text, no role prefix; :104-105)
MAP_PROMPT_MAPREDUCE = (
    "Bạn là một chuyên gia tóm tắt nội dung.\n"
    "Vui lòng viết một bản tóm tắt chi tiết cho đoạn văn bản sau bằng **tiếng Việt**.\n"
    "\n"
    "{content}\n"
    "\n"
    "Lưu ý: Không sử dụng dấu đầu dòng, hãy viết bằng câu đầy đủ và theo đoạn văn."
)

# runners/run_summarization_ollama_mapreduce_critique.py:118-130 (same .messages[0].content use, :207-210)
MAP_PROMPT_CRITIQUE = (
    "Hãy tóm tắt những thông tin quan trọng từ đoạn văn bản sau bằng tiếng Việt.\n"
    "        Lưu ý bao gồm đầy đủ các chi tiết quan trọng như sự kiện hay nhân vật, các chủ đề chính. "
    "Không bỏ sót thông tin quan trọng. Nên tóm tắt theo từng chương nếu có.\n"
    "\n"
    "Chỉ viết nội dung tóm tắt. Không giải thích, không xin lỗi, không nói về quy trình.\n"
    "\n"
    "Văn bản:\n"
    "<content>\n"
    "{content}\n"
    "</content>\n"
    "\n"
    "Tóm tắt:"
)

# runners/run_summarization_ollama_mapreduce_hierarchical.py:83-103 (commented lines dropped by
# Python's implicit concatenation, as in the reference)
MAP_PROMPT_HIERARCHICAL = (
    "Bạn là một chuyên gia tóm tắt nội dung. Hãy tóm tắt những thông tin quan trọng từ đoạn văn bản "
    "sau bằng tiếng Việt.\n"
    "Lưu ý bao gồm đầy đủ các chi tiết quan trọng như sự kiện hay nhân vật, các chủ đề chính. "
    "Không bỏ sót thông tin quan trọng. Nên tóm tắt theo từng chương nếu có."
    "<content>\n"
    "{content}\n\n"
    "</content>\n\n"
    "Chỉ viết nội dung tóm tắt. Không giải thích, không xin lỗi, không nói về quy trình.\n"
    "Tóm tắt:"
)

MAP_PROMPTS = {"mapreduce": MAP_PROMPT_MAPREDUCE, "mapreduce_critique": MAP_PROMPT_CRITIQUE,
               "mapreduce_hierarchical": MAP_PROMPT_HIERARCHICAL}


def map_prompt(approach: str, chunk: str) -> str:
    """The exact string a runner hands to ``llm`` for one chunk.

    mapreduce / critique send ``prompt.messages[0].content`` (bare text).  The
    hierarchical runner pipes a ChatPromptTemplate into the LLM (``MAP_PROMPT | llm``,
    hierarchical.py:128), which LangChain renders with ``get_buffer_string`` -- a
    "System: " role prefix (EXT LangChain semantics)."""
    text = MAP_PROMPTS[approach].replace("{content}", chunk)
    if approach == "mapreduce_hierarchical":
        return "System: " + text
    return text


# EXT: Ollama's llama3.2 TEMPLATE for /api/generate without system prompt or tools.
BOS = "<|begin_of_text|>"
LLAMA32_TEMPLATE = ("<|start_header_id|>system<|end_header_id|>\n\n"
                    "Cutting Knowledge Date: December 2023\n\n"
                    "<|eot_id|><|start_header_id|>user<|end_header_id|>\n\n"
                    "{prompt}<|eot_id|><|start_header_id|>assistant<|end_header_id|>\n\n")
STOP_STRINGS = ("<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>")


def render_llama32(prompt: str, add_bos: bool = True) -> str:
    return (BOS if add_bos else "") + LLAMA32_TEMPLATE.replace("{prompt}", prompt)
