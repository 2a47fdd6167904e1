"""Generate tests/golden/prompts.json: SHA-256 of the reference's map-prompt strings.

Reads the reference runners as TEXT (ast string constants; nothing is imported or run)
and records the digest of the exact map-prompt constant each runner formats per chunk (and the map-reduce
runner's reduce prompt),
so tests/test_host.py can check mapsum/template.py byte for byte without the
reference being present (it is absent on the GPU box).
"""
import ast
import hashlib
import json
import os

REF = "/root/reference/runners"
HERE = os.path.dirname(os.path.abspath(__file__))
SRC = {"mapreduce": ("run_summarization_ollama_mapreduce.py", "Vui lòng viết một bản tóm tắt chi tiết cho đoạn"),
       "mapreduce_critique": ("run_summarization_ollama_mapreduce_critique.py", "Văn bản:\n<content>"),
       "mapreduce_hierarchical": ("run_summarization_ollama_mapreduce_hierarchical.py", "<content>\n{content}\n\n</content>"),
       # the reduce prompt of the map-reduce graph (mapreduce.py:88-94), for mapsum/mapreduce.py
       "reduce_mapreduce": ("run_summarization_ollama_mapreduce.py", "Sau đây là một tập hợp các bản tóm tắt:\n{docs}"),
       # mapsum/hierarchical.py: reduce (:104-112) and review (:297-311) prompts
       "reduce_hierarchical": ("run_summarization_ollama_mapreduce_hierarchical.py", "Sau đây là một tập hợp các bản tóm tắt:\n<docs>"),
       "review_hierarchical": ("run_summarization_ollama_mapreduce_hierarchical.py", "Bạn là một biên tập viên chuyên nghiệp")}


def main():
    out = {}
    for key, (fname, marker) in SRC.items():
        tree = ast.parse(open(os.path.join(REF, fname), encoding="utf-8").read())
        hits = [n.value for n in ast.walk(tree)
                if isinstance(n, ast.Constant) and isinstance(n.value, str) and marker in n.value]
        assert len(hits) == 1, (key, len(hits))
        out[key] = {"file": f"runners/{fname}", "sha256": hashlib.sha256(hits[0].encode()).hexdigest(),
                    "n_chars": len(hits[0])}
    json.dump(out, open(os.path.join(HERE, "prompts.json"), "w"), indent=1, ensure_ascii=False)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
