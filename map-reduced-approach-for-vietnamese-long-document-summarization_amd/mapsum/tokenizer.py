"""Text <-> ids for the map call (the part of /api/generate before prefill and after decode).

Llama-3.2 uses a 128256-entry byte-level BPE (tiktoken-style pre-tokenizer regex,
BOS 128000, <|eot_id|> 128009).  The tokenizer files are not in this container
(SURVEY.md §8c), so this wraps any HF ``tokenizer.json`` through the ``tokenizers``
library (Rust BPE, releases the GIL); point ``MAPSUM_TOKENIZER`` or the constructor
at the Llama-3.2 file.  Special tokens written in the rendered template text
(``<|eot_id|>`` ...) are matched as added tokens, as llama.cpp does with parse_special.
"""
from __future__ import annotations

import os


class Tokenizer:
    def __init__(self, path: str | None = None, bos_id: int | None = None):
        from tokenizers import Tokenizer as _T
        path = path or os.environ.get("MAPSUM_TOKENIZER")
        if not path or not os.path.exists(path):
            raise FileNotFoundError("no tokenizer.json: pass a path or set MAPSUM_TOKENIZER "
                                    "(the Llama-3.2 tokenizer is not bundled)")
        self.tk = _T.from_file(path)
        self.bos_id = bos_id if bos_id is not None else self.tk.token_to_id("<|begin_of_text|>")

    @classmethod
    def from_object(cls, tk, bos_id=None):
        self = cls.__new__(cls)
        self.tk = tk
        self.bos_id = bos_id if bos_id is not None else tk.token_to_id("<|begin_of_text|>")
        return self

    def encode(self, text: str, add_bos: bool = True) -> list:
        ids = self.tk.encode(text, add_special_tokens=False).ids
        if add_bos and self.bos_id is not None:
            ids = [self.bos_id] + ids
        return ids

    def encode_batch(self, texts, add_bos: bool = True) -> list:
        encs = self.tk.encode_batch(list(texts), add_special_tokens=False)
        pre = [self.bos_id] if (add_bos and self.bos_id is not None) else []
        return [pre + e.ids for e in encs]

    def decode(self, ids) -> str:
        return self.tk.decode(list(ids), skip_special_tokens=True)

    def decode_batch(self, seqs) -> list:
        return self.tk.decode_batch([list(s) for s in seqs], skip_special_tokens=True)
