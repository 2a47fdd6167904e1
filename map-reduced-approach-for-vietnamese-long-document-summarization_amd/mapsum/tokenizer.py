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


_NO_BOS = object()  # from_object(bos_id=_NO_BOS): the vocabulary prepends no BOS at all


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
        if bos_id is _NO_BOS:
            self.bos_id = None
        else:
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


# ------------------------------------------------------------------ from GGUF metadata
# An Ollama install keeps no tokenizer.json: the vocabulary lives in the GGUF blob's metadata
# (EXT, llama.cpp's converter: tokenizer.ggml.model "gpt2" = byte-level BPE, .pre the
# pre-tokenizer family, .tokens / .token_type / .merges, .bos/.eos/.eot_token_id), which is
# what Ollama tokenises with for llama3.2:3b (README.md:32).  The pre-tokenizer regexes are the
# published ones of each family: "llama-bpe" is Llama-3's tiktoken pattern, as in Meta's
# tokenizer.json (Split isolated, then ByteLevel without its own regex; BPE with
# ignore_merges -- a pre-token that is itself a vocabulary entry is not merged further).
PRE_TOKENIZERS = {
    "llama-bpe": (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                  r"|\s*[\r\n]+|\s+(?!\S)|\s+", True),
    "default": (r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+", False),
}
TOKEN_CONTROL, TOKEN_USER_DEFINED = 3, 4  # llama.cpp token types matched as special tokens


def tokenizer_from_gguf(meta: dict) -> "Tokenizer":
    """A Tokenizer from a GGUF's tokenizer.ggml.* metadata (byte-level BPE families only)."""
    from tokenizers import AddedToken, Regex, decoders, models, pre_tokenizers
    from tokenizers import Tokenizer as _T
    model = meta.get("tokenizer.ggml.model")
    if model != "gpt2":
        raise ValueError(f"GGUF tokenizer model {model!r} is not byte-level BPE ('gpt2')")
    pre = meta.get("tokenizer.ggml.pre", "default")
    if pre not in PRE_TOKENIZERS:
        raise ValueError(f"GGUF pre-tokenizer {pre!r} is not supported ({sorted(PRE_TOKENIZERS)})")
    pattern, ignore_merges = PRE_TOKENIZERS[pre]
    tokens = list(meta["tokenizer.ggml.tokens"])
    types = list(meta.get("tokenizer.ggml.token_type", [1] * len(tokens)))
    merges = [tuple(m.split(" ", 1)) for m in meta.get("tokenizer.ggml.merges", [])]
    vocab = {}
    for i, t in enumerate(tokens):
        vocab.setdefault(t, i)
    tk = _T(models.BPE(vocab=vocab, merges=merges, ignore_merges=ignore_merges, fuse_unk=False,
                       byte_fallback=False))
    tk.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(pattern), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, trim_offsets=False, use_regex=False)])
    tk.decoder = decoders.ByteLevel()
    tk.add_special_tokens([AddedToken(tokens[i], special=True, normalized=False)
                           for i, ty in enumerate(types) if ty in (TOKEN_CONTROL, TOKEN_USER_DEFINED)])
    if not meta.get("tokenizer.ggml.add_bos_token", True):
        return Tokenizer.from_object(tk, bos_id=_NO_BOS)  # (None would look <|begin_of_text|> up)
    bos = meta.get("tokenizer.ggml.bos_token_id")
    return Tokenizer.from_object(tk, bos_id=int(bos) if bos is not None else None)


def gguf_stop_ids(meta: dict) -> tuple:
    """End-of-generation ids of a GGUF vocabulary: eos, eot and eom where present (llama.cpp's
    end-of-generation set; Llama-3.2: <|eot_id|> 128009, <|end_of_text|> 128001, <|eom_id|>)."""
    out = []
    for k in ("tokenizer.ggml.eos_token_id", "tokenizer.ggml.eot_token_id", "tokenizer.ggml.eom_token_id"):
        v = meta.get(k)
        if v is not None and int(v) not in out:
            out.append(int(v))
    tokens = meta.get("tokenizer.ggml.tokens", [])
    for name in ("<|eot_id|>", "<|eom_id|>", "<|end_of_text|>"):
        if name in tokens:
            i = tokens.index(name)
            if i not in out:
                out.append(i)
    return tuple(out[:8])
