"""Resolve an Ollama model tag to the GGUF blob Ollama serves it from.

The reference names its model only by Ollama tag -- ``llama3.2:3b`` (README.md:32,
run_full_evaluation_pipeline.py:961, runners/run_summarization_ollama_mapreduce.py:206) --
and ``ollama pull`` stores it as (EXT, Ollama's published on-disk layout):

    $OLLAMA_MODELS (default ~/.ollama/models)/
      manifests/<host>/<namespace>/<model>/<tag>      OCI-style JSON manifest
      blobs/sha256-<hex>                                content-addressed layers

A tag ``model[:tag]`` means registry.ollama.ai/library/model:tag (tag "latest" when absent);
``ns/model:tag`` and ``host/ns/model:tag`` name the other parts.  The manifest's layer of media
type application/vnd.ollama.image.model is the GGUF; .params is JSON generation defaults
(Ollama's ``stop`` strings for llama3.2); .template the chat template (the engine renders
Llama-3.2's template itself: mapsum/template.py).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

MODEL_MEDIA = "application/vnd.ollama.image.model"
PARAMS_MEDIA = "application/vnd.ollama.image.params"
TEMPLATE_MEDIA = "application/vnd.ollama.image.template"
DEFAULT_HOST, DEFAULT_NS, DEFAULT_TAG = "registry.ollama.ai", "library", "latest"


class OllamaStoreError(FileNotFoundError):
    pass


def models_dir() -> str:
    return os.environ.get("OLLAMA_MODELS") or os.path.join(os.path.expanduser("~"), ".ollama", "models")


def parse_tag(name: str) -> tuple:
    """'llama3.2:3b' -> ('registry.ollama.ai', 'library', 'llama3.2', '3b')."""
    if not name or name.strip() != name:
        raise ValueError(f"bad model tag {name!r}")
    path, tag = name, DEFAULT_TAG
    last = name.rsplit("/", 1)[-1]
    if ":" in last:
        path, tag = name.rsplit(":", 1)
    parts = path.split("/")
    if len(parts) == 1:
        host, ns, model = DEFAULT_HOST, DEFAULT_NS, parts[0]
    elif len(parts) == 2:
        host, (ns, model) = DEFAULT_HOST, parts
    elif len(parts) == 3:
        host, ns, model = parts
    else:
        raise ValueError(f"bad model tag {name!r}")
    if not (model and tag and ns and host):
        raise ValueError(f"bad model tag {name!r}")
    return host, ns, model, tag


def blob_path(root: str, digest: str) -> str:
    algo, _, hexd = digest.partition(":")
    if algo != "sha256" or not hexd or any(c not in "0123456789abcdef" for c in hexd):
        raise OllamaStoreError(f"unexpected layer digest {digest!r}")
    return os.path.join(root, "blobs", f"sha256-{hexd}")


@dataclass
class OllamaModel:
    tag: str
    gguf: str                           # path of the GGUF blob
    params: dict = field(default_factory=dict)
    template: str | None = None


# what a llama3-family chat template must contain for mapsum.template.render_llama32 (the
# engine's own rendering of Ollama's llama3.2 TEMPLATE) to be the prompt Ollama would build
LLAMA3_TEMPLATE_MARKERS = ("<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>")


def template_problems(text: str) -> list:
    """Why a manifest's chat template is not the llama3 family the engine renders (empty: it is).
    The layer is Go template source, so the check is structural: Llama-3's header / end-of-turn
    markers and a prompt or messages action."""
    out = [f"no {m!r}" for m in LLAMA3_TEMPLATE_MARKERS if m not in text]
    if ".Prompt" not in text and ".Messages" not in text:
        out.append("no .Prompt / .Messages action")
    return out


def resolve(name: str, root: str | None = None, allow_foreign_template: bool = False) -> OllamaModel:
    """Manifest -> blobs of one pulled model (OllamaStoreError if it is not there, or if its
    chat template is not the llama3 family mapsum.template renders -- unless
    allow_foreign_template, or MAPSUM_ALLOW_TEMPLATE=1)."""
    root = root or models_dir()
    host, ns, model, tag = parse_tag(name)
    man = os.path.join(root, "manifests", host, ns, model, tag)
    if not os.path.isfile(man):
        raise OllamaStoreError(f"model {name!r} not found: no manifest {man} (ollama pull {name})")
    with open(man, "rb") as f:
        m = json.loads(f.read().decode("utf-8"))
    out = OllamaModel(tag=name, gguf="")
    for layer in m.get("layers", []):
        mt, dg = layer.get("mediaType"), layer.get("digest", "")
        if mt == MODEL_MEDIA:
            out.gguf = blob_path(root, dg)
        elif mt == PARAMS_MEDIA:
            with open(blob_path(root, dg), "rb") as f:
                out.params = json.loads(f.read().decode("utf-8"))
        elif mt == TEMPLATE_MEDIA:
            with open(blob_path(root, dg), "rb") as f:
                out.template = f.read().decode("utf-8")
    if not out.gguf:
        raise OllamaStoreError(f"manifest {man} has no {MODEL_MEDIA} layer")
    if out.template is not None:
        why = template_problems(out.template)
        if why and not (allow_foreign_template or os.environ.get("MAPSUM_ALLOW_TEMPLATE") == "1"):
            raise OllamaStoreError(f"model {name!r}: its chat template is not Llama-3's ({'; '.join(why)}); "
                                   "the engine renders Llama-3.2's template (mapsum/template.py) -- refusing "
                                   "(MAPSUM_ALLOW_TEMPLATE=1 overrides)")
    if not os.path.isfile(out.gguf):
        raise OllamaStoreError(f"model blob {out.gguf} missing (ollama pull {name})")
    return out


def config_from_gguf(meta: dict, base=None):
    """ModelConfig of a llama GGUF: shapes from llama.* metadata, vocabulary size from the token
    list, BOS / stop ids from tokenizer.ggml.*; the llama3 RoPE scaling constants (not in the
    metadata: Ollama ships them as the rope_freqs tensor) are Llama-3.2's (config.LLAMA32_3B)."""
    from .config import LLAMA32_3B
    from .tokenizer import gguf_stop_ids
    base = base or LLAMA32_3B
    g = lambda k, d: meta.get(f"llama.{k}", d)  # noqa: E731
    hidden = int(g("embedding_length", base.hidden))
    heads = int(g("attention.head_count", base.n_heads))
    head_dim = int(g("attention.key_length", hidden // heads))
    tokens = meta.get("tokenizer.ggml.tokens")
    kw = dict(name=str(meta.get("general.name", base.name)), n_layers=int(g("block_count", base.n_layers)),
              hidden=hidden, n_heads=heads, n_kv_heads=int(g("attention.head_count_kv", base.n_kv_heads)),
              head_dim=head_dim, ffn=int(g("feed_forward_length", base.ffn)),
              vocab=int(g("vocab_size", len(tokens) if tokens else base.vocab)),
              rope_theta=float(g("rope.freq_base", base.rope_theta)),
              norm_eps=float(g("attention.layer_norm_rms_epsilon", base.norm_eps)))
    if "tokenizer.ggml.bos_token_id" in meta:
        kw["bos_id"] = int(meta["tokenizer.ggml.bos_token_id"])
    stops = gguf_stop_ids(meta)
    if stops:
        kw["eos_ids"] = stops
    return base.with_(**kw)
