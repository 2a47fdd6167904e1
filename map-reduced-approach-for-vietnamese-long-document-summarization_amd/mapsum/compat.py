"""Drop-in for the reference's ``OllamaLLM`` (the map-phase boundary).

Reference class (run_full_evaluation_pipeline.py:66-117; runner copies
runners/run_summarization_ollama_mapreduce.py:23-60, ..._critique.py:51-91,
..._hierarchical.py:43-80, ..._iterative.py:50-92):

    OllamaLLM(ollama_url, model_name, max_new_tokens=2048)
    _call(prompt, stop=None, run_manager=None, **kw) -> str   # POST /api/generate, clean
    async _acall(...)                                         # blocking: calls _call
    _llm_type -> "ollama";  get_num_tokens(text) -> len(text.split())

This class keeps that surface -- same constructor, same return strings (template ->
greedy generate -> detokenize -> the caller's clean_thinking_tokens variant), same
``get_num_tokens`` (the collapse logic at mapreduce.py:98-100,147-154 depends on it) --
but runs the chunk on libmapsum instead of an Ollama server.  ``_acall`` is genuinely
asynchronous: concurrent calls (the LangGraph ``Send`` fan-out, mapreduce.py:109-112)
join one continuous batch on the GPU instead of running one after another.
Errors surface as RuntimeError, as ``resp.raise_for_status()`` did (pipeline.py:91).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import os
import threading

from .postprocess import CLEANERS
from .template import render_llama32

try:  # be a real LangChain LLM when LangChain is installed (it is not in this container)
    from langchain_core.language_models.llms import LLM as _Base  # type: ignore
    _HAVE_LC = True
except Exception:  # pragma: no cover - exercised when langchain is absent
    _Base = object
    _HAVE_LC = False


class MapBackend:
    """One engine + tokenizer, shared by every OllamaLLM that names the same model.

    All engine calls run on one worker thread (the engine is not thread-safe); async
    callers are batched: every request queued before a scheduler tick joins it."""

    def __init__(self, engine, tokenizer, template=render_llama32, retries: int = 0):
        self.engine = engine
        self.retries = retries    # re-queues of a MS_FINISH_ERROR chunk (see Engine.generate)
        self.tok = tokenizer
        self.template = template
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="mapsum")
        self._lock = threading.Lock()
        self._queue = []          # (ids, num_predict, future) waiting for the driver
        self._inflight = {}       # tag -> future
        self._driver = None
        self._tag = _ASYNC_TAG0

    # -- text <-> ids ----------------------------------------------------------
    def encode_prompt(self, prompt: str) -> list:
        return self.tok.encode(self.template(prompt, add_bos=False), add_bos=True)

    # -- synchronous path (one chunk, or a list of chunks) ----------------------
    def generate_ids(self, id_lists, num_predict: int) -> list:
        res = self._pool.submit(self.engine.generate, id_lists, num_predict, False, self.retries).result()
        for r in res:
            if r.finish == "error":  # deterministic: a re-run would fail the same way
                raise RuntimeError("mapsum: chunk failed (no finite logit)")
        return res

    def generate(self, prompts, num_predict: int) -> list:
        ids = [self.encode_prompt(p) for p in prompts]
        res = self.generate_ids(ids, num_predict)
        return [self.tok.decode(r.ids) for r in res]

    # -- asynchronous path: continuous batching across concurrent callers ---------
    async def agenerate(self, prompt: str, num_predict: int) -> str:
        return (await self.agenerate_full(prompt, num_predict))[0]

    async def agenerate_full(self, prompt: str, num_predict: int):
        """(text, finish) with finish in {"eos", "length"} -- Ollama's done_reason
        "stop" / "length"."""
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        ids = self.encode_prompt(prompt)
        with self._lock:
            self._tag += 1
            tag = self._tag
        self._queue.append((tag, ids, num_predict))
        self._inflight[tag] = (fut, ids, num_predict, self.retries)
        if self._driver is None or self._driver.done():
            self._driver = asyncio.ensure_future(self._drive())
        r = await fut
        return self.tok.decode(r.ids), r.finish

    def _tick(self, new):
        """Engine thread: submit the new requests (a request the engine refuses fails
        alone), run one scheduler iteration, return this backend's finished results."""
        refused = []
        for tag, ids, n in new:
            try:
                self.engine.submit(ids, n, tag=tag)
            except Exception as e:  # noqa: BLE001 -- e.g. ENOSPC: prompt + num_predict > max_ctx
                refused.append((tag, e))
        self.engine.step()
        self.engine.collect()
        return refused, self.engine.take_where(lambda t: t > _ASYNC_TAG0)

    async def _drive(self):
        loop = asyncio.get_running_loop()
        try:
            while self._queue or self._inflight:
                new, self._queue = self._queue, []
                refused, done = await loop.run_in_executor(self._pool, self._tick, new)
                for tag, e in refused:
                    fut = self._inflight.pop(tag, (None,))[0]
                    if fut is not None and not fut.done():
                        fut.set_exception(RuntimeError(f"mapsum: request refused: {e}"))
                for r in done:
                    ent = self._inflight.pop(r.tag, None)
                    if ent is None:
                        continue
                    fut, ids, n, retries = ent
                    if fut.done():
                        continue
                    if r.finish != "error":
                        fut.set_result(r)
                    elif retries > 0:  # opt-in re-queue (transient device faults only)
                        with self._lock:
                            self._tag += 1
                            tag = self._tag
                        self._queue.append((tag, ids, n))
                        self._inflight[tag] = (fut, ids, n, retries - 1)
                    else:
                        fut.set_exception(RuntimeError("mapsum: chunk failed (no finite logit)"))
        except Exception as e:  # the engine itself failed: every waiter fails loudly
            for ent in self._inflight.values():
                if not ent[0].done():
                    ent[0].set_exception(RuntimeError(f"mapsum engine failed: {e}"))
            self._inflight.clear()
            raise


_ASYNC_TAG0 = 1 << 40  # async tags live above the engine's own generate() tags
_BACKENDS: dict = {}
_FACTORY = None


def register_backend(model_name: str, backend: MapBackend):
    """Bind an Ollama model tag (e.g. 'llama3.2:3b') to an engine backend."""
    _BACKENDS[model_name] = backend


def set_backend_factory(fn):
    """fn(model_name) -> MapBackend, called on first use of an unknown model tag."""
    global _FACTORY
    _FACTORY = fn


def _engine_kwargs() -> dict:
    # the decode regime is fixed per engine, so any max_batch keeps a batched
    # call equal to the same call alone; 64 in flight runs the large-batch regime
    return dict(device=int(os.environ.get("LOCAL_RANK", 0)),
                max_batch=int(os.environ.get("MAPSUM_MAX_BATCH", 64)),
                max_ctx=int(os.environ.get("MAPSUM_MAX_CTX", 16384)),
                max_prefill_tokens=int(os.environ.get("MAPSUM_MAX_PREFILL", 32768)))


def gguf_backend(path: str, engine_cls=None, params: dict | None = None) -> MapBackend:
    """A backend on a GGUF file: the model config and the tokenizer both come from the file's
    own metadata (an Ollama blob has no tokenizer.json), the weights through gguf.load_gguf
    (F16 / BF16 / F32 as fp16; Q4_K / Q6_K as the dequant-fused K-quant path).  ``params`` is
    the Ollama manifest's params layer: its single-token ``stop`` strings join the stop set."""
    from .gguf import load_gguf, read_gguf
    from .ollama_store import config_from_gguf
    from .tokenizer import tokenizer_from_gguf
    if engine_cls is None:
        from .engine import Engine as engine_cls
    meta, ts = read_gguf(path)
    cfg = config_from_gguf(meta).with_(tie_embeddings="output.weight" not in ts)
    tok = tokenizer_from_gguf(meta)
    stops = list(cfg.eos_ids)
    for s in (params or {}).get("stop", []):
        ids = tok.encode(s, add_bos=False)
        if len(ids) == 1 and ids[0] not in stops:
            stops.append(ids[0])
    del ts
    eng = engine_cls(cfg, eos_ids=tuple(stops[:8]), **_engine_kwargs())
    load_gguf(eng, path)
    return MapBackend(eng, tok)


def _default_factory(model_name: str) -> MapBackend:
    """Real-weight path, in order: MAPSUM_MODEL_DIR (HF Llama-3.2 safetensors + tokenizer.json),
    MAPSUM_GGUF (a GGUF file), else the Ollama store ($OLLAMA_MODELS or ~/.ollama/models): the
    tag the reference passes (``llama3.2:3b``, run_full_evaluation_pipeline.py:961) -> manifest
    -> GGUF blob, exactly the file `ollama serve` would run."""
    d = os.environ.get("MAPSUM_MODEL_DIR")
    if d:
        from .config import LLAMA32_3B
        from .engine import Engine
        from .tokenizer import Tokenizer
        from .weights import load_hf_dir
        eng = Engine(LLAMA32_3B, **_engine_kwargs())
        load_hf_dir(eng, d)
        return MapBackend(eng, Tokenizer(os.path.join(d, "tokenizer.json")))
    g = os.environ.get("MAPSUM_GGUF")
    if g:
        return gguf_backend(g)
    from . import ollama_store
    try:
        m = ollama_store.resolve(model_name)
    except (FileNotFoundError, ValueError) as e:
        raise RuntimeError(f"no backend for model {model_name!r}: MAPSUM_MODEL_DIR / MAPSUM_GGUF unset and "
                           f"the Ollama store has no such model ({e})") from e
    return gguf_backend(m.gguf, params=m.params)


def get_backend(model_name: str) -> MapBackend:
    if model_name not in _BACKENDS:
        _BACKENDS[model_name] = (_FACTORY or _default_factory)(model_name)
    return _BACKENDS[model_name]


class OllamaLLM(_Base):
    """Same constructor and methods as the reference's OllamaLLM; runs on libmapsum."""

    ollama_url: str = "http://localhost:11434"
    model_name: str = "llama3.2:3b"
    max_new_tokens: int = 2048
    clean: str = "pipeline"  # 'pipeline' | 'hierarchical' | 'none' (which runner's cleaner)

    def __init__(self, ollama_url: str = "http://localhost:11434", model_name: str = "llama3.2:3b",
                 max_new_tokens: int = 2048, clean: str = "pipeline", **kwargs):
        if _HAVE_LC:
            super().__init__(ollama_url=ollama_url, model_name=model_name,
                             max_new_tokens=max_new_tokens, clean=clean, **kwargs)
        else:
            self.ollama_url = ollama_url  # kept for signature parity; no HTTP is made
            self.model_name = model_name
            self.max_new_tokens = max_new_tokens
            self.clean = clean
        if clean not in CLEANERS:
            raise ValueError(f"clean must be one of {sorted(CLEANERS)}")

    # ---- the reference surface --------------------------------------------------
    def _call(self, prompt: str, stop=None, run_manager=None, **kwargs) -> str:
        b = get_backend(self.model_name)
        raw = b.generate([prompt], self.max_new_tokens)[0]
        return CLEANERS[self.clean](raw)

    async def _acall(self, prompt: str, stop=None, run_manager=None, **kwargs) -> str:
        b = get_backend(self.model_name)
        raw = await b.agenerate(prompt, self.max_new_tokens)
        return CLEANERS[self.clean](raw)

    @property
    def _llm_type(self) -> str:
        return "ollama"

    def get_num_tokens(self, text: str) -> int:
        # the reference's whitespace approximation (pipeline.py:115-117) -- kept verbatim
        # because map-reduce's collapse decisions (mapreduce.py:147-154) depend on it
        return len(text.split())

    # ---- minimal Runnable surface when LangChain is absent -------------------------
    if not _HAVE_LC:
        def invoke(self, input, config=None, **kwargs) -> str:
            return self._call(_as_text(input), **kwargs)

        async def ainvoke(self, input, config=None, **kwargs) -> str:
            return await self._acall(_as_text(input), **kwargs)

        def __call__(self, prompt: str, **kwargs) -> str:
            return self._call(prompt, **kwargs)

        def batch(self, inputs, config=None, **kwargs) -> list:
            """All prompts in one continuous batch (what the Send fan-out should have been)."""
            b = get_backend(self.model_name)
            raw = b.generate([_as_text(i) for i in inputs], self.max_new_tokens)
            return [CLEANERS[self.clean](r) for r in raw]


def _as_text(x) -> str:
    if isinstance(x, str):
        return x
    to_string = getattr(x, "to_string", None)  # LangChain PromptValue
    if callable(to_string):
        return to_string()
    return str(x)
