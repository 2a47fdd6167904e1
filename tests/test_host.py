"""CPU tests of the host side of the boundary (no GPU): prompts, post-processing, the
OllamaLLM mirror, chunk sharding, the C-ABI export table."""
import asyncio
import hashlib
import json
import os
import re

import numpy as np
import pytest

from mapsum import compat, template
from mapsum.dist import Unit, pack_results, shard_lpt, shard_static, unpack_results
from mapsum.postprocess import clean_thinking_tokens, clean_thinking_tokens_hierarchical

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


# ------------------------------------------------------------------ known answers
def test_clean_thinking_kat_from_pipeline_selfcheck():
    """run_full_evaluation_pipeline.py:193-197 feeds this string and expects it shorter."""
    s = ("This is a summary. <think>This is thinking content that should be removed.</think> "
         "This is the rest of the summary.")
    out = clean_thinking_tokens(s)
    assert len(out) < len(s)
    assert out == "This is a summary.  This is the rest of the summary."
    assert clean_thinking_tokens_hierarchical(s) == "This is a summary. This is the rest of the summary."


@pytest.mark.parametrize("tag", ["think", "THINKING", "Thought", "reasoning", "analysis"])
def test_clean_thinking_tags_case_and_multiline(tag):
    s = f"Tóm tắt.\n<{tag}>\nbước 1\nbước 2\n</{tag}>\n\n\n\nKết luận."
    assert clean_thinking_tokens(s) == "Tóm tắt.\n\nKết luận."
    assert clean_thinking_tokens_hierarchical(s) == "Tóm tắt. Kết luận."


def test_clean_thinking_edge_cases():
    assert clean_thinking_tokens("") == ""
    assert clean_thinking_tokens(None) is None
    assert clean_thinking_tokens("  a\n \n \n b  ") == "a\n\n b"  # \n\s*\n\s*\n -> \n\n, inner space kept
    assert clean_thinking_tokens("<think>x</think>") == ""
    # unterminated tags are left alone (non-greedy pattern needs the closing tag)
    assert clean_thinking_tokens("<think>open") == "<think>open"


def test_map_prompts_match_reference_bytes():
    fx = json.load(open(os.path.join(HERE, "golden", "prompts.json"), encoding="utf-8"))
    for key, want in fx.items():
        if key not in template.MAP_PROMPTS:
            continue  # reduce/review prompts: tests/test_mapreduce.py, tests/test_hierarchical.py
        s = template.MAP_PROMPTS[key]
        assert len(s) == want["n_chars"], key
        assert hashlib.sha256(s.encode()).hexdigest() == want["sha256"], key


def test_map_prompt_rendering():
    chunk = "Chương 1. Nội dung chính của văn bản."
    p = template.map_prompt("mapreduce", chunk)
    assert chunk in p and "{content}" not in p and p.startswith("Bạn là một chuyên gia")
    h = template.map_prompt("mapreduce_hierarchical", chunk)
    assert h.startswith("System: Bạn là một chuyên gia")
    full = template.render_llama32(p)
    assert full.startswith("<|begin_of_text|><|start_header_id|>system<|end_header_id|>\n\n")
    assert full.endswith(p + "<|eot_id|><|start_header_id|>assistant<|end_header_id|>\n\n")


# ------------------------------------------------------------------ OllamaLLM mirror
from mapsum.engine import RequestQueue, Result  # noqa: E402


class FakeEngine(RequestQueue):
    """Test double with libmapsum's request primitives (submit/step/poll); generate(),
    the mailbox and the one-retry logic are the real RequestQueue's.  Each chunk's
    'summary' is its last prompt ids reversed (deterministic), so the adapter's plumbing
    is checkable on CPU.  ``fail_first``: prompts (as tuples) whose first run finishes
    with "error" (a chunk with a non-finite logit); ``refuse``: prompt lengths submit()
    rejects (as ms_submit's ENOSPC does)."""

    def __init__(self, fail_first=(), refuse_len=None):
        self.q, self.done, self.steps, self.batches = {}, [], 0, []
        self._tag = 1
        self._mailbox = {}
        self.fail_first = set(fail_first)
        self.refuse_len = refuse_len

    def submit(self, ids, n, ignore_eos=False, tag=None):
        if self.refuse_len is not None and len(ids) > self.refuse_len:
            raise RuntimeError("libmapsum ms_submit failed (-28): prompt exceeds max_ctx")
        if tag is None:
            tag, self._tag = self._tag, self._tag + 1
        self.q[tag] = (list(ids), n)
        return tag

    def step(self):
        self.steps += 1
        self.batches.append(len(self.q))
        for tag, (ids, n) in self.q.items():
            if tuple(ids) in self.fail_first:
                self.fail_first.discard(tuple(ids))
                self.done.append(Result(tag, [], "error", len(ids)))
            else:
                self.done.append(Result(tag, ids[::-1][:n], "length", len(ids)))
        self.q = {}
        return 0

    def poll(self, cap=256):
        out, self.done = self.done[:cap], self.done[cap:]
        return out


@pytest.fixture(scope="module")
def toy_tokenizer():
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    specials = ["<|begin_of_text|>", "<|eot_id|>", "<|start_header_id|>", "<|end_header_id|>"]
    tr = trainers.BpeTrainer(vocab_size=400, special_tokens=specials,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator([template.MAP_PROMPT_MAPREDUCE, "Tóm tắt nội dung văn bản tiếng Việt."] * 4, tr)
    from mapsum.tokenizer import Tokenizer as MT
    return MT.from_object(tk)


@pytest.fixture
def llm(toy_tokenizer):
    eng = FakeEngine()
    compat.register_backend("fake:test", compat.MapBackend(eng, toy_tokenizer))
    yield compat.OllamaLLM("http://localhost:11434", "fake:test", max_new_tokens=1000), eng
    compat._BACKENDS.pop("fake:test", None)


def test_ollamallm_surface(llm):
    m, _ = llm
    assert m._llm_type == "ollama"
    assert m.get_num_tokens("  một hai\nba  ") == 3
    assert (m.ollama_url, m.model_name, m.max_new_tokens) == ("http://localhost:11434", "fake:test", 1000)


def test_ollamallm_call_roundtrip(llm, toy_tokenizer):
    m, eng = llm
    prompt = "Tóm tắt"
    out = m._call(prompt)
    ids = toy_tokenizer.encode(template.render_llama32(prompt, add_bos=False))
    assert out == clean_thinking_tokens(toy_tokenizer.decode(ids[::-1]))
    assert m.invoke(prompt) == out


def test_ollamallm_async_fanout_is_one_batch(llm):
    """The Send fan-out (mapreduce.py:109-112) issues every chunk's ainvoke concurrently;
    here they must all reach the engine in the same scheduler tick."""
    m, eng = llm
    chunks = [f"đoạn {i}" for i in range(7)]

    async def fan_out():
        return await asyncio.gather(*[m.ainvoke(template.map_prompt("mapreduce", c)) for c in chunks])
    outs = asyncio.run(fan_out())
    assert len(outs) == 7 and eng.batches[0] == 7 and eng.steps == 1
    sync = [m._call(template.map_prompt("mapreduce", c)) for c in chunks]
    assert outs == sync


def test_ollamallm_engine_error_is_raised(toy_tokenizer):
    class Broken(FakeEngine):
        def step(self):
            raise RuntimeError("libmapsum ms_step failed (-5): device lost")
    compat.register_backend("fake:broken", compat.MapBackend(Broken(), toy_tokenizer))
    m = compat.OllamaLLM("u", "fake:broken")
    with pytest.raises(RuntimeError):
        asyncio.run(m.ainvoke("x"))
    compat._BACKENDS.pop("fake:broken")


def test_generate_failed_chunk_fails_alone_and_retry_is_opt_in():
    """a chunk finishing with MS_FINISH_ERROR fails alone and, by default, at
    once (deterministic greedy decoding would recompute the same non-finite logits); with
    retries=1 it is re-queued once and the others are not re-run."""
    eng = FakeEngine(fail_first=[(7,)])
    res = eng.generate([[7], [8]], 4)
    assert res[0].finish == "error" and res[1].ids == [8] and eng.batches == [2]
    eng = FakeEngine(fail_first=[(1, 2, 3)])
    res = eng.generate([[1, 2, 3], [4, 5]], num_predict=8, retries=1)
    assert [r.ids for r in res] == [[3, 2, 1], [5, 4]] and eng.batches == [2, 1]


def test_generate_leaves_foreign_results_in_the_mailbox():
    """The synchronous path must not consume (or count) results of requests another
    caller (the async driver) submitted to the same engine."""
    eng = FakeEngine()
    foreign = eng.submit([9, 9, 9], 2, tag=(1 << 40) + 5)
    res = eng.generate([[1, 2]], 4)
    assert res[0].ids == [2, 1]
    assert [r.tag for r in eng.take_where(lambda t: t == foreign)] == [foreign]


def test_async_refused_request_fails_alone(toy_tokenizer):
    """One over-long prompt (ms_submit ENOSPC) fails its own future only; the concurrent
    requests of the same tick still complete."""
    eng = FakeEngine(refuse_len=400)
    compat.register_backend("fake:refuse", compat.MapBackend(eng, toy_tokenizer))
    m = compat.OllamaLLM("u", "fake:refuse", max_new_tokens=50)

    async def fan_out():
        return await asyncio.gather(m.ainvoke("ngắn"), m.ainvoke("dài " * 600), m.ainvoke("vừa"),
                                    return_exceptions=True)
    try:
        a, b, c = asyncio.run(fan_out())
    finally:
        compat._BACKENDS.pop("fake:refuse", None)
    assert isinstance(b, RuntimeError) and "refused" in str(b)
    assert isinstance(a, str) and isinstance(c, str)


def test_async_failed_chunk_fails_alone_and_retry_is_opt_in(toy_tokenizer):
    prompt = "Tóm tắt lỗi"
    for retries in (0, 1):
        be = compat.MapBackend(FakeEngine(), toy_tokenizer, retries=retries)
        ids = tuple(be.encode_prompt(prompt))
        be.engine.fail_first = {ids}
        compat.register_backend("fake:retry", be)
        m = compat.OllamaLLM("u", "fake:retry", max_new_tokens=1000)
        try:
            if retries == 0:  # default: the deterministic failure is reported once, at once
                with pytest.raises(RuntimeError, match="no finite logit"):
                    asyncio.run(m.ainvoke(prompt))
                assert be.engine.steps == 1
                continue
            out = asyncio.run(m.ainvoke(prompt))
        finally:
            compat._BACKENDS.pop("fake:retry", None)
        assert out == clean_thinking_tokens(toy_tokenizer.decode(list(ids)[::-1]))
        assert be.engine.steps == 2


# ------------------------------------------------------------------ chunk sharding
def test_shard_static_partitions():
    units = [Unit(d, c, 2048) for d in range(3) for c in range(8)]
    parts = [shard_static(units, r, 4) for r in range(4)]
    assert sorted(u for p in parts for u in p) == sorted(units)
    assert [len(p) for p in parts] == [6, 6, 6, 6]


def test_shard_lpt_balances_ragged():
    rng = np.random.default_rng(1)
    lens = np.clip(np.exp(rng.normal(np.log(600), 1.0, size=200)), 64, 4096).astype(int)
    units = [Unit(i // 10, i % 10, int(n)) for i, n in enumerate(lens)]
    parts = [shard_lpt(units, r, 8) for r in range(8)]
    assert sorted(u for p in parts for u in p) == sorted(units)
    loads = [sum(u.n_tokens for u in p) for p in parts]
    assert max(loads) - min(loads) <= max(lens)


def test_pack_unpack_roundtrip():
    units = [Unit(0, 0, 10), Unit(3, 5, 10)]
    rows = pack_results(units, [[1, 2, 3], []], 8)
    assert unpack_results(rows) == {(0, 0): [1, 2, 3], (3, 5): []}


def _gather_worker(rank, world, port, q):
    import torch.distributed as dist
    from mapsum.dist import gather_summaries
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    units = [Unit(rank, c, 100) for c in range(rank + 1)]
    packed = pack_results(units, [[rank * 10 + c] * (c + 1) for c in range(rank + 1)], 4)
    rows = gather_summaries(packed, max_rows=3)
    if rank == 0:
        q.put(unpack_results(rows))
    dist.destroy_process_group()


def test_gather_summaries_gloo_world2():
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = q.get(timeout=120)
    for p in ps:
        p.join(60)
    assert res == {(0, 0): [0], (1, 0): [10], (1, 1): [11, 11]}


# ------------------------------------------------------------------ C-ABI
def test_cabi_exports_every_header_symbol():
    from mapsum import _lib
    hdr = open(os.path.join(ROOT, "include", "mapsum.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(ms_\w+)\(", hdr, re.M))
    assert len(declared) >= 19
    assert declared == set(_lib.EXPORTED)
    lib = _lib.load()
    for sym in declared:
        assert hasattr(lib, sym), sym


def test_cabi_errors_without_gpu():
    """Bad arguments are rejected before any device work, with a readable error."""
    import ctypes as C
    from mapsum import _lib
    lib = _lib.load()
    cfg = _lib.MsConfig()
    cfg.abi_version = 999
    h = C.c_void_p()
    assert lib.ms_create(C.byref(cfg), C.byref(h)) == _lib.MS_EINVAL
    assert b"abi_version" in lib.ms_last_error(None)
    assert lib.ms_step(None) == _lib.MS_EINVAL
    assert lib.ms_op_gemv_workspace(0, 16, 64) == _lib.MS_EINVAL


class _HostWeights:
    """CPU stand-in for an engine's weight regions and K-quant manifest."""

    def __init__(self, rank):
        import torch
        self.regions = [torch.full((n,), rank + 1, dtype=torch.uint8) for n in (7, 1024, 3)]
        self.manifest = [(2, 0, 12), (9, 1, 14)] if rank == 0 else []
        self.declared = []

    def quant_manifest(self):
        return list(self.manifest)

    def declare_weight_q(self, t, l, ty):
        self.declared.append((t, l, ty))
        self.regions.append(__import__("torch").zeros(16, dtype=__import__("torch").uint8))

    def region_views(self):
        return self.regions


def _bcast_worker(rank, world, port, q):
    import torch.distributed as dist
    from mapsum.dist import broadcast_engine_weights
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    e = _HostWeights(rank)
    if rank == 0:  # rank 0's quantised regions exist already
        e.regions += [__import__("torch").full((16,), 9, dtype=__import__("torch").uint8) for _ in range(2)]
    n = broadcast_engine_weights(e, src=0)
    q.put((rank, n, e.declared, [r.tolist() for r in e.regions]))
    dist.destroy_process_group()


def test_weight_broadcast_gloo_world2():
    """Rank 0's weights (and its K-quant layout) reach the other rank byte for byte."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict((r, (n, d, regs)) for r, n, d, regs in (q.get(timeout=120) for _ in range(2)))
    for p in ps:
        p.join(60)
    assert got[1][1] == [(2, 0, 12), (9, 1, 14)]  # the receiver declared rank 0's layout
    assert got[0][2] == got[1][2] and got[0][0] == got[1][0] == 7 + 1024 + 3 + 32
