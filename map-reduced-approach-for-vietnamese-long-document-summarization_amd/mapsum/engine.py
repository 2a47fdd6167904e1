"""Python handle on one libmapsum engine (one GPU, one process).

The reference makes one blocking HTTP generate per chunk
(run_full_evaluation_pipeline.py:80-106).  Here the same unit of work -- prompt ids
in, greedy summary ids out, stop at an end-of-turn id or ``num_predict`` -- is a
``submit``; ``step`` advances every submitted chunk together (continuous batching
inside libmapsum), ``poll`` returns finished ones.  ``generate`` is the batch
convenience the bench and the adapter use.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .config import ModelConfig


@dataclass
class Result:
    tag: int
    ids: list
    finish: str  # "eos" | "length" | "error"
    n_prompt: int


_FINISH = {L.MS_FINISH_EOS: "eos", L.MS_FINISH_LENGTH: "length", L.MS_FINISH_ERROR: "error"}


class RequestQueue:
    """The request-level half of an engine, over four primitives the subclass provides:
    ``submit(ids, n, ignore_eos, tag) -> tag``, ``step() -> pending``, ``poll() -> [Result]``.

    Finished results are parked in a mailbox keyed by tag, so several submitters (the
    synchronous generate() and MapBackend's async driver) can share one engine: each
    takes only its own tags and never consumes -- or counts -- another caller's."""

    _mailbox: dict

    def collect(self) -> None:
        """Move every finished result into the mailbox."""
        while True:
            got = self.poll()
            for r in got:
                self._mailbox[r.tag] = r
            if len(got) < 256:
                return

    def take(self, tags) -> dict:
        """Remove and return the mailbox entries of ``tags`` that have finished."""
        return {t: self._mailbox.pop(t) for t in list(tags) if t in self._mailbox}

    def take_where(self, pred) -> list:
        """Remove and return the mailbox entries whose tag satisfies ``pred``."""
        mine = [t for t in self._mailbox if pred(t)]
        return [self._mailbox.pop(t) for t in mine]

    def generate(self, prompts, num_predict: int, ignore_eos: bool = False, retries: int = 0) -> list:
        """Run every prompt (list of id lists) to completion; results in input order.

        A chunk that finishes with MS_FINISH_ERROR (no finite logit: SURVEY.md §5 failure
        row) fails alone; the rest of the batch is unaffected.  Greedy decoding is
        deterministic and batch-invariant, so re-running such a chunk recomputes the same
        non-finite logits: by default it is reported at once.  ``retries`` > 0 re-queues it
        that many times, a guard against transient device faults only.  The reference has
        no retry at all (run_full_evaluation_pipeline.py:627-638)."""
        tags = [self.submit(p, num_predict, ignore_eos) for p in prompts]
        order = {t: i for i, t in enumerate(tags)}
        left = {t: retries for t in tags}
        out = [None] * len(tags)
        waiting = set(tags)
        while waiting:
            pending = self.step()
            self.collect()
            for t, r in self.take(waiting).items():
                waiting.discard(t)
                i = order.pop(t)
                if r.finish == "error" and left[t] > 0:
                    nt = self.submit(prompts[i], num_predict, ignore_eos)
                    order[nt], left[nt] = i, left[t] - 1
                    waiting.add(nt)
                    pending += 1
                else:
                    out[i] = r
            if pending == 0 and waiting:
                self.collect()
                if not any(t in self._mailbox for t in waiting):
                    raise RuntimeError("engine drained without finishing every request")
        return out


class Engine(RequestQueue):
    def __init__(self, cfg: ModelConfig, device: int = 0, max_batch: int = 8, max_ctx: int = 4096,
                 max_prefill_tokens: int = 16384, n_pages: int = 0, eos_ids=None):
        self.cfg = cfg
        self.lib = L.load()
        c = L.MsConfig()
        c.abi_version = L.MS_ABI_VERSION
        c.n_layers, c.hidden, c.n_heads = cfg.n_layers, cfg.hidden, cfg.n_heads
        c.n_kv_heads, c.head_dim, c.ffn, c.vocab = cfg.n_kv_heads, cfg.head_dim, cfg.ffn, cfg.vocab
        c.rope_theta, c.rope_factor = cfg.rope_theta, cfg.rope_factor
        c.rope_low_freq_factor, c.rope_high_freq_factor = cfg.rope_low_freq_factor, cfg.rope_high_freq_factor
        c.rope_orig_ctx, c.norm_eps = cfg.rope_orig_ctx, cfg.norm_eps
        c.tie_embeddings = int(cfg.tie_embeddings)
        c.device, c.max_batch, c.max_ctx = device, max_batch, max_ctx
        c.max_prefill_tokens, c.n_pages = max_prefill_tokens, n_pages
        eos = tuple(cfg.eos_ids if eos_ids is None else eos_ids)
        if len(eos) > 8:
            raise ValueError("at most 8 eos ids")
        c.n_eos = len(eos)
        for i, t in enumerate(eos):
            c.eos_ids[i] = int(t)
        h = C.c_void_p()
        L.check(self.lib.ms_create(C.byref(c), C.byref(h)), None, "ms_create")
        self.h = h
        self.max_batch, self.max_ctx, self.max_prefill_tokens = max_batch, max_ctx, max_prefill_tokens
        self.device = device
        self._next_tag = 1
        self._mailbox = {}

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "h", None):
            self.lib.ms_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc, what):
        return L.check(rc, self.h, what)

    # ------------------------------------------------------------ weights
    def init_synthetic(self, seed: int = 0, std: float = 0.02, norm_jitter: float = 0.0):
        self._chk(self.lib.ms_init_synthetic(self.h, seed, std, norm_jitter), "ms_init_synthetic")

    def init_synthetic_q(self, seed: int = 2, scale: float = 0.02, norm_jitter: float = 0.0):
        """Random Q4_K/Q6_K blocks in the Q4_K_M per-tensor mix (BASELINE config 5)."""
        self._chk(self.lib.ms_init_synthetic_q(self.h, seed, scale, norm_jitter), "ms_init_synthetic_q")

    def load_tensor_q(self, tensor: int, layer: int, ggml_type: int, blocks: np.ndarray):
        b = np.ascontiguousarray(blocks, dtype=np.uint8)
        self._chk(self.lib.ms_load_weight_q(self.h, tensor, layer, ggml_type, b.ctypes.data, b.size),
                  "ms_load_weight_q")

    def weight_regions(self) -> list:
        """[(device pointer, bytes)] of every weight buffer, in the engine's fixed order."""
        n = self._chk(self.lib.ms_weight_regions(self.h, None, None, 0), "ms_weight_regions")
        ptrs, sizes = (C.c_void_p * n)(), (C.c_int64 * n)()
        self._chk(self.lib.ms_weight_regions(self.h, ptrs, sizes, n), "ms_weight_regions")
        return [(int(ptrs[i] or 0), int(sizes[i])) for i in range(n)]

    def quant_manifest(self) -> list:
        n = self._chk(self.lib.ms_quant_manifest(self.h, None, 0), "ms_quant_manifest")
        buf = (C.c_int32 * (3 * max(n, 1)))()
        self._chk(self.lib.ms_quant_manifest(self.h, buf, n), "ms_quant_manifest")
        return [tuple(buf[3 * i:3 * i + 3]) for i in range(n)]

    def declare_weight_q(self, tensor: int, layer: int, ggml_type: int):
        self._chk(self.lib.ms_declare_weight_q(self.h, tensor, layer, ggml_type), "ms_declare_weight_q")

    def load_tensor(self, tensor: int, layer: int, f16_bits: np.ndarray):
        """Upload one logical tensor as IEEE fp16 bit patterns (mapsum.weights.f32_to_f16_bits)."""
        a = np.ascontiguousarray(f16_bits, dtype=np.uint16)
        self._chk(self.lib.ms_load_weight(self.h, tensor, layer, a.ctypes.data, a.size), "ms_load_weight")

    def set_eos_ids(self, ids):
        """Replace the end-of-turn ids by a stop set (empty: back to the config's)."""
        a = np.ascontiguousarray(ids, dtype=np.int32)
        self._chk(self.lib.ms_set_eos_ids(self.h, a.ctypes.data_as(C.POINTER(C.c_int32)) if a.size else None,
                                          a.size), "ms_set_eos_ids")

    # ------------------------------------------------------------ request path
    def submit(self, ids, num_predict: int, ignore_eos: bool = False, tag: int | None = None) -> int:
        a = np.ascontiguousarray(ids, dtype=np.int32)
        if tag is None:
            tag = self._next_tag
            self._next_tag += 1
        flags = L.MS_FLAG_IGNORE_EOS if ignore_eos else 0
        self._chk(self.lib.ms_submit(self.h, a.ctypes.data_as(C.POINTER(C.c_int32)), a.size,
                                     int(num_predict), flags, int(tag)), "ms_submit")
        return tag

    def submit_forced(self, ids, forced, num_predict: int, ignore_eos: bool = True) -> int:
        """Teacher forcing through the decode path (parity tests): decode step j is fed
        ``forced[j-1]``; the result ids are the engine's own greedy choices."""
        a = np.ascontiguousarray(ids, dtype=np.int32)
        f = np.ascontiguousarray(forced, dtype=np.int32)
        if f.size == 0:
            f = np.zeros(1, np.int32)
        tag = self._next_tag
        self._next_tag += 1
        flags = L.MS_FLAG_IGNORE_EOS if ignore_eos else 0
        p32 = C.POINTER(C.c_int32)
        self._chk(self.lib.ms_submit_forced(self.h, a.ctypes.data_as(p32), a.size, f.ctypes.data_as(p32),
                                            f.size, int(num_predict), flags, int(tag)), "ms_submit_forced")
        return tag

    def generate_forced(self, prompts, forced, num_predict: int) -> list:
        """ids[j] = the engine's greedy choice at step j after prompt + forced[:j]."""
        tags = [self.submit_forced(p, f, num_predict) for p, f in zip(prompts, forced)]
        waiting = set(tags)
        got = {}
        while waiting:
            pending = self.step()
            self.collect()
            for t, r in self.take(waiting).items():
                waiting.discard(t)
                got[t] = r
            if pending == 0 and waiting and not any(t in self._mailbox for t in waiting):
                raise RuntimeError("engine drained without finishing every request")
        return [got[t] for t in tags]

    def step(self) -> int:
        return self._chk(self.lib.ms_step(self.h), "ms_step")

    def pending(self) -> int:
        return self._chk(self.lib.ms_pending(self.h), "ms_pending")

    def poll(self, cap: int = 256) -> list:
        buf = (L.MsResult * cap)()
        n = self._chk(self.lib.ms_poll(self.h, buf, cap), "ms_poll")
        out = []
        for i in range(n):
            r = buf[i]
            ids = [r.ids[j] for j in range(r.n_ids)] if r.n_ids else []
            out.append(Result(int(r.tag), ids, _FINISH.get(r.finish_reason, "error"), int(r.n_prompt)))
        return out

    # ------------------------------------------------------------ probes / stats
    def forward(self, ids, n_layers: int | None = None, hidden: bool = True, logits: bool = False):
        cfg = self.cfg
        a = np.ascontiguousarray(ids, dtype=np.int32)
        n = a.size
        nl = cfg.n_layers if n_layers is None else n_layers
        hid = np.empty((n, cfg.hidden), np.float32) if hidden else None
        lg = np.empty((n, cfg.vocab), np.float32) if logits else None
        self._chk(self.lib.ms_forward(self.h, a.ctypes.data_as(C.POINTER(C.c_int32)), n, nl,
                                      hid.ctypes.data if hid is not None else None,
                                      lg.ctypes.data if lg is not None else None), "ms_forward")
        return hid, lg

    def forward_packed(self, prompts, n_layers: int | None = None, hidden: bool = True, logits: bool = False):
        """ms_forward_packed: the prompts in ONE varlen prefill pass; rows in packed order."""
        cfg = self.cfg
        a = np.ascontiguousarray(np.concatenate([np.asarray(p, np.int32) for p in prompts]), dtype=np.int32)
        lens = np.ascontiguousarray([len(p) for p in prompts], dtype=np.int32)
        n = a.size
        nl = cfg.n_layers if n_layers is None else n_layers
        hid = np.empty((n, cfg.hidden), np.float32) if hidden else None
        lg = np.empty((n, cfg.vocab), np.float32) if logits else None
        p32 = C.POINTER(C.c_int32)
        self._chk(self.lib.ms_forward_packed(self.h, a.ctypes.data_as(p32), lens.ctypes.data_as(p32), lens.size,
                                             nl, hid.ctypes.data if hid is not None else None,
                                             lg.ctypes.data if lg is not None else None), "ms_forward_packed")
        return hid, lg

    def set_profiling(self, mask: int):
        self._chk(self.lib.ms_set_profiling(self.h, mask), "ms_set_profiling")

    def reset_stats(self):
        self._chk(self.lib.ms_reset_stats(self.h), "ms_reset_stats")

    def synchronize(self):
        self._chk(self.lib.ms_synchronize(self.h), "ms_synchronize")

    def stats(self) -> dict:
        s = L.MsStats()
        self._chk(self.lib.ms_get_stats(self.h, C.byref(s)), "ms_get_stats")
        return {"prefill_tokens": s.prefill_tokens, "decode_tokens": s.decode_tokens,
                "prefill_passes": s.prefill_passes, "decode_steps": s.decode_steps,
                "finished": s.finished, "prefill_ms": s.prefill_ms, "decode_ms": s.decode_ms,
                "kernel_ms": list(s.kernel_ms), "kernel_launches": list(s.kernel_launches),
                "decode_kv_tokens": s.decode_kv_tokens, "graphs_built": s.graphs_built,
                "persist_fallbacks": s.persist_fallbacks, "persist_steps": s.persist_steps}

    def set_persist(self, on: bool) -> bool:
        """The decode step's layers as one persistent launch (k_persist.hip) or the per-layer
        launches; returns whether this engine supports the persistent step at all."""
        return bool(self._chk(self.lib.ms_set_persist(self.h, 1 if on else 0), "ms_set_persist"))

    def debug_read(self, which: int, offset: int, nbytes: int) -> np.ndarray:
        """Test hook: `nbytes` of an engine buffer (L.MS_DBG_*) from byte `offset`, as uint8."""
        out = np.empty(nbytes, np.uint8)
        self._chk(self.lib.ms_debug_read(self.h, which, offset, out.ctypes.data, nbytes), "ms_debug_read")
        return out
