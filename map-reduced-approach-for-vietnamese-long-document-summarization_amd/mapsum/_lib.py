"""ctypes binding of libmapsum.so (C-ABI declared in include/mapsum.h).

The library is built in-tree (``make -C csrc`` / ``__graft_entry__.build()``).  There
is no fallback: if it is missing or fails to load, ``load()`` raises, so the product
path can never silently run on anything but the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MAPSUM_LIB: an alternative in-tree build of the same library (A/B timing of build variants)
LIB_PATH = os.environ.get("MAPSUM_LIB") or os.path.join(_HERE, "libmapsum.so")

MS_ABI_VERSION = 3
MS_OK, MS_EIO, MS_ENOMEM, MS_EBUSY, MS_EINVAL, MS_ENOSPC = 0, -5, -12, -16, -22, -28
MS_FINISH_EOS, MS_FINISH_LENGTH, MS_FINISH_ERROR = 1, 2, 3
MS_FLAG_IGNORE_EOS = 1
(MS_T_EMBED, MS_T_ATTN_NORM, MS_T_WQ, MS_T_WK, MS_T_WV, MS_T_WO, MS_T_FFN_NORM, MS_T_WGATE,
 MS_T_WUP, MS_T_WDOWN, MS_T_FINAL_NORM, MS_T_LM_HEAD) = range(12)
MS_EPI_STORE_F16, MS_EPI_ADD_F32, MS_EPI_SWIGLU, MS_EPI_STORE_F32 = range(4)
MS_EPI_ARGMAX = 5
# the prefill GEMM dispatch the library starts with (ms_set_gemm_variant; tests restore it)
GEMM_DEFAULT = 4
MS_GGML_Q4_K, MS_GGML_Q6_K = 12, 14
# kernel classes of ms_stats.kernel_ms
K_GEMM, K_ATTN_PREFILL, K_GEMV, K_ATTN_DECODE, K_LMHEAD, K_MISC, K_PERSIST = range(7)
MS_DBG_KPOOL, MS_DBG_VPOOL, MS_DBG_DECODE_LOGITS, MS_DBG_DECODE_X = range(4)

EXPORTED = (
    "ms_create", "ms_destroy", "ms_last_error", "ms_load_weight", "ms_init_synthetic",
    "ms_load_weight_q", "ms_init_synthetic_q", "ms_op_dequant", "ms_op_quant_rows", "ms_op_qgemv", "ms_op_qgemv_split", "ms_op_qdgemm",
    "ms_submit", "ms_step", "ms_poll", "ms_pending", "ms_get_stats", "ms_reset_stats",
    "ms_set_profiling", "ms_synchronize", "ms_forward", "ms_op_gemm", "ms_op_gemv_workspace",
    "ms_op_gemv", "ms_op_gemv_tuned", "ms_op_gemv_split", "ms_op_dgemm", "ms_op_residual_rmsnorm", "ms_op_rmsnorm",
    "ms_op_argmax", "ms_op_argmax_partials", "ms_set_gemm_variant", "ms_set_qgemv_gs", "ms_set_attn_tuning", "ms_set_dgemm_kh", "ms_set_dgemm_wn",
    "ms_weight_regions", "ms_quant_manifest", "ms_declare_weight_q",
    "ms_forward_packed", "ms_submit_forced", "ms_set_eos_ids", "ms_op_gemv_strided",
    "ms_op_gemv_resid", "ms_op_set_row_scale", "ms_op_gemm_resid", "ms_gemm_resid_tiles",
    "ms_trace_push", "ms_trace_pop", "ms_debug_a2_stamps", "ms_set_persist", "ms_debug_read", "ms_debug_pk_stamps",
)


class MsConfig(C.Structure):
    _fields_ = [("abi_version", C.c_int32),
                ("n_layers", C.c_int32), ("hidden", C.c_int32), ("n_heads", C.c_int32),
                ("n_kv_heads", C.c_int32), ("head_dim", C.c_int32), ("ffn", C.c_int32),
                ("vocab", C.c_int32),
                ("rope_theta", C.c_float), ("rope_factor", C.c_float),
                ("rope_low_freq_factor", C.c_float), ("rope_high_freq_factor", C.c_float),
                ("rope_orig_ctx", C.c_int32), ("norm_eps", C.c_float), ("tie_embeddings", C.c_int32),
                ("device", C.c_int32), ("max_batch", C.c_int32), ("max_ctx", C.c_int32),
                ("max_prefill_tokens", C.c_int32), ("n_pages", C.c_int32), ("n_eos", C.c_int32),
                ("eos_ids", C.c_int32 * 8)]


class MsResult(C.Structure):
    _fields_ = [("tag", C.c_uint64), ("ids", C.POINTER(C.c_int32)), ("n_ids", C.c_int32),
                ("finish_reason", C.c_int32), ("n_prompt", C.c_int32), ("_pad", C.c_int32)]


class MsStats(C.Structure):
    _fields_ = [("prefill_tokens", C.c_int64), ("decode_tokens", C.c_int64),
                ("prefill_passes", C.c_int64), ("decode_steps", C.c_int64), ("finished", C.c_int64),
                ("prefill_ms", C.c_double), ("decode_ms", C.c_double),
                ("kernel_ms", C.c_double * 8), ("kernel_launches", C.c_int64 * 8),
                ("decode_kv_tokens", C.c_int64), ("graphs_built", C.c_int64),
                ("persist_fallbacks", C.c_int64), ("persist_steps", C.c_int64)]


_lib = None


def load() -> C.CDLL:
    """Load libmapsum.so (raises if it was not built -- there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libmapsum.so not found at {LIB_PATH}; build it with "
                           f"`make -C csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
    _lib = load_at(LIB_PATH, bool(os.environ.get("MAPSUM_LIB")))
    return _lib


def load_at(path: str, ab: bool = True) -> C.CDLL:
    """A build of the library at `path` with the C-ABI signatures set (tools: same-process A/B
    of two builds; ab: tolerate entry points an older build lacks)."""
    lib = C.CDLL(path)
    vp, i32, i64, u32, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
    pi32 = C.POINTER(C.c_int32)
    sig = {
        "ms_create": (i32, [C.POINTER(MsConfig), C.POINTER(vp)]),
        "ms_destroy": (i32, [vp]),
        "ms_last_error": (C.c_char_p, [vp]),
        "ms_load_weight": (i32, [vp, i32, i32, vp, i64]),
        "ms_init_synthetic": (i32, [vp, u64, C.c_float, C.c_float]),
        "ms_load_weight_q": (i32, [vp, i32, i32, i32, vp, i64]),
        "ms_init_synthetic_q": (i32, [vp, u64, C.c_float, C.c_float]),
        "ms_op_dequant": (i32, [i32, vp, i64, vp, vp]),
        "ms_op_quant_rows": (i32, [i32, vp, i32, i32, vp, vp, vp]),
        "ms_op_qgemv": (i32, [vp, i32, vp, vp, i32, i32, i32, i32, i32, vp]),
        "ms_op_qgemv_split": (i32, [vp, i32, vp, vp, i32, i32, i32, i32, vp]),
        "ms_op_qdgemm": (i32, [vp, i32, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
        "ms_submit": (i32, [vp, pi32, i32, i32, u32, u64]),
        "ms_step": (i32, [vp]),
        "ms_poll": (i32, [vp, C.POINTER(MsResult), i32]),
        "ms_pending": (i32, [vp]),
        "ms_get_stats": (i32, [vp, C.POINTER(MsStats)]),
        "ms_reset_stats": (i32, [vp]),
        "ms_set_profiling": (i32, [vp, u32]),
        "ms_synchronize": (i32, [vp]),
        "ms_forward": (i32, [vp, pi32, i32, i32, vp, vp]),
        "ms_forward_packed": (i32, [vp, pi32, pi32, i32, i32, vp, vp]),
        "ms_set_eos_ids": (i32, [vp, pi32, i32]),
        "ms_op_gemv_strided": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
        "ms_op_gemv_resid": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp]),
        "ms_op_set_row_scale": (i32, [vp, i32, i32, C.c_float]),
        "ms_op_gemm_resid": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, vp]),
        "ms_gemm_resid_tiles": (i32, [i32, i32]),
        "ms_submit_forced": (i32, [vp, pi32, i32, pi32, i32, i32, u32, u64]),
        "ms_op_gemm": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp]),
        "ms_op_gemv_workspace": (i64, [i32, i32, i32]),
        "ms_op_gemv": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, vp]),
        "ms_op_gemv_tuned": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp]),
        "ms_op_gemv_split": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp]),
        "ms_op_dgemm": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
        "ms_op_residual_rmsnorm": (i32, [vp, vp, i32, vp, vp, vp, i32, i32, vp]),
        "ms_op_rmsnorm": (i32, [vp, vp, vp, vp, i32, i32, vp, vp]),
        "ms_set_gemm_variant": (i32, [i32]),
        "ms_set_qgemv_gs": (i32, [i32]),
        "ms_set_attn_tuning": (i32, [i32, i32]),
        "ms_set_dgemm_kh": (i32, [i32]),
        "ms_set_dgemm_wn": (i32, [i32]),
        "ms_op_argmax": (i32, [vp, i32, i32, vp, vp]),
        "ms_op_argmax_partials": (i32, [vp, i32, i32, vp, vp]),
        "ms_weight_regions": (i32, [vp, C.POINTER(vp), C.POINTER(i64), i32]),
        "ms_quant_manifest": (i32, [vp, pi32, i32]),
        "ms_declare_weight_q": (i32, [vp, i32, i32, i32]),
        "ms_trace_push": (i32, [C.c_char_p]),
        "ms_trace_pop": (i32, []),
        "ms_set_persist": (i32, [vp, i32]),
        "ms_debug_read": (i32, [vp, i32, i64, vp, i64]),
        "ms_debug_pk_stamps": (i32, [vp, i32]),
        "ms_debug_a2_stamps": (i32, [vp, i32]),
    }
    for name, (res, args) in sig.items():
        if ab and not hasattr(lib, name):  # an A/B build may predate the newest op hooks
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def check(rc: int, handle=None, what: str = "") -> int:
    """Raise RuntimeError on a negative status (mirrors resp.raise_for_status(),
    run_full_evaluation_pipeline.py:91)."""
    if rc < 0:
        msg = load().ms_last_error(handle)
        raise RuntimeError(f"libmapsum {what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


class trace:
    """``with trace("mapsum.gather"):`` -- a roctx range (ms_trace_push / ms_trace_pop) around a
    host phase, shown by rocprofv3 --marker-trace next to the engine's own ranges; a no-op when
    libmapsum cannot be loaded (CPU-only tests of the host code)."""

    def __init__(self, name: str):
        self.name = name.encode()
        self.lib = None

    def __enter__(self):
        try:
            lib = load()
            if hasattr(lib, "ms_trace_push"):
                lib.ms_trace_push(self.name)
                self.lib = lib
        except (OSError, RuntimeError):
            self.lib = None
        return self

    def __exit__(self, *exc):
        if self.lib is not None:
            self.lib.ms_trace_pop()
        return False
