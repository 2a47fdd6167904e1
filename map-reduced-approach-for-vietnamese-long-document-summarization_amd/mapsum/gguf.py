"""GGUF reader and loader: the weights Ollama serves (`ollama pull llama3.2:3b`,
README.md:28-33) straight into a libmapsum engine.

Format (EXT, ggml's published GGUF v2/v3): magic "GGUF", version, tensor count, metadata
key/values, tensor infos (name, dims innermost first, ggml type, offset), then the tensor
data at ``general.alignment`` (default 32).  The file is memory-mapped; nothing in it is
executed.

llama.cpp's HF -> GGUF converter permutes the rows of attn_q / attn_k per head so that
rotary pairs are adjacent (``permute``: reshape(n_head, 2, hd/2) -> swap -> flatten).
The kernels implement HF's rotate-half convention, so those rows are put back here.  A
row of a quantised matrix is a whole run of blocks, so the same row permutation applies
to Q4_K / Q6_K data without dequantising.

Supported: every matrix float (F32 / F16 / BF16, uploaded as fp16 -- the engine's type, so an
F16 file such as llama3.2:3b-instruct-fp16 loads bit for bit) or every matrix Q4_K / Q6_K (the
Q4_K_M mix) with float norms.
"""
from __future__ import annotations

import struct

import numpy as np

from .weights import load_logical, load_quantized

GGML_F32, GGML_F16, GGML_Q4_K, GGML_Q6_K, GGML_BF16 = 0, 1, 12, 14, 30
QBLOCK = {GGML_Q4_K: (256, 144), GGML_Q6_K: (256, 210)}  # weights, bytes per block
_FLOAT = {GGML_F32: np.float32, GGML_F16: np.float16}

# value types of the metadata section
_SCALAR = {0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?", 10: "<Q", 11: "<q",
           12: "<d"}


class GGUFError(ValueError):
    pass


class _Cursor:
    def __init__(self, buf):
        self.buf, self.off = buf, 0

    def take(self, fmt):
        v = struct.unpack_from(fmt, self.buf, self.off)[0]
        self.off += struct.calcsize(fmt)
        return v

    def string(self):
        n = self.take("<Q")
        s = bytes(self.buf[self.off:self.off + n]).decode("utf-8")
        self.off += n
        return s

    def value(self, t):
        if t in _SCALAR:
            return self.take(_SCALAR[t])
        if t == 8:
            return self.string()
        if t == 9:
            et, n = self.take("<I"), self.take("<Q")
            return [self.value(et) for _ in range(n)]
        raise GGUFError(f"unknown metadata value type {t}")


def read_gguf(path: str):
    """-> (metadata dict, {name: (ggml_type, dims innermost-first, uint8 memmap view)})."""
    buf = np.memmap(path, dtype=np.uint8, mode="r")
    c = _Cursor(buf)
    if bytes(buf[:4]) != b"GGUF":
        raise GGUFError("not a GGUF file")
    c.off = 4
    version = c.take("<I")
    if version not in (2, 3):
        raise GGUFError(f"unsupported GGUF version {version}")
    n_tensors, n_kv = c.take("<Q"), c.take("<Q")
    meta = {}
    for _ in range(n_kv):
        k = c.string()
        meta[k] = c.value(c.take("<I"))
    infos = []
    for _ in range(n_tensors):
        name = c.string()
        nd = c.take("<I")
        dims = [c.take("<Q") for _ in range(nd)]
        infos.append((name, dims, c.take("<I"), c.take("<Q")))
    align = int(meta.get("general.alignment", 32))
    base = (c.off + align - 1) // align * align
    tensors = {}
    for name, dims, t, off in infos:
        n = int(np.prod(dims))
        if t in _FLOAT:
            nbytes = n * np.dtype(_FLOAT[t]).itemsize
        elif t == GGML_BF16:
            nbytes = 2 * n
        elif t in QBLOCK:
            qk, qb = QBLOCK[t]
            if dims[0] % qk:
                raise GGUFError(f"{name}: row length {dims[0]} not a multiple of {qk}")
            nbytes = n // qk * qb
        else:
            raise GGUFError(f"{name}: ggml type {t} is not supported (F32/F16/BF16/Q4_K/Q6_K)")
        start = base + off
        if start + nbytes > buf.size:
            raise GGUFError(f"{name}: data runs past the end of the file")
        tensors[name] = (t, dims, buf[start:start + nbytes])
    return meta, tensors


def _rows(t, dims, raw):
    """Matrix as rows: float32 [rows][K] for float types, uint8 [rows][bytes] for K-quants."""
    K, rows = dims[0], int(np.prod(dims[1:])) if len(dims) > 1 else 1
    if t in _FLOAT:
        return np.frombuffer(raw, dtype=_FLOAT[t]).astype(np.float32).reshape(rows, K)
    if t == GGML_BF16:
        return (np.frombuffer(raw, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32).reshape(rows, K)
    return np.asarray(raw).reshape(rows, -1)


def unpermute_rows(a: np.ndarray, n_head: int) -> np.ndarray:
    """Inverse of llama.cpp's converter ``permute`` on the row axis."""
    r = a.shape[0]
    return a.reshape(n_head, r // n_head // 2, 2, *a.shape[1:]).swapaxes(1, 2).reshape(a.shape)


def permute_rows(a: np.ndarray, n_head: int) -> np.ndarray:
    """llama.cpp's converter ``permute`` (for building test files)."""
    r = a.shape[0]
    return a.reshape(n_head, 2, r // n_head // 2, *a.shape[1:]).swapaxes(1, 2).reshape(a.shape)


_LAYER = {"attn_q": "wq", "attn_k": "wk", "attn_v": "wv", "attn_output": "wo", "ffn_gate": "w_gate",
          "ffn_up": "w_up", "ffn_down": "w_down"}


def check_rope_freqs(cfg, ts):
    """The GGUF's rope_freqs.weight (llama.cpp's llama3 scaling divisors) must be the engine's own
    table (config.llama3_rope_factors: the cos / sin tables are built from cfg, not from the
    file), or the model would silently run with another RoPE -- refuse.  A file without the
    tensor is accepted only for an unscaled config (rope_factor 0)."""
    from .config import llama3_rope_factors
    want = llama3_rope_factors(cfg)
    if "rope_freqs.weight" not in ts:
        if cfg.rope_factor and cfg.rope_factor > 0:
            raise GGUFError("no rope_freqs.weight tensor: the engine applies llama3 RoPE scaling "
                            f"(factor {cfg.rope_factor}); a GGUF without it is another RoPE")
        return
    t, d, raw = ts["rope_freqs.weight"]
    if t in QBLOCK:
        raise GGUFError("rope_freqs.weight: quantised")
    got = _rows(t, d, raw).reshape(-1).astype(np.float64)
    if got.shape != want.shape or not np.allclose(got, want, rtol=1e-5, atol=0.0):
        bad = int(np.argmax(np.abs(got - want) / want)) if got.shape == want.shape else -1
        raise GGUFError(f"rope_freqs.weight does not match the engine's llama3 RoPE scaling (theta "
                        f"{cfg.rope_theta}, factor {cfg.rope_factor}, low/high {cfg.rope_low_freq_factor}/"
                        f"{cfg.rope_high_freq_factor}, orig ctx {cfg.rope_orig_ctx}): first mismatch at "
                        f"frequency {bad} -- refusing to run this model with another RoPE")


def load_gguf(engine, path: str):
    """Upload a llama-architecture GGUF into ``engine`` (shape checked against engine.cfg)."""
    cfg = engine.cfg
    meta, ts = read_gguf(path)
    arch = meta.get("general.architecture", "llama")
    if arch != "llama":
        raise GGUFError(f"architecture {arch!r} is not llama")
    for key, want in (("block_count", cfg.n_layers), ("embedding_length", cfg.hidden),
                      ("attention.head_count", cfg.n_heads), ("attention.head_count_kv", cfg.n_kv_heads)):
        got = meta.get(f"llama.{key}")
        if got is not None and int(got) != want:
            raise GGUFError(f"llama.{key} = {got}, engine config has {want}")

    def get(name):
        if name not in ts:
            raise GGUFError(f"missing tensor {name}")
        return ts[name]

    check_rope_freqs(cfg, ts)
    mats = {"embed": get("token_embd.weight")}
    if "output.weight" in ts and not cfg.tie_embeddings:
        mats["lm_head"] = ts["output.weight"]
    for i in range(cfg.n_layers):
        for g, n in _LAYER.items():
            mats[(i, n)] = get(f"blk.{i}.{g}.weight")
    heads = {"wq": cfg.n_heads, "wk": cfg.n_kv_heads}

    def norm(name):
        t, d, raw = get(name)
        if t in QBLOCK:
            raise GGUFError(f"{name}: quantised norms are not supported")
        return _rows(t, d, raw).reshape(-1)

    norms = {"final_norm": norm("output_norm.weight"),
             "layers": [{"attn_norm": norm(f"blk.{i}.attn_norm.weight"),
                         "ffn_norm": norm(f"blk.{i}.ffn_norm.weight")} for i in range(cfg.n_layers)]}
    quant = {k: v[0] in QBLOCK for k, v in mats.items()}
    if all(quant.values()):
        qw = {}
        for k, (t, d, raw) in mats.items():
            rows = _rows(t, d, raw)
            name = k if isinstance(k, str) else k[1]
            if name in heads:
                rows = unpermute_rows(rows, heads[name])
            qw[k] = (t, np.ascontiguousarray(rows).reshape(-1))
        load_quantized(engine, qw, norms)
    elif not any(quant.values()):
        w = {"embed": _rows(*mats["embed"]), "final_norm": norms["final_norm"], "layers": []}
        if "lm_head" in mats:
            w["lm_head"] = _rows(*mats["lm_head"])
        for i in range(cfg.n_layers):
            ly = dict(norms["layers"][i])
            for n in _LAYER.values():
                a = _rows(*mats[(i, n)])
                ly[n] = unpermute_rows(a, heads[n]) if n in heads else a
            w["layers"].append(ly)
        load_logical(engine, w)
    else:
        raise GGUFError("mixed float / K-quant matrices are not supported")
    return meta
