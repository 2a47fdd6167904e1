"""Weight upload into a libmapsum engine.

Sources:
  * a logical weight dict (``oracle.synth.make_weights`` layout: float32 arrays holding
    bf16 values, which fp16 holds exactly) -- used by the parity tests;
  * a Hugging Face Llama-3.2 checkpoint directory (``*.safetensors``; rotate-half RoPE
    convention, which is what the kernels implement) -- the real-weight path.  The
    reference pulls ``llama3.2:3b`` through Ollama (README.md:28-33); its GGUF blobs load
    through ``mapsum.gguf.load_gguf`` (Q/K un-permutation, float or Q4_K/Q6_K matrices).
The engine itself fuses Q|K|V and interleaves gate/up rows on upload (csrc/engine.cpp
``ms_load_weight``), so callers always pass nn.Linear [out][in] tensors.
"""
from __future__ import annotations

import glob
import os

import numpy as np

from . import _lib as L


def f32_to_f16_bits(a: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even float32 -> IEEE fp16 bit patterns (uint16): the engine's weight
    type (include/mapsum.h ms_load_weight), as llama.cpp's F16 GGUF converter rounds them."""
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32).astype(np.float16)).view(np.uint16)


def load_logical(engine, w: dict):
    """Upload a logical weight dict ({embed, final_norm, lm_head, layers[...]})."""
    cfg = engine.cfg
    up = lambda t, l, a: engine.load_tensor(t, l, f32_to_f16_bits(a))  # noqa: E731
    up(L.MS_T_EMBED, 0, w["embed"])
    up(L.MS_T_FINAL_NORM, 0, w["final_norm"])
    if not cfg.tie_embeddings:
        up(L.MS_T_LM_HEAD, 0, w["lm_head"])
    for i, ly in enumerate(w["layers"]):
        up(L.MS_T_ATTN_NORM, i, ly["attn_norm"])
        up(L.MS_T_WQ, i, ly["wq"])
        up(L.MS_T_WK, i, ly["wk"])
        up(L.MS_T_WV, i, ly["wv"])
        up(L.MS_T_WO, i, ly["wo"])
        up(L.MS_T_FFN_NORM, i, ly["ffn_norm"])
        up(L.MS_T_WGATE, i, ly["w_gate"])
        up(L.MS_T_WUP, i, ly["w_up"])
        up(L.MS_T_WDOWN, i, ly["w_down"])


_Q_NAMES = {"embed": L.MS_T_EMBED, "lm_head": L.MS_T_LM_HEAD, "wq": L.MS_T_WQ, "wk": L.MS_T_WK,
            "wv": L.MS_T_WV, "wo": L.MS_T_WO, "w_gate": L.MS_T_WGATE, "w_up": L.MS_T_WUP,
            "w_down": L.MS_T_WDOWN}


def load_quantized(engine, qw: dict, norms: dict):
    """Upload a K-quant model: qw[name] = (ggml_type, uint8 blocks) for "embed"/"lm_head" and
    qw[(layer, name)] for the per-layer matrices (rows of raw ggml blocks, GGUF order after
    Q/K un-permutation); norms = {"final_norm": f32, "layers": [{"attn_norm", "ffn_norm"}]}."""
    cfg = engine.cfg
    for key, (qt, blocks) in qw.items():
        layer, name = (0, key) if isinstance(key, str) else key
        engine.load_tensor_q(_Q_NAMES[name], layer, qt, blocks)
    engine.load_tensor(L.MS_T_FINAL_NORM, 0, f32_to_f16_bits(norms["final_norm"]))
    for i, ly in enumerate(norms["layers"]):
        engine.load_tensor(L.MS_T_ATTN_NORM, i, f32_to_f16_bits(ly["attn_norm"]))
        engine.load_tensor(L.MS_T_FFN_NORM, i, f32_to_f16_bits(ly["ffn_norm"]))
    if len([k for k in qw if not isinstance(k, str)]) != 7 * cfg.n_layers:
        raise RuntimeError("quantised model is missing per-layer matrices")


_HF_LAYER = {
    "input_layernorm.weight": L.MS_T_ATTN_NORM,
    "self_attn.q_proj.weight": L.MS_T_WQ,
    "self_attn.k_proj.weight": L.MS_T_WK,
    "self_attn.v_proj.weight": L.MS_T_WV,
    "self_attn.o_proj.weight": L.MS_T_WO,
    "post_attention_layernorm.weight": L.MS_T_FFN_NORM,
    "mlp.gate_proj.weight": L.MS_T_WGATE,
    "mlp.up_proj.weight": L.MS_T_WUP,
    "mlp.down_proj.weight": L.MS_T_WDOWN,
}


def _bits(t) -> np.ndarray:
    try:
        import torch
        if isinstance(t, torch.Tensor):
            if t.dtype == torch.float16:
                return t.contiguous().view(torch.int16).numpy().view(np.uint16)
            return f32_to_f16_bits(t.float().numpy())
    except ImportError:  # pragma: no cover
        pass
    return f32_to_f16_bits(np.asarray(t, dtype=np.float32))


def load_hf_state_dict(engine, sd: dict):
    """Upload HF Llama tensors (names as in LlamaForCausalLM.state_dict())."""
    cfg = engine.cfg
    seen = set()
    for name, t in sd.items():
        if name == "model.embed_tokens.weight":
            engine.load_tensor(L.MS_T_EMBED, 0, _bits(t))
        elif name == "model.norm.weight":
            engine.load_tensor(L.MS_T_FINAL_NORM, 0, _bits(t))
        elif name == "lm_head.weight":
            if not cfg.tie_embeddings:
                engine.load_tensor(L.MS_T_LM_HEAD, 0, _bits(t))
        elif name.startswith("model.layers."):
            rest = name[len("model.layers."):]
            idx, _, key = rest.partition(".")
            if key in _HF_LAYER:
                engine.load_tensor(_HF_LAYER[key], int(idx), _bits(t))
            else:
                continue
        else:
            continue
        seen.add(name)
    need = 2 + 9 * cfg.n_layers + (0 if cfg.tie_embeddings else 1)
    if len(seen) < need:
        raise RuntimeError(f"checkpoint is missing tensors: got {len(seen)} of {need}")


def load_hf_dir(engine, path: str):
    from safetensors.torch import load_file
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {path}")
    sd = {}
    for f in files:
        sd.update(load_file(f))
    load_hf_state_dict(engine, sd)
