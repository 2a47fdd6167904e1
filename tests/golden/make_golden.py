"""Generate tests/golden/hf_tiny_llama.npz -- the fixture that pins the oracle.

The reference's arithmetic (Ollama/llama.cpp running Llama-3.2) is not in this
container (parity against Ollama is unpinned).  What *can* be pinned
is the architecture restatement in oracle/llama_ref.py: this script builds
``transformers.LlamaForCausalLM`` (the public Llama-3.2 implementation, llama3 RoPE
scaling, tied embeddings, GQA) with the TINY shape, copies in the oracle's seeded
synthetic weights, and records its outputs.  tests/test_oracle.py checks the oracle
(fp32 mode: bit-for-bit the same arithmetic, different summation order) against it.

Run:  python tests/golden/make_golden.py      (CPU, a few seconds)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))

from mapsum.config import TINY  # noqa: E402
from oracle.synth import make_weights  # noqa: E402

SEED, STD, JITTER = 4321, 0.05, 0.1
N_PROMPT, N_GEN = 48, 24


def hf_model(cfg, w):
    from transformers import LlamaConfig, LlamaForCausalLM
    hc = LlamaConfig(
        vocab_size=cfg.vocab, hidden_size=cfg.hidden, intermediate_size=cfg.ffn,
        num_hidden_layers=cfg.n_layers, num_attention_heads=cfg.n_heads,
        num_key_value_heads=cfg.n_kv_heads, head_dim=cfg.head_dim, rms_norm_eps=cfg.norm_eps,
        rope_parameters={"rope_type": "llama3", "rope_theta": cfg.rope_theta, "factor": cfg.rope_factor,
                         "low_freq_factor": cfg.rope_low_freq_factor,
                         "high_freq_factor": cfg.rope_high_freq_factor,
                         "original_max_position_embeddings": cfg.rope_orig_ctx},
        tie_word_embeddings=cfg.tie_embeddings, max_position_embeddings=131072,
        attention_bias=False, mlp_bias=False)
    m = LlamaForCausalLM(hc).float().eval()
    sd = {"model.embed_tokens.weight": w["embed"], "model.norm.weight": w["final_norm"]}
    for i, L in enumerate(w["layers"]):
        p = f"model.layers.{i}."
        sd[p + "input_layernorm.weight"] = L["attn_norm"]
        sd[p + "self_attn.q_proj.weight"] = L["wq"]
        sd[p + "self_attn.k_proj.weight"] = L["wk"]
        sd[p + "self_attn.v_proj.weight"] = L["wv"]
        sd[p + "self_attn.o_proj.weight"] = L["wo"]
        sd[p + "post_attention_layernorm.weight"] = L["ffn_norm"]
        sd[p + "mlp.gate_proj.weight"] = L["w_gate"]
        sd[p + "mlp.up_proj.weight"] = L["w_up"]
        sd[p + "mlp.down_proj.weight"] = L["w_down"]
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected and all("lm_head" in k for k in missing), (missing, unexpected)
    return m


def main():
    torch.manual_seed(0)
    w = make_weights(TINY, SEED, std=STD, jitter=JITTER)
    m = hf_model(TINY, w)
    ids = np.random.default_rng(11).integers(0, 4000, size=N_PROMPT).astype(np.int64)
    layer_out = []
    hooks = [ly.register_forward_hook(lambda mod, inp, out: layer_out.append(
        (out[0] if isinstance(out, tuple) else out).detach()[0].numpy().copy()))
        for ly in m.model.layers]
    with torch.no_grad():
        lg = m(torch.from_numpy(ids)[None]).logits[0].numpy()
    for h in hooks:
        h.remove()
    with torch.no_grad():
        gen = m.generate(torch.from_numpy(ids)[None], max_new_tokens=N_GEN, do_sample=False,
                         min_new_tokens=N_GEN, pad_token_id=0)[0, N_PROMPT:].numpy()
    top = np.argsort(-lg, axis=1, kind="stable")[:, :16]
    np.savez_compressed(
        os.path.join(HERE, "hf_tiny_llama.npz"),
        seed=SEED, std=STD, jitter=JITTER, ids=ids.astype(np.int32),
        last_logits=lg[-1].astype(np.float32),
        top16_idx=top.astype(np.int32), top16_val=np.take_along_axis(lg, top, 1).astype(np.float32),
        hidden_head=np.stack([h[:, :32] for h in layer_out]).astype(np.float32),
        hidden_norm=np.stack([np.linalg.norm(h, axis=1) for h in layer_out]).astype(np.float32),
        greedy=gen.astype(np.int32),
        transformers_version=np.array(__import__("transformers").__version__))
    print("wrote hf_tiny_llama.npz; greedy:", gen.tolist())


if __name__ == "__main__":
    main()
