"""TEST INFRASTRUCTURE ONLY -- the "sharp" synthetic Llama-3.2-3B of the 28-layer greedy fixture.

Why a second synthetic model.  The bench's random-init weights give FLAT logits: the top-2
gap over 128256 ids is the spacing of the largest of 128k Gaussians (median ~0.19 logits),
and the engine-vs-oracle logit error is RELATIVE (it comes from bf16 rounding flips inside
the stack, so scaling the final norm or the lm_head scales gap and error together).  A few
per cent of greedy positions are therefore near-ties, and after the first such flip a
free-running continuation diverges.  The north star's literal bar -- >= 99 % of the first
128 free-running greedy tokens equal (BASELINE.json) -- is only testable on a model whose
greedy choices are decisive.  Sharpening by a gain cannot do that; structure can.

The design: the bench weights (oracle/synth.py, seed/std/jitter of the fixture) with five
tensors replaced, all seeded numpy (identical here and on the GPU box):
  * embedding (tied lm_head): E[v] = bf16(N(0, 0.02) + u), where u is one fixed vector on
    dims 1024..3071 with |u| = 2 |E_rand| -- a shared direction every token carries;
  * layer 0 Wq / Wk: rank one, u -> a fixed q / k vector on the 8 highest-frequency RoPE pairs,
    with q's phases set so that q(m).k(n) peaks at m - n = COPY_OFFSET (llama3 RoPE of the
    engine, pairs (i, i+64)): every query attends ~one-hot to the key COPY_OFFSET back;
  * layer 0 Wv / Wo: v = the query-free dims 0..1023 of the normalised input, o written back
    to the same residual dims with gain 14 per head.
The residual then carries the embedding of token p - COPY_OFFSET and, through the tied
lm_head, greedy decoding continues the prompt periodically: token(p+1) = token(p - 36).  That
choice is decisive (top-2 gap ~28 logits vs a logit error ~1e-2) and it depends on RoPE
positions, on K/V written by earlier decode steps, on page crossings and on the argmax
feedback -- through all 28 layers, which keep their random-init weights.
"""
from __future__ import annotations

import math

import numpy as np

from oracle.llama_ref import rope_inv_freq
from oracle.synth import ATTN_NORM, bf16_rne, norm

COPY_OFFSET = 36
DESIGN_SEED = 2024
N_PAIRS, PAIR_AMP, U_RATIO, O_GAIN, EMB_STD = 8, 14.1, 2.0, 14.0, 0.02


def copy_head_overrides(cfg, base_seed: int, jitter: float) -> dict:
    """{"embed": [V][H], "wq" / "wk" / "wv" / "wo": layer-0 matrices} as float32 holding bf16
    values, HF nn.Linear layout.  ``base_seed`` / ``jitter`` are those of the synthetic base
    weights (layer 0's attn_norm enters the query scale)."""
    rng = np.random.default_rng(DESIGN_SEED)
    H, D, Hq, Hk, V = cfg.hidden, cfg.head_dim, cfg.n_heads, cfg.n_kv_heads, cfg.vocab
    NC = Hk * D  # copied dims 0..NC-1 (one head_dim slice per kv head)
    u = np.zeros(H, np.float32)
    u[NC:] = np.where(rng.random(H - NC) < 0.5, -1.0, 1.0)
    u *= np.float32(U_RATIO * EMB_STD * math.sqrt(H) / np.linalg.norm(u))
    E = np.empty((V, H), np.float32)
    step = 8192
    for r0 in range(0, V, step):
        r1 = min(V, r0 + step)
        E[r0:r1] = bf16_rne(rng.standard_normal((r1 - r0, H), dtype=np.float32) * np.float32(EMB_STD) + u)
    uh = (u / np.linalg.norm(u)).astype(np.float32)
    # c = u_hat . rmsnorm(E[t]) * g0, nearly the same for every token (|u| dominates)
    g0 = norm(base_seed, ATTN_NORM, 0, H, jitter)
    probe = E[:: max(1, V // 512)]
    xn = probe / np.sqrt(np.mean(probe.astype(np.float64) ** 2, 1, keepdims=True)) * g0
    c = float(np.mean(xn @ uh))
    th = rope_inv_freq(cfg)
    q = np.zeros(D, np.float32)
    k = np.zeros(D, np.float32)
    for i in range(N_PAIRS):  # rotate-half pair (i, i + 64)
        q[i], q[i + D // 2] = PAIR_AMP * math.cos(-COPY_OFFSET * th[i]), PAIR_AMP * math.sin(-COPY_OFFSET * th[i])
        k[i] = PAIR_AMP
    wq = np.tile(np.outer(q / c, uh), (Hq, 1))
    wk = np.tile(np.outer(k / c, uh), (Hk, 1))
    wv = np.zeros((Hk * D, H), np.float32)
    wv[np.arange(NC), np.arange(NC)] = 1.0
    wo = np.zeros((H, Hq * D), np.float32)
    grp = Hq // Hk
    for j in range(Hq):
        wo[(j // grp) * D + np.arange(D), j * D + np.arange(D)] = O_GAIN
    return {"embed": E, "wq": bf16_rne(wq), "wk": bf16_rne(wk), "wv": bf16_rne(wv), "wo": bf16_rne(wo)}


def apply(weights: dict, ov: dict) -> dict:
    """Oracle weight dict (oracle.synth.make_weights layout) with the overrides in place."""
    weights["embed"] = ov["embed"]
    weights["lm_head"] = ov["embed"]
    for name in ("wq", "wk", "wv", "wo"):
        weights["layers"][0][name] = ov[name]
    return weights


def expected_continuation(prompt, n: int) -> list:
    """The copy head's greedy continuation: token(p+1) = token(p - COPY_OFFSET)."""
    seq = [int(t) for t in prompt]
    for _ in range(n):
        seq.append(seq[len(seq) - 1 - COPY_OFFSET])
    return seq[len(prompt):]
