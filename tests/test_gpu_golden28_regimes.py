"""All 28 layers in the decode regimes the product actually runs (needs a GPU).

tests/test_gpu_golden28.py checks the benchmarked 8-slot engine.  An engine's decode
arithmetic is fixed at ms_create from max_batch (include/mapsum.h):
   1-16 slots  GEMV, O / down with the residual + statistics epilogue (the 8-slot bench);
  17-23 slots  GEMV, split-K O / down + residual_rmsnorm                  -> 20 slots here;
   >=24 slots  skinny GEMM (k_dgemm.hip), 8 KV pages per attention wave  -> 64 slots (the
               drop-in default, compat.py MAPSUM_MAX_BATCH) and 128 slots (configs[2]);
   >=96 slots  the same, with the lm_head's greedy partials on the prefill GEMM's 128x128
               tile                                                       -> 128 and 256 slots
               (256: 16-row-tile skinny GEMMs, the configs[2] record's width);
and K-quant engines (configs[4], Q4_K_M) keep the exact Q-GEMV at every size: <= 16 slots
with the residual epilogue, above that in row groups of <= 64 rows with split-K O / down
-> 8 and 128 slots here.  The reference hands the engine every chunk at once
(runners/run_summarization_ollama_mapreduce.py:109-112), so large engines are the normal
case of the replaced call (run_full_evaluation_pipeline.py:80-106).

Every regime is held to the same bars as the 8-slot engine, against UN-ROUNDED fp32 Llama
(tests/golden/fullshape_{flat,sharp}_fp32.npz; for Q4_K_M fullshape_q4km_fp32.npz, the
oracle on the EXACT fp32 dequantisation of bench.py's Q4_K_M weights, ms_init_synthetic_q
seed 2, whose block generator oracle/synth.py restates bit for bit):
  * per-layer hidden states (kept rows, sketch, norms) and prefill logits within 2e-2;
  * teacher forcing through the decode path (ms_submit_forced), both chunks of the model in
    one batch: every flip an oracle near-tie, >= 99 % of the decisive positions equal; the
    sharp model equal at every position;
  * free running inside a FULL engine (max(8, slots) chunks of bench.py's workload in one
    continuous batch): sharp >= 99 % of the first 128 tokens; flat / Q4_K_M: the first
    difference is an oracle near-tie.
"""
import importlib.util
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_gpu_golden28 import (CFG, DECISIVE, GOLD, TOL, _engine, _near_tie, load_fixture,  # noqa: E402
                               rel, sketch_mats)

from mapsum import _lib as L  # noqa: E402
from mapsum.engine import Engine  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
# sharpq4km: the copy head on the Q4_K_M weights, quantised into K-quant
# blocks (tests/golden/sharp_model.py q4km_overrides) -- the decisive greedy bar on K-quant weights
RUNS = [(s, w) for s in (20, 64, 128) for w in ("flat", "sharp")] + [(256, "flat"), (256, "sharp")] + \
    [(8, "q4km"), (128, "q4km")] + [(8, "sharpq4km"), (128, "sharpq4km")]
CASES = [(s, w, ci) for s, w in RUNS for ci in ((0, 3) if w in ("sharp", "sharpq4km") else (0, 5))]
_CACHE = {}
_OVERRIDES = {}


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(HERE), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def _q4km_engine(meta, slots, sharp=False):
    e = Engine(CFG, device=0, max_batch=slots, max_ctx=meta["prompt_len"] + 256,
               max_prefill_tokens=8 * meta["prompt_len"])
    e.init_synthetic_q(seed=meta["seed"], scale=meta["std"], norm_jitter=meta["jitter"])
    if sharp:
        # the copy head's quantised blocks over the synthetic Q4_K_M model (the fixture's oracle ran
        # the exact dequantisation of these same bytes)
        import sys
        sys.path.insert(0, os.path.join(HERE, "golden"))
        import sharp_model
        assert meta["copy_layer"] == sharp_model.COPY_LAYER and meta["c_layer"] == sharp_model.C_LAYER_Q4KM
        if "ov" not in _OVERRIDES:  # ~30 s of numpy quantisation, shared by the 8- and 128-slot engines
            _OVERRIDES["ov"] = sharp_model.q4km_overrides(CFG)
        ov = _OVERRIDES["ov"]
        qt, blocks = ov["embed"]
        e.load_tensor_q(L.MS_T_EMBED, 0, qt, blocks.reshape(-1))
        for name, t in (("wq", L.MS_T_WQ), ("wk", L.MS_T_WK), ("wv", L.MS_T_WV), ("wo", L.MS_T_WO)):
            qt, blocks = ov[(sharp_model.COPY_LAYER, name)]
            e.load_tensor_q(t, sharp_model.COPY_LAYER, qt, blocks.reshape(-1))
    return e


def _run(slots, which):
    """Everything the assertions need from one engine, then the engine is closed (one engine
    of <= 6.4 GB + 34 GB of KV at a time)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    meta, d = load_fixture(which, "fp32")
    eng = (_q4km_engine(meta, slots, sharp=which == "sharpq4km") if which in ("q4km", "sharpq4km")
           else _engine(meta, which, max_batch=slots))
    R, Rv = sketch_mats()
    out = {"layers": {}, "logits": {}, "forced": {}, "free": {}}
    try:
        for ci in meta["chunks"]:
            k = f"c{ci}_"
            prompt, hp = d[k + "prompt"], d[k + "hpos"]
            errs = []
            for l in range(CFG.n_layers):
                h, _ = eng.forward(prompt, n_layers=l + 1)
                errs.append((rel(h[hp], d[k + "hid_rows"][l]), rel(h[::4] @ R, d[k + "hid_sketch"][l].astype(np.float32)),
                             float(np.max(np.abs(np.linalg.norm(h, axis=1) / d[k + "hid_norm"][l] - 1.0)))))
            out["layers"][ci] = errs
            _, lg = eng.forward(prompt, hidden=False, logits=True)
            lgp = lg[d[k + "lpos"]]
            del lg
            err = rel(lgp @ Rv, d[k + "lg_sketch"])
            e16 = rel(np.take_along_axis(lgp, d[k + "lg_top_ids"].astype(np.int64), 1), d[k + "lg_top_vals"])
            out["logits"][ci] = (err, e16, err * float(np.mean(d[k + "lg_rms"])), np.argmax(lgp, 1))
        # teacher forcing: both chunks of the model in one batch
        cis = list(meta["chunks"])
        refs = [d[f"c{ci}_gen_ids"] for ci in cis]
        got = eng.generate_forced([d[f"c{ci}_prompt"] for ci in cis], [r[:-1] for r in refs], len(refs[0]))
        for ci, r in zip(cis, got):
            out["forced"][ci] = np.asarray(r.ids)
        # free running inside a full engine: bench.py's chunks of docs 0, 1, ..
        bench = _bench()
        n = max(8, slots)
        chunks = [c for doc in range((n + 7) // 8)
                  for c in bench.synthetic_chunks(8, meta["prompt_len"], doc=doc, vocab=CFG.vocab, bos=CFG.bos_id)]
        for ci in cis:
            assert np.array_equal(chunks[ci], d[f"c{ci}_prompt"]), "fixture prompt != bench.py chunk"
        res = eng.generate(chunks[:n], num_predict=meta["gen"], ignore_eos=True)
        for ci in cis:
            out["free"][ci] = np.asarray(res[ci].ids)
    finally:
        eng.close()
    return meta, d, out


def _get(slots, which):
    key = (slots, which)
    if key not in _CACHE:
        for k in [k for k in _CACHE if k != key]:  # keep one run's arrays at a time
            _CACHE.pop(k)
        _CACHE[key] = _run(slots, which)
    return _CACHE[key]


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("slots,which,ci", CASES)
def test_regime_per_layer_hidden(slots, which, ci):
    _, _, out = _get(slots, which)
    worst = 0.0
    for l, (er, es, en) in enumerate(out["layers"][ci]):
        worst = max(worst, er, es)
        assert er < TOL and es < TOL and en < TOL, (slots, which, ci, l, er, es, en)
    print(f"{slots} slots {which} c{ci} vs fp32: worst per-layer relative error {worst:.3e} (tolerance {TOL})")


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("slots,which,ci", CASES)
def test_regime_prefill_logits(slots, which, ci):
    _, d, out = _get(slots, which)
    k = f"c{ci}_"
    err, e16, noise, a = out["logits"][ci]
    ti, tv = d[k + "lg_top_ids"], d[k + "lg_top_vals"]
    dec = tv[:, 0] - tv[:, 1] > DECISIVE * noise
    print(f"{slots} slots {which} c{ci} vs fp32: logits sketch rel err {err:.3e}, top-16 rel err {e16:.3e}, "
          f"argmax agreement {np.mean(a == ti[:, 0]):.4f}, decisive {dec.sum()}/{len(dec)}")
    assert err < TOL and e16 < TOL
    assert np.all(a[dec] == ti[dec, 0])
    for i in np.nonzero(a != ti[:, 0])[0]:
        assert _near_tie(ti[i], tv[i], a[i]), (i, a[i], ti[i, :3])


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("slots,which,ci", CASES)
def test_regime_teacher_forced_decode(slots, which, ci):
    _, d, out = _get(slots, which)
    k = f"c{ci}_"
    ref, got = d[k + "gen_ids"], out["forced"][ci]
    assert len(got) == len(ref)
    ti, tv = d[k + "gen_top_ids"], d[k + "gen_top_vals"]
    dec = tv[:, 0] - tv[:, 1] > DECISIVE * out["logits"][ci][2]
    flips = np.nonzero(got != ref)[0]
    print(f"{slots} slots {which} c{ci} vs fp32: teacher-forced decode agreement {np.mean(got == ref):.4f}; "
          f"decisive {dec.sum()} agree {np.mean(got[dec] == ref[dec]):.4f}; flips {flips.tolist()}")
    for i in flips:
        assert _near_tie(ti[i], tv[i], got[i]), (i, got[i], ti[i, :3], tv[i, :3])
    assert np.mean(got[dec] == ref[dec]) >= 0.99
    if which in ("sharp", "sharpq4km"):
        assert np.array_equal(got, ref)


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("slots,which,ci", CASES)
def test_regime_free_running_greedy(slots, which, ci):
    _, d, out = _get(slots, which)
    k = f"c{ci}_"
    ref = d[k + "gen_ids"]
    got = out["free"][ci][:len(ref)]
    n = min(128, len(ref))
    match = float(np.mean(got[:n] == ref[:n]))
    pre = int(np.argmin(np.append(got[:n] == ref[:n], False)))
    print(f"{slots} slots {which} c{ci} vs fp32: free-running greedy {match:.4f} of the first {n} equal, "
          f"common prefix {pre}")
    if which in ("sharp", "sharpq4km"):
        assert match >= 0.99  # BASELINE.json north_star, literally (fp16 and Q4_K_M weights)
    elif pre < n:
        assert _near_tie(d[k + "gen_top_ids"][pre], d[k + "gen_top_vals"][pre], got[pre]), \
            (pre, got[pre], d[k + "gen_top_ids"][pre, :3], d[k + "gen_top_vals"][pre, :3])


@pytest.mark.timeout(600)
def test_q4km_device_weights_are_the_fixture_weights():
    """The engine's own Q4_K_M blocks (ms_init_synthetic_q, on the device) are the blocks the
    fixture's oracle dequantised (oracle/synth.py synth_qblocks): the fp16 copies of the tied
    embedding (Q6_K), layer 0's O (Q4_K) and down (Q6_K) and layer 5's down (Q4_K) equal the
    fp16 rounding of the host dequantisation, bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mapsum.dist import region_views
    from oracle.quants import c_dequant, q4_k_m_type
    from oracle.synth import EMBED, WDOWN, WO, synth_qblocks
    meta, _ = load_fixture("q4km", "fp32")
    H, F, QD = CFG.hidden, CFG.ffn, CFG.n_heads * CFG.head_dim
    eng = _q4km_engine(meta, 8)
    try:
        views = region_views(eng)
        checks = [(0, "embed", EMBED, 0, CFG.vocab * H), (2 + 3, "wo", WO, 0, H * QD),
                  (2 + 5, "w_down", WDOWN, 0, H * F), (2 + 6 * 5 + 5, "w_down", WDOWN, 5, H * F)]
        for idx, name, kind, layer, n in checks:
            qt = q4_k_m_type(name, layer, CFG.n_layers)
            blocks = synth_qblocks(qt, n // 256, meta["seed"], kind, layer, meta["std"])
            want = c_dequant(blocks, qt).astype(np.float16).view(np.uint16)
            got = views[idx].cpu().numpy().view(np.uint16)
            assert got.size == want.size, (name, layer, got.size, want.size)
            bad = int(np.count_nonzero(got != want))
            print(f"{name} layer {layer} (ggml type {qt}): {bad} of {n} fp16 weights differ")
            assert bad == 0
    finally:
        eng.close()
