"""The benchmarked shape on the GPU against the CPU oracle (needs a GPU).

BASELINE.json configs[1] is 8 chunks x 2048 prompt tokens -> 256 greedy tokens on
Llama-3.2-3B.  Here the engine runs that exact workload with the full Llama-3.2-3B
widths (hidden 3072, 24 q / 8 kv heads, FFN 8192, vocab 128256, llama3 RoPE) and 2 of
its 28 layers -- the kernels, their shapes, grids and split choices are the benchmarked
ones; only the layer count is cut so the numpy oracle (oracle/llama_ref.py) finishes.

Tolerances (BASELINE.json north_star, written here):
  * per-layer hidden states and all-position logits: relative (norm-wise) error < 2e-2;
  * greedy tokens: teacher-forced (the oracle sees the engine's own tokens, so one
    flip does not cascade) agreement >= 99 % on every position whose oracle top-2 gap
    is decisive (> DECISIVE x the rms logit error measured on the same chunk's prefill),
    and every disagreement at a near-tie of the oracle (gap <= 1e-2 (|top| + 1)).
    Random-weight logits are flat (median top-2 gap ~0.19 at vocab 128256), so a few
    per cent of positions are ties to within the fp16 pipeline's rounding noise; the
    free-running prefix match is printed alongside.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from mapsum import _lib as L  # noqa: E402
from mapsum.config import LLAMA32_3B  # noqa: E402
from mapsum.engine import Engine  # noqa: E402
from oracle.llama_ref import OracleLlama  # noqa: E402
from oracle.synth import make_weights  # noqa: E402

CFG = LLAMA32_3B.with_(n_layers=2)
SEED, STD, JIT = 77, 0.02, 0.1  # std 0.02 = bench.py's synthetic weights
P, GEN, NCHUNK = 2048, 256, 8
DECISIVE = 4.0


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _chunks():
    # bench.py synthetic_chunks: Llama-3 header ids + uniform body over [0, 128000)
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench.synthetic_chunks(NCHUNK, P, doc=0, vocab=CFG.vocab, bos=CFG.bos_id)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def oracle(dev):
    return OracleLlama(CFG, make_weights(CFG, SEED, std=STD, jitter=JIT))


@pytest.fixture(scope="module")
def eng(dev):
    e = Engine(CFG, device=0, max_batch=NCHUNK, max_ctx=P + GEN, max_prefill_tokens=NCHUNK * P)
    e.init_synthetic(SEED, STD, JIT)
    yield e
    e.close()


@pytest.fixture(scope="module")
def chunks():
    return _chunks()


@pytest.fixture(scope="module")
def batch_out(eng, chunks):
    """The bench workload itself: 8 x 2048 -> 256 greedy tokens in one continuous batch."""
    return eng.generate(chunks, num_predict=GEN, ignore_eos=True)


@pytest.fixture(scope="module")
def prefill0(oracle, chunks):
    """Oracle prefill of chunk 0: per-layer residuals, all-position logits, the KV cache."""
    cache = oracle.new_cache()
    lg, probes = oracle.forward(chunks[0], cache, collect=True, all_logits=True)
    return lg, probes, cache


@pytest.mark.timeout(900)
def test_fullshape_synthetic_weights_bit_exact(eng, oracle, chunks):
    """Device generator == oracle/synth.py at the full vocab: embedding rows gathered by
    the layer-0 probe come back bit for bit."""
    ids = np.concatenate([chunks[0][:512], np.arange(128000, 128256, dtype=np.int32)])
    h0, _ = eng.forward(ids, n_layers=0)
    assert np.array_equal(h0, oracle.w["embed"][ids])


@pytest.mark.timeout(900)
def test_fullshape_per_layer_hidden_and_logits(eng, prefill0, chunks):
    ref_lg, probes, _ = prefill0
    for l in range(CFG.n_layers):
        h, _ = eng.forward(chunks[0], n_layers=l + 1)
        e = rel(h, probes[l])
        print(f"layer {l}: hidden rel err {e:.3e}")
        assert e < 2e-2, f"layer {l}"
    _, lg = eng.forward(chunks[0], hidden=False, logits=True)
    err = rel(lg, ref_lg)
    a, b = np.argmax(lg, 1), np.argmax(ref_lg, 1)
    srt = np.sort(ref_lg, 1)
    gap = srt[:, -1] - srt[:, -2]
    noise = float(np.sqrt(np.mean((lg - ref_lg) ** 2)))
    flips = np.nonzero(a != b)[0]
    print(f"logits rel err {err:.3e}, rms abs err {noise:.3e}, argmax agreement {np.mean(a == b):.4f}, "
          f"{len(flips)} flips, max flip gap {gap[flips].max() if len(flips) else 0:.4f}")
    assert err < 2e-2
    assert np.all(gap[flips] <= 1e-2 * (np.abs(srt[flips, -1]) + 1.0))
    dec = gap > DECISIVE * noise
    assert np.mean(a[dec] == b[dec]) >= 0.99


def _teacher_forced(oracle, cache, first_logits, gen):
    """Oracle logits for every generated position, fed the engine's own tokens one at a
    time through the decode path (KV cache), as the engine produced them."""
    out = [first_logits]
    for t in gen[:-1]:
        lg, _ = oracle.forward([int(t)], cache)
        out.append(lg)
    return np.stack(out)


def _free_running_prefix(oracle, prompt, gen, n):
    ref, _ = oracle.generate(prompt, n, ignore_eos=True)
    k = 0
    while k < n and ref[k] == gen[k]:
        k += 1
    return k


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("ci,n", [(0, 256), (5, 128)])
def test_fullshape_batched_greedy_vs_oracle(eng, oracle, prefill0, chunks, batch_out, ci, n):
    """configs[1] through the engine (the 8 chunks in one batch); chunk ci's first n greedy
    tokens against the oracle, teacher-forced, plus the free-running prefix."""
    r = batch_out[ci]
    assert len(r.ids) == GEN and r.finish == "length"
    gen = np.asarray(r.ids[:n])
    if ci == 0:
        ref_lg, _, cache0 = prefill0
        first = ref_lg[-1]
        cache = {"k": list(cache0["k"]), "v": list(cache0["v"]), "len": cache0["len"]}
    else:
        cache = oracle.new_cache()
        first, _ = oracle.forward(chunks[ci], cache)
    lg = _teacher_forced(oracle, cache, first, gen)
    want = np.argmax(lg, 1)
    srt = np.sort(lg, 1)
    gap = srt[:, -1] - lg[np.arange(n), gen]
    top2 = srt[:, -1] - srt[:, -2]
    flips = np.nonzero(want != gen)[0]
    # rms logit noise of this pipeline, measured where both sides saw the same inputs
    _, elg = eng.forward(chunks[0][:512], hidden=False, logits=True)
    olg, _ = oracle.forward(chunks[0][:512], all_logits=True)
    noise = float(np.sqrt(np.mean((elg - olg) ** 2)))
    dec = top2 > DECISIVE * noise
    prefix = _free_running_prefix(oracle, chunks[ci], gen, min(n, 128))
    print(f"chunk {ci}: teacher-forced agreement {np.mean(want == gen):.4f} over {n}; decisive "
          f"positions {dec.sum()} agree {np.mean(want[dec] == gen[dec]):.4f}; flips at {flips.tolist()} "
          f"gaps {np.round(gap[flips], 4).tolist()}; free-running prefix {prefix}/{min(n, 128)}")
    for i in flips:
        assert gap[i] <= 1e-2 * (abs(srt[i, -1]) + 1.0), (i, gap[i], srt[i, -1])
    assert np.mean(want[dec] == gen[dec]) >= 0.99


@pytest.mark.timeout(600)
def test_fullshape_batch_invariance(eng, chunks, batch_out):
    """A chunk's summary does not depend on its batch companions at the bench shape."""
    for ci in (3, 7):
        alone = eng.generate([chunks[ci]], num_predict=GEN, ignore_eos=True)[0]
        assert alone.ids == batch_out[ci].ids, ci


@pytest.mark.timeout(900)
def test_fullshape_decode_b32(oracle, chunks):
    """B = 32 at the full width (MT = 2 GEMV tiles; the gate/up X image no longer fits LDS
    and is read from L2): tokens agree with the oracle (teacher-forced, near-tie rule)."""
    e = Engine(CFG, device=0, max_batch=32, max_ctx=256, max_prefill_tokens=4096)
    try:
        e.init_synthetic(SEED, STD, JIT)
        prompts = [chunks[i % NCHUNK][64 * (i // NCHUNK):64 * (i // NCHUNK) + 40 + i] for i in range(32)]
        res = e.generate(prompts, num_predict=8, ignore_eos=True)
        for i in (0, 13, 31):
            p, gen = prompts[i], np.asarray(res[i].ids)
            cache = oracle.new_cache()
            first, _ = oracle.forward(p, cache)
            lg = _teacher_forced(oracle, cache, first, gen)
            srt = np.sort(lg, 1)
            for j in np.nonzero(np.argmax(lg, 1) != gen)[0]:
                assert srt[j, -1] - lg[j, gen[j]] <= 1e-2 * (abs(srt[j, -1]) + 1.0), (i, j)
    finally:
        e.close()


# ------------------------------------------------------------------ ops at the bench shapes
def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.timeout(600)
@pytest.mark.parametrize("N,K,epi", [(5120, 3072, L.MS_EPI_STORE_F16), (3072, 3072, L.MS_EPI_ADD_F32),
                                     (16384, 3072, L.MS_EPI_SWIGLU), (3072, 8192, L.MS_EPI_ADD_F32),
                                     (16384, 3072, L.MS_EPI_STORE_F32)])
def test_prefill_gemm_bench_shapes(dev, N, K, epi):
    """gemm256 at M = 8 x 2048 packed prompt rows and the Llama-3.2-3B projection shapes
    (QKV / O / gate-up / down), against a float64 GPU reference (torch)."""
    lib = L.load()
    M = NCHUNK * P
    g = torch.Generator(device="cuda").manual_seed(N + K + epi)
    A = torch.randn(M, K, device=dev, generator=g).to(torch.float16)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.float16)
    ref = A.double() @ W.double().T
    if epi == L.MS_EPI_SWIGLU:
        out = torch.zeros(M, N // 2, dtype=torch.float16, device=dev)
        r = ref.view(M, N // 32, 2, 16)
        exp, ldo, tol = (torch.nn.functional.silu(r[:, :, 0]) * r[:, :, 1]).reshape(M, N // 2), N // 2, 4e-3
    elif epi == L.MS_EPI_STORE_F16:
        out = torch.zeros(M, N, dtype=torch.float16, device=dev)
        exp, ldo, tol = ref, N, 4e-3
    elif epi == L.MS_EPI_ADD_F32:
        out = torch.randn(M, N, device=dev, generator=g)
        exp, ldo, tol = out.double() + ref, N, 2e-6
    else:
        out = torch.zeros(M, N, dtype=torch.float32, device=dev)
        exp, ldo, tol = ref, N, 2e-6
    L.check(lib.ms_op_gemm(A.data_ptr(), W.data_ptr(), out.data_ptr(), M, N, K, ldo, epi, _stream()))
    torch.cuda.synchronize()
    e = float((out.double() - exp).norm() / exp.norm())
    assert e < tol, e


@pytest.mark.timeout(300)
@pytest.mark.parametrize("M", [1, 8, 64])
def test_lm_head_gemv_full_vocab(dev, M):
    """The decode lm_head: [M][3072] x [128256][3072]^T fp32 logits + greedy argmax."""
    lib = L.load()
    K, N = 3072, 128256
    g = torch.Generator(device="cuda").manual_seed(M)
    X = torch.randn(M, K, device=dev, generator=g).to(torch.float16)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.float16)
    out = torch.zeros(M, N, dtype=torch.float32, device=dev)
    ws = torch.zeros(lib.ms_op_gemv_workspace(M, N, K), dtype=torch.uint8, device=dev)
    L.check(lib.ms_op_gemv(X.data_ptr(), W.data_ptr(), out.data_ptr(), M, N, K, N, L.MS_EPI_STORE_F32,
                           ws.data_ptr(), _stream()))
    ids = torch.empty(M, dtype=torch.int32, device=dev)
    L.check(lib.ms_op_argmax(out.data_ptr(), M, N, ids.data_ptr(), _stream()))
    torch.cuda.synchronize()
    ref = X.double() @ W.double().T
    assert float((out.double() - ref).norm() / ref.norm()) < 2e-6
    assert torch.equal(ids.long(), torch.argmax(out, 1))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("qtype", [12, 14])
@pytest.mark.parametrize("N,K,epi", [(3072, 8192, L.MS_EPI_ADD_F32), (16384, 3072, L.MS_EPI_SWIGLU),
                                     (5120, 3072, L.MS_EPI_STORE_F32)])
def test_qgemv_bench_shapes(dev, qtype, N, K, epi):
    """configs[4]: the dequant-fused decode GEMV at the down (3072 x 8192), gate/up
    (16384 x 3072) and QKV (5120 x 3072) shapes, B = 8, against float64."""
    from oracle import quants as Q
    lib = L.load()
    M = 8
    qt = qtype
    b = Q.random_blocks(qtype, N * K // 256, seed=N + K, scale=0.02)
    bd = torch.from_numpy(b.reshape(-1)).to(dev)
    wbf = torch.empty(N, K, dtype=torch.float16, device=dev)
    pk = torch.empty(N * (K // 256) * (144 if qtype == 12 else 224), dtype=torch.uint8, device=dev)
    L.check(lib.ms_op_quant_rows(qtype, bd.data_ptr(), N, K, wbf.data_ptr(), pk.data_ptr(), _stream()))
    g = torch.Generator(device="cuda").manual_seed(K)
    X = torch.randn(M, K, device=dev, generator=g).to(torch.float16)
    # Q4_K: the decode GEMV computes with the exact fp32 dequant; Q6_K: with the fp16 copy
    wd = torch.from_numpy(Q.c_dequant(b, qt).reshape(N, K)).to(dev).double() if qt == 12 else wbf.double()
    ref = X.double() @ wd.T
    if epi == L.MS_EPI_SWIGLU:
        out = torch.zeros(M, N // 2, dtype=torch.float16, device=dev)
        r = ref.view(M, N // 32, 2, 16)
        exp, ldo, tol = (torch.nn.functional.silu(r[:, :, 0]) * r[:, :, 1]).reshape(M, N // 2), N // 2, 4e-3
    elif epi == L.MS_EPI_ADD_F32:
        out = torch.randn(M, N, device=dev, generator=g)
        exp, ldo, tol = out.double() + ref, N, 1e-5 if qt == 12 else 2e-6
    else:  # Q4_K codes enter the fp16 MFMA as subnormals: ~3e-6 (test_gpu_parity._qtol)
        out = torch.zeros(M, N, dtype=torch.float32, device=dev)
        exp, ldo, tol = ref, N, 1e-5 if qt == 12 else 2e-6
    L.check(lib.ms_op_qgemv(X.data_ptr(), qtype, pk.data_ptr(), out.data_ptr(), M, N, K, ldo, epi, _stream()))
    torch.cuda.synchronize()
    assert float((out.double() - exp).norm() / exp.norm()) < tol


@pytest.fixture(scope="module")
def q4km(dev):
    """configs[4] weights at the full widths (2 layers): random Q4_K/Q6_K blocks in the Q4_K_M
    mix, and the oracle on their fp16-rounded dequantisation."""
    from oracle import quants as Q
    from oracle.synth import f16_rne
    H, D, F, V = CFG.hidden, CFG.head_dim, CFG.ffn, CFG.vocab
    shapes = {"wq": (CFG.n_heads * D, H), "wk": (CFG.n_kv_heads * D, H), "wv": (CFG.n_kv_heads * D, H),
              "wo": (H, CFG.n_heads * D), "w_gate": (F, H), "w_up": (F, H), "w_down": (H, F)}
    from oracle.synth import ATTN_NORM, FFN_NORM, FINAL_NORM, norm
    qw, w = {}, {"final_norm": norm(SEED, FINAL_NORM, 0, H, JIT), "layers": []}
    qt = Q.q4_k_m_type("embed", 0, CFG.n_layers)
    eb = Q.random_blocks(qt, V * H // 256, seed=5, scale=STD)
    qw["embed"] = (qt, eb)
    w["embed"] = f16_rne(Q.dequant(eb, qt)).reshape(V, H)
    w["lm_head"] = w["embed"]
    for l in range(CFG.n_layers):
        ly = {"attn_norm": norm(SEED, ATTN_NORM, l, H, JIT), "ffn_norm": norm(SEED, FFN_NORM, l, H, JIT)}
        for i, (name, (r, c)) in enumerate(shapes.items()):
            qt = Q.q4_k_m_type(name, l, CFG.n_layers)
            blk = Q.random_blocks(qt, r * c // 256, seed=100 + l * 10 + i, scale=STD)
            qw[(l, name)] = (qt, blk)
            ly[name] = f16_rne(Q.dequant(blk, qt)).reshape(r, c)
        w["layers"].append(ly)
    return qw, w, OracleLlama(CFG, w)


_Q4_GEN = {}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("slots", [2, 16, 32, 128])
def test_fullshape_q4_k_m_engine_vs_oracle(q4km, slots):
    """configs[4] at the full widths (2 layers): Q4_K_M blocks through ms_load_weight_q;
    prefill logits and 64 teacher-forced greedy tokens against the oracle run on the
    dequantised weights.  Every engine size decodes with the dequant-fused K-quant GEMVs
    (exact Q4_K arithmetic): 2 and 16 slots in one row group with the residual epilogue on O /
    down (engines of <= 16 slots, as fp16), 32 and 128 slots (the large-batch regime of fp16
    engines) in row groups of <= 64 with split-K O / down -- with 96 chunks in flight at 128
    slots the batch really spans two groups.  Within a regime the chunk's tokens do not depend
    on the engine size."""
    from mapsum.weights import load_quantized
    qw, w, o = q4km
    prompt = _chunks()[2][:768]
    e = Engine(CFG, device=0, max_batch=slots, max_ctx=1024, max_prefill_tokens=2048 if slots < 128 else 8192)
    try:
        load_quantized(e, qw, w)
        _, lg = e.forward(prompt, hidden=False, logits=True)
        cache = o.new_cache()
        ref_lg, _ = o.forward(prompt, cache, all_logits=True)
        err = rel(lg, ref_lg)
        noise = float(np.sqrt(np.mean((lg - ref_lg) ** 2)))
        assert err < 2e-2, err
        if slots == 128:  # the chunk among 95 others (two row groups of the decode GEMVs)
            others = [c[:256] for c in _chunks()[3:8]] * 19
            res = e.generate([prompt] + others, num_predict=64, ignore_eos=True)
            gen = np.asarray(res[0].ids)
        else:
            gen = np.asarray(e.generate([prompt], num_predict=64, ignore_eos=True)[0].ids)
        _Q4_GEN[slots] = gen
        if 2 in _Q4_GEN and slots == 16:
            # engine-size invariance: the K-quant GEMV arithmetic is per row, and 2- and 16-slot
            # engines share the residual-epilogue regime and the decode-attention plan (2 pages
            # per wave); 32 slots sum O / down over split-K slabs, and a 128-slot engine splits
            # attention at 8 pages per wave (attn_decode_ppw) -- different fp32 sum orders, so
            # there only the oracle check below applies
            assert np.array_equal(gen, _Q4_GEN[2]), (slots, np.nonzero(gen != _Q4_GEN[2])[0][:5])
        tl = _teacher_forced(o, cache, ref_lg[-1], gen)
        want = np.argmax(tl, 1)
        srt = np.sort(tl, 1)
        top2 = srt[:, -1] - srt[:, -2]
        dec = top2 > DECISIVE * noise
        print(f"q4_k_m ({slots} slots): logits rel err {err:.3e}; teacher-forced {np.mean(want == gen):.4f}, "
              f"decisive {dec.sum()} agree {np.mean(want[dec] == gen[dec]):.4f}")
        for i in np.nonzero(want != gen)[0]:
            assert srt[i, -1] - tl[i, gen[i]] <= 1e-2 * (abs(srt[i, -1]) + 1.0)
        assert np.mean(want[dec] == gen[dec]) >= 0.99
    finally:
        e.close()


# ------------------------------------------------- configs[2] and configs[3] at full width
def _tf_check(oracle, prompt, gen, tag, eng=None):
    """Teacher-forced oracle logits after the engine's own tokens; every disagreement must be
    an oracle near-tie.  Returns (agreement fraction, agreement on the decisive positions --
    oracle top-2 gap > DECISIVE x the rms logit error of the engine's prefill at the prompt's
    last position -- and their count); without an engine every position counts as decisive."""
    cache = oracle.new_cache()
    first, _ = oracle.forward(prompt, cache)
    noise = 0.0
    if eng is not None:
        _, elg = eng.forward(prompt, hidden=False, logits=True)
        noise = float(np.sqrt(np.mean((elg[-1].astype(np.float64) - first) ** 2)))
        del elg
    lg = _teacher_forced(oracle, cache, first, gen)
    want = np.argmax(lg, 1)
    srt = np.sort(lg, 1)
    for j in np.nonzero(want != gen)[0]:
        assert srt[j, -1] - lg[j, gen[j]] <= 1e-2 * (abs(srt[j, -1]) + 1.0), (tag, j)
    dec = srt[:, -1] - srt[:, -2] > DECISIVE * noise
    return float(np.mean(want == gen)), float(np.mean(want[dec] == gen[dec])) if dec.any() else 1.0, int(dec.sum())


@pytest.mark.timeout(1200)
def test_config2_continuous_batching_full_width(oracle):
    """BASELINE configs[2] per GPU at full width (2 layers): max_batch 128 slots over 2304-token
    contexts, 160 chunks of 2048 tokens (more chunks than slots: admission as slots free),
    32 greedy tokens each.  The B=128 decode plan (skinny GEMM regime, per-engine attention
    pages-per-wave) against the oracle for three chunks, and batch invariance against solo
    runs (runners/run_summarization_ollama_mapreduce.py:109-112 hands the engine every chunk)."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    chunks = [c for d in range(20) for c in bench.synthetic_chunks(8, P, doc=d, vocab=CFG.vocab, bos=CFG.bos_id)]
    e = Engine(CFG, device=0, max_batch=128, max_ctx=P + 256, max_prefill_tokens=8 * P)
    try:
        e.init_synthetic(SEED, STD, JIT)
        res = e.generate(chunks, num_predict=32, ignore_eos=True)
        assert all(len(r.ids) == 32 and r.finish == "length" for r in res)
        for i in (0, 77, 159):
            agree, dagree, ndec = _tf_check(oracle, chunks[i], np.asarray(res[i].ids), i, eng=e)
            print(f"configs[2] chunk {i}: teacher-forced agreement {agree:.4f}, decisive {ndec} agree {dagree:.4f}")
            assert dagree >= 0.99, (i, dagree, ndec)
        for i in (5, 130):
            alone = e.generate([chunks[i]], num_predict=32, ignore_eos=True)[0]
            assert alone.ids == res[i].ids, i
    finally:
        e.close()


@pytest.mark.parametrize("slots", [NCHUNK, 32])
def test_decode_tail_bit_exact(dev, chunks, monkeypatch, slots):
    """The one-launch decode step tail (k_misc.hip decode_tail_kernel: the lm_head partials'
    argmax, the chained-step advance with its last-arrival step ticket, the next step's
    embedding and first-norm statistics) against the three launches it replaces: identical
    greedy ids over chained runs, on the GEMV lm_head (8 slots) and the skinny-GEMM one
    (32 slots, >= 24: the large regime)."""
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("MS_DECODE_TAIL", fused)
        e = Engine(CFG, device=0, max_batch=slots, max_ctx=P + 64, max_prefill_tokens=NCHUNK * P)
        try:
            e.init_synthetic(SEED, STD, JIT)
            res = e.generate(list(chunks), num_predict=40, ignore_eos=True)
            outs.append([r.ids for r in res])
        finally:
            e.close()
    assert outs[0] == outs[1]


def test_decode_attention_tuning_bit_exact(dev, chunks):
    """Decode attention's tuning knob is placement only (ms_set_attn_tuning): the split combine on
    the XCD-matched 1-D grid (default) or the (B, Hq) grid -- identical greedy ids over chained
    runs of the per-layer launches (the persistent step, which has its own merge, is off)."""
    lib = L.load()
    outs = {}
    try:
        for grp, order in ((1, 0), (0, 0)):
            L.check(lib.ms_set_attn_tuning(grp, order))
            e = Engine(CFG, device=0, max_batch=NCHUNK, max_ctx=P + 64, max_prefill_tokens=NCHUNK * P)
            try:
                e.set_persist(False)
                e.init_synthetic(SEED, STD, JIT)
                res = e.generate(list(chunks), num_predict=40, ignore_eos=True)
                outs[(grp, order)] = [r.ids for r in res]
            finally:
                e.close()
    finally:
        L.check(lib.ms_set_attn_tuning(1, 0))
    assert outs[(0, 0)] == outs[(1, 0)]


def test_prefill_packing_invariance(dev):
    """A prompt's prefill does not depend on what it is packed with: alone (600 rows: the
    128x128 GEMM tile) and behind a 1500-token prompt (2100 rows: the 256x256 tile) its hidden
    states after every layer are bitwise equal, and so are its greedy tokens -- the prefill
    residual epilogue writes its norm statistics per 128 columns on both tiles (round 4 first
    wrote them per column tile, and configs[3]'s ragged batch-invariance check caught it)."""
    rng = np.random.default_rng(12)
    a = rng.integers(0, 128000, size=600).astype(np.int32)
    b = rng.integers(0, 128000, size=1500).astype(np.int32)
    e = Engine(CFG, device=0, max_batch=2, max_ctx=2048, max_prefill_tokens=4096)
    try:
        e.init_synthetic(SEED, STD, JIT)
        for nl in range(1, CFG.n_layers + 1):
            h1, _ = e.forward_packed([a], n_layers=nl)
            h2, _ = e.forward_packed([b, a], n_layers=nl)
            assert np.array_equal(h1, h2[len(b):]), nl
        alone = e.generate([a], num_predict=16, ignore_eos=True)[0].ids
        both = e.generate([b, a], num_predict=16, ignore_eos=True)[1].ids
        assert alone == both
    finally:
        e.close()


@pytest.mark.timeout(1200)
def test_config3_ragged_sections_full_width(oracle):
    """BASELINE configs[3] at full width (2 layers): ragged hierarchical sections of 64, 611,
    1500 and 4096 tokens packed into ONE varlen prefill pass (max_ctx 4352): per-layer hidden
    states of every section against the oracle, then 64 greedy tokens per section in one
    continuous batch, teacher-forced against the oracle
    (runners/run_summarization_ollama_mapreduce_hierarchical.py:242-274)."""
    rng = np.random.default_rng(11)
    lens = (64, 611, 1500, 4096)
    secs = [rng.integers(0, 128000, size=n).astype(np.int32) for n in lens]
    e = Engine(CFG, device=0, max_batch=4, max_ctx=4352, max_prefill_tokens=8192)
    try:
        e.init_synthetic(SEED, STD, JIT)
        offs = np.cumsum((0,) + lens)
        probes = [oracle.forward(s, collect=True)[1] for s in secs]
        for l in range(CFG.n_layers):
            h, _ = e.forward_packed(secs, n_layers=l + 1)
            for i, s in enumerate(secs):
                err = rel(h[offs[i]:offs[i + 1]], probes[i][l])
                print(f"configs[3] layer {l} section {len(s)}: hidden rel err {err:.3e}")
                assert err < 2e-2, (l, len(s))
        del probes
        res = e.generate(secs, num_predict=64, ignore_eos=True)
        for s, r in zip(secs, res):
            assert len(r.ids) == 64
            agree, dagree, ndec = _tf_check(oracle, s, np.asarray(r.ids), len(s), eng=e)
            print(f"configs[3] section {len(s)}: teacher-forced agreement {agree:.4f}, decisive {ndec} "
                  f"agree {dagree:.4f}")
            assert dagree >= 0.99, (len(s), dagree, ndec)
    finally:
        e.close()
