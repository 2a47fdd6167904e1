"""The large-batch K-quant decode GEMM (k_qdgemm.hip, ms_op_qdgemm).

A Q4_K_M engine of >= 65 slots streams every quantised matrix's packed blocks once per decode
step through this kernel instead of re-streaming them per 64-row group through the Q-GEMV.
Each weight is dequantised in registers to f16(ggml dequant) -- exactly the value the engine's
fp16 copy holds (ms_op_quant_rows) -- so the reference is that fp16 copy in float64: fp32
outputs differ from it only by summation order.  Rows are independent of the launch's other
rows (the engine's batch-invariance contract inside a regime)."""
import numpy as np
import pytest

from mapsum import _lib as L

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def lib(dev):
    return L.load()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def rel(a, b):
    return float((a - b).norm() / b.norm())


_W = {}


def _weights(dev, lib, qtype, N, K):
    """(fp16 copy [N][K], packed rows) of seeded random blocks (oracle/quants.py random_blocks)."""
    key = (qtype, N, K)
    if key not in _W:
        from oracle import quants as Q
        _W.clear()
        b = Q.random_blocks(qtype, N * K // 256, seed=N + 3 * K + qtype, scale=0.02)
        bd = torch.from_numpy(b.reshape(-1)).to(dev)
        wf = torch.empty(N, K, dtype=torch.float16, device=dev)
        pk = torch.empty(N * (K // 256) * (144 if qtype == 12 else 224), dtype=torch.uint8, device=dev)
        L.check(lib.ms_op_quant_rows(qtype, bd.data_ptr(), N, K, wf.data_ptr(), pk.data_ptr(), _stream()))
        torch.cuda.synchronize()
        want = torch.from_numpy(Q.c_dequant(b, qtype).reshape(N, K).astype(np.float16))
        assert torch.equal(wf.cpu().view(torch.int16), want.view(torch.int16))  # f16(ggml dequant)
        _W[key] = (wf, pk)
    return _W[key]


SHAPES = [(16384, 3072, 1, L.MS_EPI_SWIGLU), (3072, 8192, 8, L.MS_EPI_STORE_F32),
          (5120, 3072, 6, L.MS_EPI_STORE_F32), (4096, 3072, 1, L.MS_EPI_ARGMAX), (1024, 768, 1, L.MS_EPI_STORE_F32)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("qtype", [12, 14])
@pytest.mark.parametrize("M", [1, 17, 100, 128, 256])
@pytest.mark.parametrize("N,K,S,epi", SHAPES)
def test_qdgemm_vs_fp64(lib, dev, qtype, M, N, K, S, epi):
    wf, pk = _weights(dev, lib, qtype, N, K)
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K + S + epi)
    X = torch.randn(M, K, generator=g).to(torch.float16).to(dev)
    ref = X.double() @ wf.double().T
    if epi == L.MS_EPI_STORE_F32:
        out = torch.full((S, M, N), float("nan"), device=dev)
        L.check(lib.ms_op_qdgemm(X.data_ptr(), qtype, pk.data_ptr(), out.data_ptr(), M, N, K, S, N, epi, _stream()))
        torch.cuda.synchronize()
        ks = K // S
        for s_ in range(S):
            exp = X.double()[:, s_ * ks:(s_ + 1) * ks] @ wf.double()[:, s_ * ks:(s_ + 1) * ks].T
            assert rel(out[s_].double(), exp) < 2e-6, s_
        return
    if epi == L.MS_EPI_ARGMAX:
        part = torch.empty(M, N // 16, 2, device=dev)
        ids = torch.empty(M, dtype=torch.int32, device=dev)
        L.check(lib.ms_op_qdgemm(X.data_ptr(), qtype, pk.data_ptr(), part.data_ptr(), M, N, K, 1, N // 16, epi,
                                 _stream()))
        L.check(lib.ms_op_argmax_partials(part.data_ptr(), M, N // 16, ids.data_ptr(), _stream()))
        torch.cuda.synchronize()
        srt = torch.sort(ref, 1).values
        got = ids.cpu().long()
        for r in range(M):  # the fp64 argmax, unless the top two are within fp32 noise
            if srt[r, -1] - srt[r, -2] > 1e-4 * (1 + abs(float(srt[r, -1]))):
                assert int(got[r]) == int(torch.argmax(ref[r])), r
        return
    out = torch.zeros(M, N // 2, dtype=torch.float16, device=dev)  # SwiGLU
    r = ref.view(M, N // 32, 2, 16)
    exp, ldo, tol = (torch.nn.functional.silu(r[:, :, 0]) * r[:, :, 1]).reshape(M, N // 2), N // 2, 4e-3
    L.check(lib.ms_op_qdgemm(X.data_ptr(), qtype, pk.data_ptr(), out.data_ptr(), M, N, K, S, ldo, epi, _stream()))
    torch.cuda.synchronize()
    assert rel(out.double(), exp) < tol


@pytest.mark.timeout(300)
@pytest.mark.parametrize("qtype", [12, 14])
@pytest.mark.parametrize("N,K,S,epi", [SHAPES[0], SHAPES[1], SHAPES[3]])
def test_qdgemm_rows_independent_of_batch(lib, dev, qtype, N, K, S, epi):
    """A row's result is bitwise the same whatever the other rows of the launch (24..256 rows:
    admission ramps and tails of a large K-quant engine)."""
    wf, pk = _weights(dev, lib, qtype, N, K)
    g = torch.Generator(device="cpu").manual_seed(N + K + S + epi)
    X = torch.randn(256, K, generator=g).to(torch.float16).to(dev)
    ncol = N // 2 if epi == L.MS_EPI_SWIGLU else (N // 16 if epi == L.MS_EPI_ARGMAX else N)
    dt = torch.float16 if epi == L.MS_EPI_SWIGLU else torch.float32
    width = ncol * (2 if epi == L.MS_EPI_ARGMAX else 1)
    outs = {}
    ms = (24, 77, 128, 256)
    for M in ms:
        o = torch.zeros(S, M, width, dtype=dt, device=dev)
        L.check(lib.ms_op_qdgemm(X.data_ptr(), qtype, pk.data_ptr(), o.data_ptr(), M, N, K, S, ncol, epi, _stream()))
        torch.cuda.synchronize()
        outs[M] = o.cpu()
    for M in ms[1:]:
        assert torch.equal(outs[M][:, :24], outs[24]), M


def test_qdgemm_refuses_bad_shapes(lib, dev):
    wf, pk = _weights(dev, lib, 12, 1024, 768)
    X = torch.zeros(8, 768, dtype=torch.float16, device=dev)
    out = torch.zeros(4, 8, 1024, device=dev)
    for M, N, K, S, epi in ((257, 1024, 768, 1, L.MS_EPI_STORE_F32), (8, 1000, 768, 1, L.MS_EPI_STORE_F32),
                            (8, 1024, 768, 2, L.MS_EPI_STORE_F32), (8, 1024, 768, 3, L.MS_EPI_SWIGLU),
                            (8, 1024, 768, 3, L.MS_EPI_STORE_F32), (8, 1024, 768, 1, L.MS_EPI_STORE_F16)):
        assert lib.ms_op_qdgemm(X.data_ptr(), 12, pk.data_ptr(), out.data_ptr(), M, N, K, S, N, epi,
                                _stream()) == L.MS_EINVAL


# the fp16-rows form as fp16 engines of >= 192 slots launch it (engine.cpp qdf): QKV split 3,
# O and down split 4, gate/up SwiGLU
F16_ENGINE_SHAPES = [(5120, 3072, 3, L.MS_EPI_STORE_F32), (3072, 3072, 4, L.MS_EPI_STORE_F32),
                     (3072, 8192, 4, L.MS_EPI_STORE_F32)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("M", [1, 100, 128, 256])
@pytest.mark.parametrize("N,K,S,epi", SHAPES + F16_ENGINE_SHAPES)
def test_qdgemm_fp16_rows(lib, dev, M, N, K, S, epi):
    """The same kernel on fp16 rows (ggml type F16 = 1): fp32 outputs against float64, rows
    independent of the launch's other rows."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + S + epi)
    W = (torch.randn(N, K, generator=g) * 0.05).to(torch.float16).to(dev)
    X = torch.randn(256, K, generator=g).to(torch.float16).to(dev)
    ncol = N // 2 if epi == L.MS_EPI_SWIGLU else (N // 16 if epi == L.MS_EPI_ARGMAX else N)
    dt = torch.float16 if epi == L.MS_EPI_SWIGLU else torch.float32
    width = ncol * (2 if epi == L.MS_EPI_ARGMAX else 1)
    o = torch.zeros(S, M, width, dtype=dt, device=dev)
    L.check(lib.ms_op_qdgemm(X.data_ptr(), 1, W.data_ptr(), o.data_ptr(), M, N, K, S, ncol, epi, _stream()))
    full = torch.zeros(S, 256, width, dtype=dt, device=dev)
    L.check(lib.ms_op_qdgemm(X.data_ptr(), 1, W.data_ptr(), full.data_ptr(), 256, N, K, S, ncol, epi, _stream()))
    torch.cuda.synchronize()
    assert torch.equal(o.cpu(), full[:, :M].cpu())
    ref = X[:M].double() @ W.double().T
    if epi == L.MS_EPI_STORE_F32:
        ks = K // S
        for s_ in range(S):
            exp = X[:M].double()[:, s_ * ks:(s_ + 1) * ks] @ W.double()[:, s_ * ks:(s_ + 1) * ks].T
            assert rel(o[s_].double(), exp) < 2e-6, s_
    elif epi == L.MS_EPI_SWIGLU:
        r = ref.view(M, N // 32, 2, 16)
        exp = (torch.nn.functional.silu(r[:, :, 0]) * r[:, :, 1]).reshape(M, N // 2)
        assert rel(o[0].double(), exp) < 4e-3
