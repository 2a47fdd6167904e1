"""The large-regime decode lm_head on the prefill GEMM's 128x128 tile (k_gemm.hip gemm_kernel,
epilogue MS_EPI_ARGMAX through ms_op_gemm): {max, id} partials per 16-column tile, the layout the
decode tail and ms_op_argmax_partials finish.  Checked against float64 logits (the id is the
float64 argmax unless the top two are within fp32 summation noise; each partial max is the
tile's fp32 maximum) and for row independence from the launch's other rows (an engine's
arithmetic must not change with the rows of a step)."""
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


def _partials(lib, X, W, M, N, K):
    part = torch.full((M, N // 16, 2), float("nan"), device=X.device)
    L.check(lib.ms_op_gemm(X.data_ptr(), W.data_ptr(), part.data_ptr(), M, N, K, N // 16, L.MS_EPI_ARGMAX,
                           _stream()))
    return part


@pytest.mark.timeout(300)
@pytest.mark.parametrize("N", [16384, 128256])
@pytest.mark.parametrize("M", [1, 77, 128, 256])
def test_gemm_argmax_vs_fp64(lib, dev, M, N):
    K = 3072
    g = torch.Generator(device="cpu").manual_seed(M + N)
    W = (torch.randn(N, K, generator=g) * 0.05).to(torch.float16).to(dev)
    X = torch.randn(M, K, generator=g).to(torch.float16).to(dev)
    part = _partials(lib, X, W, M, N, K)
    ids = torch.empty(M, dtype=torch.int32, device=dev)
    L.check(lib.ms_op_argmax_partials(part.data_ptr(), M, N // 16, ids.data_ptr(), _stream()))
    torch.cuda.synchronize()
    ref = X.double() @ W.double().T
    # every partial: the tile's maximum (fp32 noise) at an id inside the tile holding it
    tiles = ref.view(M, N // 16, 16)
    tmax, targ = tiles.max(2)
    p = part.cpu().double()
    pid = part[..., 1].contiguous().view(torch.int32).cpu().long()
    assert torch.allclose(p[..., 0], tmax.cpu(), rtol=1e-5, atol=1e-4)
    base = torch.arange(N // 16).view(1, -1) * 16
    assert bool(((pid >= base) & (pid < base + 16)).all())
    got_val = tiles.cpu().gather(2, (pid - base).unsqueeze(2)).squeeze(2)
    assert torch.allclose(got_val, tmax.cpu(), rtol=1e-5, atol=1e-4)  # the id holds the max
    srt = torch.sort(ref, 1).values.cpu()
    top = torch.argmax(ref, 1).cpu()
    got = ids.cpu().long()
    for r in range(M):  # the fp64 argmax, unless the top two are within fp32 noise
        if srt[r, -1] - srt[r, -2] > 1e-4 * (1 + abs(float(srt[r, -1]))):
            assert int(got[r]) == int(top[r]), r


@pytest.mark.timeout(300)
def test_gemm_argmax_rows_independent_of_batch(lib, dev):
    N, K = 128256, 3072
    g = torch.Generator(device="cpu").manual_seed(7)
    W = (torch.randn(N, K, generator=g) * 0.05).to(torch.float16).to(dev)
    X = torch.randn(256, K, generator=g).to(torch.float16).to(dev)
    outs = {M: _partials(lib, X, W, M, N, K).cpu() for M in (24, 77, 128, 256)}
    torch.cuda.synchronize()
    for M in (77, 128, 256):
        assert torch.equal(outs[M][:24].view(torch.int32), outs[24].view(torch.int32)), M


def test_gemm_argmax_refuses_bad_shapes(lib, dev):
    X = torch.zeros(8, 128, dtype=torch.float16, device=dev)
    W = torch.zeros(1000, 128, dtype=torch.float16, device=dev)
    out = torch.zeros(8 * 1000, device=dev)
    assert lib.ms_op_gemm(X.data_ptr(), W.data_ptr(), out.data_ptr(), 8, 1000, 128, 1000 // 16, L.MS_EPI_ARGMAX,
                          _stream()) == L.MS_EINVAL  # N % 16
    assert lib.ms_op_gemm(X.data_ptr(), W.data_ptr(), out.data_ptr(), 8, 992, 128, 61, L.MS_EPI_ARGMAX,
                          _stream()) == L.MS_EINVAL  # ldo < N / 16
