"""The persistent decode GEMV (k_gemv.hip pgemv_kernel) computes exactly what the one-block-
per-tile GEMV computes for the same split: bit-identical slabs / SwiGLU outputs at the
Llama-3.2-3B decode shapes (needs a GPU)."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from mapsum import _lib as L  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _st():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("N,K,S", [(5120, 3072, 4), (3072, 3072, 4), (3072, 8192, 4), (3072, 3072, 6)])
def test_pgemv_split_bit_exact(dev, M, N, K, S):
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(N + K + M)
    X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    a = torch.full((S, M, N), float("nan"), device=dev)
    b = torch.full((S, M, N), float("nan"), device=dev)
    L.check(lib.ms_op_gemv_split(X.data_ptr(), W.data_ptr(), a.data_ptr(), M, N, K, S, 0, _st()))
    rc = lib.ms_op_pgemv(X.data_ptr(), W.data_ptr(), b.data_ptr(), M, N, K, S, N, L.MS_EPI_STORE_F32, _st())
    if S == 6 and (K // S) % 64:
        assert rc < 0
        return
    L.check(rc)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    ref = torch.stack([X[:, s * K // S:(s + 1) * K // S].double() @ W[:, s * K // S:(s + 1) * K // S].double().T
                       for s in range(S)])
    assert float((b.double() - ref).norm() / ref.norm()) < 2e-6


@pytest.mark.parametrize("M", [1, 8, 16])
def test_pgemv_swiglu_bit_exact(dev, M):
    lib = L.load()
    N, K = 16384, 3072
    g = torch.Generator(device="cuda").manual_seed(M)
    X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    a = torch.zeros(M, N // 2, dtype=torch.bfloat16, device=dev)
    b = torch.ones(M, N // 2, dtype=torch.bfloat16, device=dev)
    ws = torch.zeros(256, dtype=torch.uint8, device=dev)
    L.check(lib.ms_op_gemv(X.data_ptr(), W.data_ptr(), a.data_ptr(), M, N, K, N // 2, L.MS_EPI_SWIGLU,
                           ws.data_ptr(), _st()))
    rc = lib.ms_op_pgemv(X.data_ptr(), W.data_ptr(), b.data_ptr(), M, N, K, 1, N // 2, L.MS_EPI_SWIGLU, _st())
    if M == 16:  # X image (96 KB) + two reduction stages exceed the 160 KB of LDS: refused
        assert rc < 0
        return
    L.check(rc)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
