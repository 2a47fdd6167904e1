"""Probe: the large-batch lm_head (M = 128 rows, N = 128256, K = 3072) on the prefill GEMM
tiles (fp32 logits + an argmax pass) against the skinny GEMM's argmax epilogue (GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from bench_kernels import timeit  # noqa: E402
from mapsum import _lib as L  # noqa: E402

lib = L.load()
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
M, N, K = 128, 128256, 3072
Ws = [torch.randn(N, K, device=dev).to(torch.float16) * 0.02 for _ in range(2)]
X = torch.randn(M, K, device=dev).to(torch.float16)
logits = torch.empty(M, N, device=dev)
ids = torch.empty(M, dtype=torch.int32, device=dev)
part = torch.empty(M, N // 16, 2, device=dev)
i = [0]


def nextw():
    i[0] += 1
    return Ws[i[0] % 2]


for v in (1, 2, 3, 4):
    L.check(lib.ms_set_gemm_variant(v))
    t = timeit(lambda: lib.ms_op_gemm(X.data_ptr(), nextw().data_ptr(), logits.data_ptr(), M, N, K, N, 3, st), reps=10,
               rounds=3)
    ta = timeit(lambda: lib.ms_op_argmax(logits.data_ptr(), M, N, ids.data_ptr(), st), reps=10, rounds=3)
    print(f"gemm variant {v}: {t*1e3:7.1f} us + argmax {ta*1e3:6.1f} us", flush=True)
lib.ms_set_gemm_variant(L.GEMM_DEFAULT)
for wn in (4, 8):
    L.check(lib.ms_set_dgemm_kh(1))
    L.check(lib.ms_set_dgemm_wn(wn))
    t = timeit(lambda: lib.ms_op_dgemm(X.data_ptr(), nextw().data_ptr(), part.data_ptr(), M, N, K, 1, N // 16, 5, st),
               reps=10, rounds=3)
    tp = timeit(lambda: lib.ms_op_argmax_partials(part.data_ptr(), M, N // 16, ids.data_ptr(), st), reps=10, rounds=3)
    print(f"dgemm argmax wn {wn}: {t*1e3:7.1f} us + partials {tp*1e3:6.1f} us", flush=True)
lib.ms_set_dgemm_wn(4)
lib.ms_set_dgemm_kh(2)
