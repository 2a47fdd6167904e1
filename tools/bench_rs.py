"""Micro-benchmarks of the decode projections around the deferred RMSNorm (GPU): the gate/up
GEMV with no row scale, one-tile and 256-tile statistics; the QKV split-K GEMV; O / down as
split-K slabs + residual_rmsnorm against the fused residual epilogue (ms_op_gemv_resid).
Back-to-back launches on >512 MB weight rotations (no MALL reuse), HIP-event timed.

    python tools/bench_rs.py            (MAPSUM_LIB=... for another build: ops it lacks are skipped)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from bench_kernels import timeit  # noqa: E402
from mapsum import _lib as L  # noqa: E402


def main():
    lib = L.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    M, H, F = 8, 3072, 8192
    ws = torch.zeros(4096, dtype=torch.uint8, device=dev)
    has_rs = hasattr(lib, "ms_op_set_row_scale") and hasattr(lib.ms_op_set_row_scale, "argtypes")
    has_resid = hasattr(lib, "ms_op_gemv_resid")

    def rot(N, K):
        return [torch.randn(N, K, device=dev).to(torch.float16) * 0.02
                for _ in range(max(4, -(-512 * 2**20 // (N * K * 2))))]

    def run(tag, fn, byts):
        t = timeit(fn, reps=40, rounds=7)
        print(f"{tag:34s} {t * 1e3:7.2f} us  {byts / t / 1e6:6.0f} GB/s", flush=True)

    # gate/up + SwiGLU
    Wg = rot(2 * F, H)
    X = torch.randn(M, H, device=dev).to(torch.float16)
    h = torch.empty(M, F, dtype=torch.float16, device=dev)
    i = [0]

    def gu():
        i[0] += 1
        L.check(lib.ms_op_gemv(X.data_ptr(), Wg[i[0] % len(Wg)].data_ptr(), h.data_ptr(), M, 2 * F, H, F, 2,
                               ws.data_ptr(), st))
    run("gate/up", gu, 2 * F * H * 2)
    if has_rs:
        for tiles in (1, 256):
            ssq = torch.rand(tiles, M, device=dev) * 10 + 1
            L.check(lib.ms_op_set_row_scale(ssq.data_ptr(), tiles, H, 1e-5))
            run(f"gate/up rs tiles={tiles}", gu, 2 * F * H * 2)
            L.check(lib.ms_op_set_row_scale(None, 0, 0, 0.0))
    # QKV split-K
    Wq = rot(5120, H)
    slabs = torch.empty(8, M, 5120, device=dev)

    def qkv():
        i[0] += 1
        L.check(lib.ms_op_gemv_split(X.data_ptr(), Wq[i[0] % len(Wq)].data_ptr(), slabs.data_ptr(), M, 5120, H, 6, 0, st))
    run("qkv split6", qkv, 5120 * H * 2)
    # O / down: slabs + residual_rmsnorm vs the fused residual epilogue
    x = torch.randn(M, H, device=dev)
    g = torch.ones(H, dtype=torch.float16, device=dev)
    xb = torch.empty(M, H, dtype=torch.float16, device=dev)
    ssq = torch.empty(256, M, device=dev)
    for name, K, S in (("o", H, 6), ("down", F, 4)):
        Wo = rot(H, K)
        Xo = torch.randn(M, K, device=dev).to(torch.float16)

        def split():
            i[0] += 1
            L.check(lib.ms_op_gemv_split(Xo.data_ptr(), Wo[i[0] % len(Wo)].data_ptr(), slabs.data_ptr(), M, H, K, S, 0, st))
        run(f"{name} split{S}", split, H * K * 2)

        def split_norm():
            split()
            L.check(lib.ms_op_residual_rmsnorm(x.data_ptr(), slabs.data_ptr(), S, g.data_ptr(), xb.data_ptr(),
                                               ssq.data_ptr(), M, H, st))
        if has_resid:
            run(f"{name} split{S} + residual_rmsnorm", split_norm, H * K * 2)

            def resid():
                i[0] += 1
                L.check(lib.ms_op_gemv_resid(Xo.data_ptr(), Wo[i[0] % len(Wo)].data_ptr(), x.data_ptr(), xb.data_ptr(),
                                             g.data_ptr(), ssq.data_ptr(), M, H, K, 12, st))
            run(f"{name} resid rt12", resid, H * K * 2)


if __name__ == "__main__":
    main()
