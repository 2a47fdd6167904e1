"""The large-batch skinny GEMM's two block forms side by side (GPU): 4-wave blocks (kh 1) and
8-wave blocks splitting each 128-k step in two k halves (kh 2), through ms_op_dgemm.

    python tools/dgemm_kh.py [--m 24,64,128,256]

Per shape and batch size: the max |err| of each form against a torch fp32 product of the same
fp16 operands (SwiGLU / argmax applied in fp32), whether kh 2's rows are bitwise independent of
M, and the median launch time (weights rotated over > 512 MB, so no MALL reuse)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from bench_kernels import timeit  # noqa: E402
from mapsum import _lib as L  # noqa: E402

SHAPES = [("gate_up", 16384, 3072, 2), ("lm_head", 128256, 3072, 5), ("o_f32", 3072, 3072, 3)]


def ref(X, W, epi):
    y = X.float() @ W.float().t()
    if epi == 2:  # rows 32 q .. +15 gate, +16 .. +31 up of feature block q
        g = y.view(y.shape[0], -1, 2, 16)
        return (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(y.shape[0], -1)
    return y


def run(lib, X, W, out, M, N, K, epi, st):
    ldo = N // 2 if epi == 2 else (N // 16 if epi == 5 else N)
    rc = lib.ms_op_dgemm(X.data_ptr(), W.data_ptr(), out.data_ptr(), M, N, K, 1, ldo, epi, st)
    assert rc == 0, rc
    return ldo


def view(out, M, N, epi):
    if epi == 2:
        return out.view(torch.float16)[: M * (N // 2)].view(M, N // 2).float()
    if epi == 5:
        return out[: M * (N // 16) * 2].view(M, N // 16, 2)
    return out[: M * N].view(M, N)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="24,64,128,256")
    a = ap.parse_args()
    lib = L.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    for name, N, K, epi in SHAPES:
        Ws = [torch.randn(N, K, device=dev).to(torch.float16) * 0.02
              for _ in range(max(2, -(-512 * 2**20 // (N * K * 2))))]
        Xall = torch.randn(256, K, device=dev).to(torch.float16)
        for M in (int(v) for v in a.m.split(",")):
            X = Xall[:M].contiguous()
            y = ref(X, Ws[0], epi)
            line = f"{name:8s} N={N:6d} K={K} M={M:3d} |"
            res = {}
            for kh in (1, 2):
                assert lib.ms_set_dgemm_kh(kh) == 0
                out = torch.zeros(M * N * 2, device=dev)
                run(lib, X, Ws[0], out, M, N, K, epi, st)
                torch.cuda.synchronize()
                o = view(out, M, N, epi).clone()
                res[kh] = o
                if epi == 5:  # per-16-column {max, id}: the max against the fp32 max of those columns
                    err = (o[..., 0] - y.view(M, -1, 16).max(-1).values).abs().max().item()
                else:
                    err = (o - y).abs().max().item()
                i = [0]

                def fn():
                    i[0] += 1
                    run(lib, X, Ws[i[0] % len(Ws)], out, M, N, K, epi, st)
                t = timeit(fn)
                line += f" kh{kh} err {err:.2e} {t*1e3:6.1f}us {N*K*2/t/1e6:5.0f} GB/s |"
            # kh 2: the first rows of an M-row launch equal those rows launched alone (M = 24)
            out = torch.zeros(24 * N * 2, device=dev)
            run(lib, Xall[:24].contiguous(), Ws[0], out, 24, N, K, epi, st)
            torch.cuda.synchronize()
            same = torch.equal(view(out, 24, N, epi), res[2][:24]) if M >= 24 else True
            line += f" kh2 rows M-invariant {same}"
            print(line, flush=True)
    lib.ms_set_dgemm_kh(1)


if __name__ == "__main__":
    main()
