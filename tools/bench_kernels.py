"""Kernel micro-benchmarks through the C-ABI op entry points (GPU).

    python tools/bench_kernels.py gemv [--m 8]
    python tools/bench_kernels.py gemm

Operands are fp16 (the engine's storage type).  Times each launch with HIP events on the
launch stream (median of interleaved rounds),
reports algorithmic GB/s (gemv: weight + activation bytes) or TFLOP/s (gemm).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mapsum import _lib as L  # noqa: E402


def timeit(fn, reps=20, rounds=5):
    s = torch.cuda.current_stream()
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / reps)
    return float(np.median(res))


def bench_gemv(lib, M, shapes, waves_list):
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.zeros(4096, dtype=torch.uint8, device=dev)
    # a 1 GB buffer swept between rounds keeps weights out of the 256 MB MALL
    flush = torch.empty(256 * 1024 * 1024, dtype=torch.float32, device=dev)
    for name, N, K, epi in shapes:
        Ws = [torch.randn(N, K, device=dev).to(torch.float16) * 0.02 for _ in range(8)]
        X = torch.randn(M, K, device=dev).to(torch.float16)
        out = torch.zeros(M, N if epi != 2 else N // 2, device=dev,
                          dtype=torch.float32 if epi in (1, 3) else torch.float16)
        ldo = N if epi != 2 else N // 2
        byts = N * K * 2 + M * K * 2 + out.numel() * out.element_size() * (2 if epi == 1 else 1)
        line = f"{name:8s} N={N:6d} K={K:5d} M={M:3d} {byts/1e6:8.1f} MB |"
        for wv in waves_list:
            i = [0]

            def fn():
                W = Ws[i[0] % len(Ws)]
                i[0] += 1
                rc = lib.ms_op_gemv_tuned(X.data_ptr(), W.data_ptr(), out.data_ptr(), M, N, K, ldo, epi,
                                          ws.data_ptr(), wv, st)
                if rc:
                    raise RuntimeError(lib.ms_last_error(None))
            try:
                flush.zero_()
                t = timeit(fn)
                line += f" w{wv}: {t*1e3:7.1f}us {byts/t/1e6:6.0f}GB/s |"
            except RuntimeError:
                line += f" w{wv}: n/a |"
        print(line, flush=True)


def bench_split(lib, M):
    """Split-K decode GEMV into fp32 slabs (O / down projections) over (S, waves)."""
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for name, N, K in [("o", 3072, 3072), ("down", 3072, 8192), ("qkv", 5120, 3072)]:
        # enough weight copies that the rotation streams > 512 MB: the 256 MB MALL never
        # holds the matrix a launch reads (as in a decode step, which streams 6.4 GB)
        Ws = [torch.randn(N, K, device=dev).to(torch.float16) * 0.02
              for _ in range(max(8, -(-512 * 2**20 // (N * K * 2))))]
        X = torch.randn(M, K, device=dev).to(torch.float16)
        slabs = torch.zeros(8, M, N, device=dev)
        for S in (1, 2, 3, 4, 6, 8):
            byts = N * K * 2 + M * K * 2 + S * M * N * 4
            line = f"{name:5s} N={N:5d} K={K:5d} M={M:2d} S={S} |"
            for wv in (0, 1, 2, 3, 4, 6, 8, 12, 16):
                i = [0]

                def fn():
                    W = Ws[i[0] % len(Ws)]
                    i[0] += 1
                    rc = lib.ms_op_gemv_split(X.data_ptr(), W.data_ptr(), slabs.data_ptr(), M, N, K, S, wv, st)
                    if rc:
                        raise RuntimeError(lib.ms_last_error(None))
                try:
                    t = timeit(fn)
                    line += f" w{wv}: {t*1e3:6.1f}us {byts/t/1e6:5.0f} |"
                except RuntimeError:
                    line += f" w{wv}: n/a |"
            print(line, flush=True)


def bench_dgemm(lib):
    """Decode projections over the batch sizes of the continuous batch: the weight-streaming
    GEMV (M <= 64), the large-batch skinny GEMM (k_dgemm.hip) over split counts, and the
    prefill GEMM fallback, all on >512 MB weight rotations (no MALL reuse)."""
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.zeros(4096, dtype=torch.uint8, device=dev)
    for name, N, K, epi, splits in [("qkv", 5120, 3072, 3, (1, 2, 3, 6)), ("o", 3072, 3072, 3, (1, 2, 4, 6)),
                                    ("gu", 16384, 3072, 2, (1,)), ("down", 3072, 8192, 3, (1, 2, 4, 8)),
                                    ("lm_head", 128256, 3072, 5, (1,))]:
        Ws = [torch.randn(N, K, device=dev).to(torch.float16) * 0.02
              for _ in range(max(2, -(-512 * 2**20 // (N * K * 2))))]
        for M in (8, 16, 32, 64, 128, 256):
            X = torch.randn(M, K, device=dev).to(torch.float16)
            out = torch.zeros(8 * M * N, device=dev)
            wbytes = N * K * 2
            line = f"{name:7s} N={N:6d} K={K:5d} M={M:3d} |"
            i = [0]

            def nextw():
                i[0] += 1
                return Ws[i[0] % len(Ws)]
            ldo = N // 2 if epi == 2 else (N // 16 if epi == 5 else N)
            if M <= 64:
                t = timeit(lambda: lib.ms_op_gemv(X.data_ptr(), nextw().data_ptr(), out.data_ptr(), M, N, K, ldo,
                                                  epi, ws.data_ptr(), st))
                line += f" gemv {t*1e3:6.1f}us {wbytes/t/1e6:5.0f} |"
            for S in splits:
                e = epi if S == 1 else 3
                rc = lib.ms_op_dgemm(X.data_ptr(), Ws[0].data_ptr(), out.data_ptr(), M, N, K, S, ldo if S == 1 else N,
                                     e, st)
                if rc:
                    line += f" dg S{S} n/a |"
                    continue
                t = timeit(lambda: lib.ms_op_dgemm(X.data_ptr(), nextw().data_ptr(), out.data_ptr(), M, N, K, S,
                                                   ldo if S == 1 else N, e, st))
                line += f" dg S{S} {t*1e3:6.1f}us {wbytes/t/1e6:5.0f} |"
            if M > 16 and epi != 5:
                e = epi if epi != 5 else 3
                t = timeit(lambda: lib.ms_op_gemm(X.data_ptr(), nextw().data_ptr(), out.data_ptr(), M, N, K, ldo, e, st))
                line += f" gemm {t*1e3:6.1f}us |"
            print(line, flush=True)


def bench_qgemv(lib, M):
    """Dequant-fused decode GEMV (k_qgemv.hip) on the Q4_K_M shapes at M rows: plain launch
    and split-K slabs over S, on > 512 MB rotations of packed weights (no MALL reuse).
    GB/s = compressed weight bytes / time."""
    from oracle import quants as Q
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for name, N, K, qt, epi in [("qkv", 5120, 3072, 12, 3), ("o", 3072, 3072, 12, 1), ("gu", 16384, 3072, 12, 2),
                                ("down", 3072, 8192, 12, 1), ("down6", 3072, 8192, 14, 1),
                                ("lm_head6", 128256, 3072, 14, 3)]:
        bpb = 144 if qt == 12 else 224
        nbytes = N * (K // 256) * bpb
        b = Q.random_blocks(qt, min(N, 4096) * K // 256, seed=1, scale=0.02)
        bd = torch.from_numpy(b.reshape(-1)).to(dev)
        rows_src = min(N, 4096)
        pks = []
        for _ in range(max(2, -(-512 * 2**20 // nbytes))):
            pk = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            wbf = torch.empty(rows_src, K, dtype=torch.float16, device=dev)
            for r0 in range(0, N, rows_src):  # tile the random rows over the matrix
                rr = min(rows_src, N - r0)
                tmp = torch.empty(rr * (K // 256) * bpb, dtype=torch.uint8, device=dev)
                lib.ms_op_quant_rows(qt, bd.data_ptr(), rr, K, wbf.data_ptr(), tmp.data_ptr(), st)
                pk[r0 * (K // 256) * bpb:(r0 + rr) * (K // 256) * bpb] = tmp
            pks.append(pk)
        X = torch.randn(M, K, device=dev).to(torch.float16)
        out = torch.zeros(8 * M * N, device=dev)
        ldo = N // 2 if epi == 2 else N
        i = [0]

        def nextp():
            i[0] += 1
            return pks[i[0] % len(pks)]
        line = f"{name:8s} N={N:6d} K={K:5d} M={M:2d} {nbytes/1e6:6.1f} MB |"
        t = timeit(lambda: lib.ms_op_qgemv(X.data_ptr(), qt, nextp().data_ptr(), out.data_ptr(), M, N, K, ldo, epi, st))
        line += f" plain {t*1e3:6.1f}us {nbytes/t/1e6:5.0f} |"
        if epi != 2:
            for S in (2, 3, 4, 6, 8):
                if (K // 256) % S:
                    continue
                t = timeit(lambda: lib.ms_op_qgemv_split(X.data_ptr(), qt, nextp().data_ptr(), out.data_ptr(), M, N, K,
                                                         S, st))
                line += f" S{S} {t*1e3:6.1f}us {nbytes/t/1e6:5.0f} |"
        print(line, flush=True)



def bench_qdgemm(lib, ms=(64, 128, 256), only=None):
    """Large-batch K-quant decode GEMM (k_qdgemm.hip) against the fp16 skinny GEMM (k_dgemm.hip)
    on the same shapes, > 512 MB rotations of packed / fp16 weights (no MALL reuse).
    GB/s = the weight bytes each reads / time."""
    from oracle import quants as Q
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for name, N, K, qt, epi, splits in [("qkv", 5120, 3072, 12, 3, (1, 2, 3, 6)), ("o", 3072, 3072, 12, 3, (1, 2, 4)),
                                        ("gu", 16384, 3072, 12, 2, (1,)), ("down", 3072, 8192, 12, 3, (1, 2, 4, 8)),
                                        ("down6", 3072, 8192, 14, 3, (2, 4, 8)), ("lm_head6", 128256, 3072, 14, 5, (1,))]:
        if only and name not in only:
            continue
        bpb = 144 if qt == 12 else 224
        nbytes = N * (K // 256) * bpb
        rows_src = min(N, 4096)
        b = Q.random_blocks(qt, rows_src * K // 256, seed=1, scale=0.02)
        bd = torch.from_numpy(b.reshape(-1)).to(dev)
        wbf = torch.empty(rows_src, K, dtype=torch.float16, device=dev)
        tmp = torch.empty(rows_src * (K // 256) * bpb, dtype=torch.uint8, device=dev)
        lib.ms_op_quant_rows(qt, bd.data_ptr(), rows_src, K, wbf.data_ptr(), tmp.data_ptr(), st)
        pks, ws16 = [], []
        for _ in range(max(2, -(-512 * 2**20 // nbytes))):
            pk = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            for r0 in range(0, N, rows_src):  # tile the random rows over the matrix
                rr = min(rows_src, N - r0)
                pk[r0 * (K // 256) * bpb:(r0 + rr) * (K // 256) * bpb] = tmp[:rr * (K // 256) * bpb]
            pks.append(pk)
        for _ in range(max(2, -(-512 * 2**20 // (N * K * 2)))):
            ws16.append(wbf.repeat((N + rows_src - 1) // rows_src, 1)[:N].contiguous())
        ldo = N // 2 if epi == 2 else (N // 16 if epi == 5 else N)
        for M in ms:
            X = torch.randn(M, K, device=dev).to(torch.float16)
            out = torch.zeros(8 * M * N, device=dev)
            i = [0]

            def nxt(lst):
                i[0] += 1
                return lst[i[0] % len(lst)]
            line = f"{name:8s} N={N:6d} K={K:5d} M={M:3d} {nbytes/1e6:6.1f} MB |"
            for S in splits:
                e, lo = (epi, ldo) if S == 1 else (3, N)
                if lib.ms_op_qdgemm(X.data_ptr(), qt, pks[0].data_ptr(), out.data_ptr(), M, N, K, S, lo, e, st):
                    line += f" q S{S} n/a |"
                else:
                    t = timeit(lambda: lib.ms_op_qdgemm(X.data_ptr(), qt, nxt(pks).data_ptr(), out.data_ptr(), M, N, K,
                                                        S, lo, e, st))
                    line += f" q S{S} {t*1e3:6.1f}us {nbytes/t/1e6:5.0f} |"
                if lib.ms_op_dgemm(X.data_ptr(), ws16[0].data_ptr(), out.data_ptr(), M, N, K, S, lo, e, st) == 0:
                    t = timeit(lambda: lib.ms_op_dgemm(X.data_ptr(), nxt(ws16).data_ptr(), out.data_ptr(), M, N, K, S,
                                                       lo, e, st))
                    line += f" f16 {t*1e3:6.1f}us"
                if lib.ms_op_qdgemm(X.data_ptr(), 1, ws16[0].data_ptr(), out.data_ptr(), M, N, K, S, lo, e, st) == 0:
                    t = timeit(lambda: lib.ms_op_qdgemm(X.data_ptr(), 1, nxt(ws16).data_ptr(), out.data_ptr(), M, N, K,
                                                        S, lo, e, st))
                    line += f" h {t*1e3:6.1f}us |"
            print(line, flush=True)

def bench_camp(lib, M):
    """Unsplit decode GEMV over weight rows padded to ldk = K + pad elements: does the row
    stride (16 KB for the down projection) concentrate a launch on a few HBM channels?"""
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for name, N, K, epi in [("o", 3072, 3072, 1), ("down", 3072, 8192, 1), ("qkv", 5120, 3072, 3),
                            ("gu-like", 16384, 3072, 3)]:
        line = f"{name:8s} N={N:6d} K={K:5d} M={M:2d} |"
        for pad in (0, 64, 128, 256, 512):
            ldk = K + pad
            Ws = [torch.randn(N, ldk, device=dev).to(torch.float16) * 0.02
                  for _ in range(max(2, -(-512 * 2**20 // (N * ldk * 2))))]
            X = torch.randn(M, ldk, device=dev).to(torch.float16)
            out = torch.zeros(M, N, device=dev)
            i = [0]

            def fn():
                i[0] += 1
                rc = lib.ms_op_gemv_strided(X.data_ptr(), Ws[i[0] % len(Ws)].data_ptr(), out.data_ptr(), M, N, K,
                                            ldk, N, epi, st)
                if rc:
                    raise RuntimeError(lib.ms_last_error(None))
            t = timeit(fn)
            line += f" pad{pad}: {t*1e3:6.1f}us {N*K*2/t/1e6:5.0f} |"
            del Ws
        print(line, flush=True)


def _trunc(x, bits):
    """fp16 tensor with the low `bits` mantissa bits cleared (bits = 3: bf16-like precision)"""
    if bits <= 0:
        return x
    return (x.view(torch.int16) & ~((1 << bits) - 1)).view(torch.float16)


def bench_gemm(lib, rs=False, variants=(1, 2), ascale=1.0, trunc=0, torch_ref=False, ref_lib=None, resid=False):
    """rs: the normalised projections (epi 0 / 2) take a one-tile deferred-norm row scale, as
    in prefill (ms_op_set_row_scale; needs a library that has it).  ref_lib: a second build
    (L.load_at) timed on the same operands right after each variant, and checked bit for bit"""
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    ssq = (torch.rand(16384, device=dev) * 3072 + 1.0).float()
    for name, M, N, K, epi in [("qkv", 16384, 5120, 3072, 0), ("o", 16384, 3072, 3072, 1),
                               ("gu", 16384, 16384, 3072, 2), ("down", 16384, 3072, 8192, 1),
                               ("sq4k", 4096, 4096, 4096, 0), ("sq8k", 8192, 8192, 8192, 0)]:
        A = _trunc(((torch.rand(M, K, device=dev) * 2 - 1) * ascale).to(torch.float16), trunc)
        W = _trunc((torch.rand(N, K, device=dev) * 2 - 1).to(torch.float16), trunc)
        out = torch.zeros(M, N if epi != 2 else N // 2, device=dev,
                          dtype=torch.float32 if epi in (1, 3) else torch.float16)
        ldo = N if epi != 2 else N // 2
        # the engine's residual form (--resid): x += A W^T, f16(x g 2^-4) and the 128-column
        # statistics (ms_op_gemm_resid) instead of the plain add
        xg = torch.empty(M, N, device=dev, dtype=torch.float16) if resid and epi == 1 else None
        gam = torch.rand(N, device=dev).to(torch.float16) if xg is not None else None
        sq = torch.empty(N // 128, M, device=dev) if xg is not None else None

        def call(L_, o_):
            if xg is not None:
                L_.ms_op_gemm_resid(A.data_ptr(), W.data_ptr(), o_.data_ptr(), xg.data_ptr(), gam.data_ptr(),
                                    sq.data_ptr(), M, N, K, st)
            else:
                L_.ms_op_gemm(A.data_ptr(), W.data_ptr(), o_.data_ptr(), M, N, K, ldo, epi, st)

        def fn():
            if rs:
                lib.ms_op_set_row_scale(ssq.data_ptr() if epi in (0, 2) else None, 1, K, 1e-5)
            call(lib, out)
        ref_out = None
        for variant in variants:
            L.check(lib.ms_set_gemm_variant(variant))
            if epi == 1:
                out.zero_()
            fn()
            torch.cuda.synchronize()
            same = ""
            if ref_out is None:
                ref_out = out.clone()
            else:
                same = " bit-identical" if torch.equal(out, ref_out) else \
                    f" DIFFERS (max abs {float((out.float() - ref_out.float()).abs().max()):.3e})"
            t = timeit(fn, reps=5, rounds=3)
            print(f"  (v{variant} vs v{variants[0]}:{same or ' reference'})", flush=True)
            print(f"gemm v{variant} {name:5s} M={M} N={N} K={K}: {t:.3f} ms  {2*M*N*K/t/1e9:.0f} TFLOP/s",
                  flush=True)
            if ref_lib is not None:
                mine = out.clone()

                def fn_ref():
                    if rs:
                        ref_lib.ms_op_set_row_scale(ssq.data_ptr() if epi in (0, 2) else None, 1, K, 1e-5)
                    call(ref_lib, out)
                L.check(ref_lib.ms_set_gemm_variant(variant))
                if epi == 1:  # the residual epilogue accumulates: compare one launch on zeros each
                    out.zero_()
                    fn()
                    torch.cuda.synchronize()
                    mine = out.clone()
                    out.zero_()
                fn_ref()
                torch.cuda.synchronize()
                eq = "bit-identical" if torch.equal(out, mine) else \
                    f"DIFFERS (max abs {float((out.float() - mine.float()).abs().max()):.3e})"
                tr = timeit(fn_ref, reps=5, rounds=3)
                t2 = timeit(fn, reps=5, rounds=3)
                print(f"base v{variant} {name:5s} M={M} N={N} K={K}: {tr:.3f} ms  {2*M*N*K/tr/1e9:.0f} TFLOP/s "
                      f"(this build again {t2:.3f} ms; outputs {eq})", flush=True)
                ref_lib.ms_set_gemm_variant(4)
        lib.ms_set_gemm_variant(L.GEMM_DEFAULT)
        if torch_ref:  # the library GEMM (hipBLASLt via torch.matmul) on the same operands, no epilogue
            t = timeit(lambda: torch.matmul(A, W.t()), reps=5, rounds=3)
            print(f"torch   {name:5s} M={M} N={N} K={K}: {t:.3f} ms  {2*M*N*K/t/1e9:.0f} TFLOP/s", flush=True)


def bench_rows(lib, ms=(128, 192, 256)):
    """Decode projections at M = 128-256 rows: the decode skinny GEMM (k_dgemm.hip, its split-K
    options) against the prefill GEMM's 128x128 tile (k_gemm.hip gemm_kernel, the small-M
    dispatch) on the same operands, > 512 MB weight rotations (no MALL reuse)."""
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for name, N, K, epi, splits in [("qkv", 5120, 3072, 0, (1, 2, 3)), ("o", 3072, 3072, 3, (1, 2, 4)),
                                    ("gu", 16384, 3072, 2, (1,)), ("down", 3072, 8192, 3, (1, 2, 4, 8)),
                                    ("lm_head", 128256, 3072, 0, (1,))]:
        ws = [(torch.rand(N, K, device=dev) * 2 - 1).to(torch.float16)
              for _ in range(max(2, -(-512 * 2**20 // (N * K * 2))))]
        ldo = N // 2 if epi == 2 else N
        i = [0]

        def nxt():
            i[0] += 1
            return ws[i[0] % len(ws)]
        for M in ms:
            X = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.float16)
            out = torch.zeros(8 * M * N, device=dev)
            line = f"{name:8s} N={N:6d} K={K:5d} M={M:3d} {N*K*2/1e6:6.1f} MB |"
            for S in splits:
                e, lo = (epi, ldo) if S == 1 else (3, N)
                if lib.ms_op_dgemm(X.data_ptr(), ws[0].data_ptr(), out.data_ptr(), M, N, K, S, lo, e, st) == 0:
                    t = timeit(lambda: lib.ms_op_dgemm(X.data_ptr(), nxt().data_ptr(), out.data_ptr(), M, N, K, S,
                                                       lo, e, st))
                    line += f" dgemm S{S} {t*1e3:6.1f}us |"
            L.check(lib.ms_set_gemm_variant(1))
            t = timeit(lambda: lib.ms_op_gemm(X.data_ptr(), nxt().data_ptr(), out.data_ptr(), M, N, K, ldo, epi, st))
            line += f" gemm128 {t*1e3:6.1f}us |"
            L.check(lib.ms_set_gemm_variant(L.GEMM_DEFAULT))
            print(line, flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["gemv", "gemm", "split", "dgemm", "qgemv", "camp", "qdgemm", "rows"])
    ap.add_argument("--m", type=int, default=8)
    ap.add_argument("--ascale", type=float, default=1.0, help="gemm: scale of the uniform A entries")
    ap.add_argument("--trunc", type=int, default=0, help="gemm: clear this many low mantissa bits of A and W")
    ap.add_argument("--rs", action="store_true", help="gemm: deferred-norm row scale on epi 0 / 2")
    ap.add_argument("--variants", default="1,2", help="gemm: tile variants (1: 128x128, 2: 256x256)")
    ap.add_argument("--torch", action="store_true", help="gemm: also time torch.matmul (hipBLASLt) on the same operands")
    ap.add_argument("--ref-lib", default="", help="gemm: a second build (e.g. libmapsum_base.so) timed and compared")
    ap.add_argument("--resid", action="store_true", help="gemm: O / down through ms_op_gemm_resid (the engine's form)")
    ap.add_argument("--kh", type=int, default=1, help="dgemm: block form (ms_set_dgemm_kh: 1 4-wave, 2 k-half 8-wave)")
    ap.add_argument("--ms", default="64,128,256", help="qdgemm: batch rows")
    ap.add_argument("--only", default="", help="qdgemm: comma-separated shape names")
    a = ap.parse_args()
    lib = L.load()
    if a.what == "gemv":
        shapes = [("qkv", 5120, 3072, 0), ("o", 3072, 3072, 1), ("gu", 16384, 3072, 2),
                  ("down", 3072, 8192, 1), ("lm_head", 128256, 3072, 3)]
        bench_gemv(lib, a.m, shapes, [0, 6, 8, 12, 16])
    elif a.what == "split":
        bench_split(lib, a.m)
    elif a.what == "dgemm":
        assert lib.ms_set_dgemm_kh(a.kh) == 0
        bench_dgemm(lib)
    elif a.what == "qgemv":
        bench_qgemv(lib, a.m)
    elif a.what == "camp":
        bench_camp(lib, a.m)
    elif a.what == "rows":
        bench_rows(lib, tuple(int(v) for v in a.ms.split(",")))
    elif a.what == "qdgemm":
        bench_qdgemm(lib, tuple(int(v) for v in a.ms.split(",")), a.only.split(",") if a.only else None)
    else:
        ref = L.load_at(a.ref_lib) if a.ref_lib else None
        bench_gemm(lib, a.rs, tuple(int(v) for v in a.variants.split(",")), a.ascale, a.trunc, a.torch, ref, a.resid)
