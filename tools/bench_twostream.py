"""Does a second decode stream hide the per-launch ramp of the weight-streaming GEMVs? (GPU)

A decode "layer" here is four weight streams (QKV, O, gate/up + SwiGLU, down) of the
Llama-3.2-3B shapes, over 28 distinct layers' weights (5.6 GB: every launch streams from
HBM, as in a decode step).  Case 1: one stream, M rows.  Case 2: two streams of M/2 rows
each running the same 28-layer sequence concurrently (the trailing stream's weight reads
can hit the Infinity Cache behind the leading one).  Prints wall time per 28-layer pass.
    python tools/bench_twostream.py [--m 8] [--reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mapsum import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--layers", type=int, default=28)
    a = ap.parse_args()
    lib = L.load()
    dev = torch.device("cuda:0")
    H, F, QKVN = 3072, 8192, 5120
    shapes = [("qkv", QKVN, H, 3), ("o", H, H, 3), ("gu", 2 * F, H, 2), ("down", H, F, 3)]
    Ws = [[(torch.randn(N, K, device=dev) * 0.02).to(torch.float16) for (_, N, K, _) in shapes]
          for _ in range(a.layers)]
    ws = torch.zeros(4096, dtype=torch.uint8, device=dev)

    def bufs(M):
        X = {K: torch.randn(M, K, device=dev).to(torch.float16) for K in (H, F)}
        out = torch.zeros(M, 2 * F, device=dev)
        return X, out

    def run(jobs):
        """jobs: [(stream, M, X, out)]: the layer sequence on every stream, launches interleaved
        so the streams start together"""
        for l in range(a.layers):
            for (name, N, K, epi), W in zip(shapes, Ws[l]):
                ldo = N // 2 if epi == 2 else N
                for stream, M, X, out in jobs:
                    rc = lib.ms_op_gemv(X[K].data_ptr(), W.data_ptr(), out.data_ptr(), M, N, K, ldo, epi,
                                        ws.data_ptr(), stream.cuda_stream)
                    if rc:
                        raise RuntimeError(lib.ms_last_error(None))

    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    M = a.m
    one = bufs(M)
    half = [bufs(M // 2), bufs(M // 2)]

    def time_it(fn):
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch.cuda.current_stream())
            s0.wait_stream(torch.cuda.current_stream())
            s1.wait_stream(torch.cuda.current_stream())
            fn()
            torch.cuda.current_stream().wait_stream(s0)
            torch.cuda.current_stream().wait_stream(s1)
            e1.record(torch.cuda.current_stream())
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    t1 = time_it(lambda: run([(s0, M, *one)]))
    t2 = time_it(lambda: run([(s0, M // 2, *half[0]), (s1, M // 2, *half[1])]))
    t1b = time_it(lambda: run([(s0, M, *one)]))
    wb = sum(N * K * 2 for (_, N, K, _) in shapes) * a.layers
    print(f"one stream M={M}: {t1:.3f} / {t1b:.3f} ms per {a.layers}-layer pass ({wb / t1 / 1e6:.0f} GB/s)")
    print(f"two streams M={M // 2} each: {t2:.3f} ms ({wb / t2 / 1e6:.0f} GB/s of distinct weights)", flush=True)


if __name__ == "__main__":
    main()
