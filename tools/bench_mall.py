"""What a decode projection gains when its weights are already in the Infinity Cache (GPU).

For each decode GEMV shape at M rows, three cache states of the weight matrix before a timed
launch (HIP events around the launch alone):
  cold  a 1 GiB sweep in between: weights come from HBM (a decode step's state);
  mall  a 64 MiB sweep in between: the L2s (4 MiB per XCD) are flushed, the 256 MiB
        Infinity Cache still holds the weights -- the state a prefetch by an earlier
        kernel would leave;
  hot   back to back: L2 + Infinity Cache.
    python tools/bench_mall.py [--m 8]
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
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    lib = L.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    ws = torch.zeros(4096, dtype=torch.uint8, device=dev)
    big = torch.empty(256 * 2**20, dtype=torch.float32, device=dev)  # 1 GiB
    big.fill_(1.0)
    small = big[: 16 * 2**20]  # 64 MiB
    acc = torch.zeros((), device=dev)
    M = a.m
    for name, N, K, epi in [("qkv", 5120, 3072, 3), ("o", 3072, 3072, 1), ("gu", 16384, 3072, 2),
                            ("down", 3072, 8192, 1)]:
        W = (torch.randn(N, K, device=dev) * 0.02).to(torch.float16)
        X = torch.randn(M, K, device=dev).to(torch.float16)
        ldo = N // 2 if epi == 2 else N
        out = torch.zeros(M, ldo, device=dev, dtype=torch.float32 if epi in (1, 3) else torch.float16)

        def run():
            rc = lib.ms_op_gemv(X.data_ptr(), W.data_ptr(), out.data_ptr(), M, N, K, ldo, epi, ws.data_ptr(),
                                st.cuda_stream)
            if rc:
                raise RuntimeError(lib.ms_last_error(None))
        line = f"{name:5s} N={N:6d} K={K:5d} M={M:3d} {N*K*2/1e6:6.1f} MB |"
        for state in ("cold", "mall", "hot"):
            ts = []
            for _ in range(a.reps):
                # read-only sweeps: a write sweep leaves dirty Infinity-Cache lines whose
                # write-back then lands inside the timed launch
                if state == "cold":
                    acc.copy_(big.sum())
                elif state == "mall":
                    acc.copy_(small.sum())
                else:
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                run()
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            t = float(np.median(ts))
            line += f" {state} {t:6.1f}us {N*K*2/t/1e6:5.2f}TB/s |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
