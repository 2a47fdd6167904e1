# torch.matmul (hipBLASLt / rocBLAS) fp16 rates at the prefill GEMM shapes, random data
import torch, time
torch.manual_seed(0)
for (M, N, K, name) in [(16384, 5120, 3072, "qkv"), (16384, 3072, 3072, "o"), (16384, 16384, 3072, "gate/up"),
                        (16384, 3072, 8192, "down"), (8192, 8192, 8192, "8192^3")]:
    a = (torch.rand(M, K, device="cuda", dtype=torch.float16) - 0.5)
    b = (torch.rand(N, K, device="cuda", dtype=torch.float16) - 0.5)
    for _ in range(5): c = a @ b.T
    torch.cuda.synchronize()
    n = 20
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): c = a @ b.T
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / n
    print(f"{name:8s} M={M} N={N} K={K}: {ms*1e3:8.1f} us  {2*M*N*K/ms/1e9:7.1f} TF/s", flush=True)
