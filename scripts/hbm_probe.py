#!/usr/bin/env python3
"""Reference points on the box: HBM write / copy bandwidth (torch fill_/copy_) and hipBLASLt bf16 GEMM
(torch.matmul) at the encoder shapes. Diagnostic only (not part of the product path)."""
import json
import torch


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev = torch.device("cuda")
x = torch.empty(32768 * 2048, device=dev, dtype=torch.bfloat16)
y = torch.empty_like(x)
ms = timeit(lambda: x.fill_(1.0))
print(json.dumps({"fill_GBps": round(x.numel() * 2 / ms / 1e6, 1)}))
ms = timeit(lambda: y.copy_(x))
print(json.dumps({"copy_GBps(r+w)": round(x.numel() * 4 / ms / 1e6, 1)}))
for M, N, K in [(32768, 2304, 768), (32768, 3072, 768), (32768, 768, 3072), (32768, 2048, 64), (32768, 2048, 3072)]:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev).to(torch.bfloat16)
    ms = timeit(lambda: A @ W.t())
    print(json.dumps({"torch_matmul": [M, N, K], "us": round(ms * 1e3, 1), "tflops": round(2 * M * N * K / ms / 1e9, 1)}))
