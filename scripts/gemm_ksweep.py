#!/usr/bin/env python3
"""GEMM fixed-cost probe: time vs K at fixed M, N for each fast-path variant (HIP events)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


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


def main():
    from dilabhelmholtzoct_amd import _lib, kernels as K
    lib = _lib.load()
    dev = torch.device("cuda")
    M, N = 32768, 2048
    for Kd in (64, 128, 256, 512, 768, 1536, 3072):
        A = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        W = torch.randn(N, Kd, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        row = {"K": Kd}
        for v in (1, 5):
            lib.octsam_gemm_set_fast_path(v)
            ms = timeit(lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=out))
            row[f"v{v}_us"] = round(ms * 1e3, 1)
            row[f"v{v}_tf"] = round(2 * M * N * Kd / ms / 1e9, 1)
        print(json.dumps(row), flush=True)
    lib.octsam_gemm_set_fast_path(1)


if __name__ == "__main__":
    main()
