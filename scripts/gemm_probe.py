#!/usr/bin/env python3
"""One GEMM shape launched repeatedly (for rocprofv3 --pmc / kernel-trace; diagnostic).
usage: gemm_probe.py M N K [act] [f32out] [residual] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dilabhelmholtzoct_amd import _lib, kernels
    fast = int(os.environ.get("FAST", "1"))
    _lib.load().octsam_gemm_set_fast_path(fast)
    M, N, K = (int(x) for x in sys.argv[1:4])
    act = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    f32 = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    res = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    reps = int(sys.argv[7]) if len(sys.argv) > 7 else 20
    dev = torch.device("cuda", 0)
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    R = torch.randn(M, N, device=dev, dtype=out.dtype) if res else None
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(reps + 3):
        if i == 3:
            s.record()
        kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=bias, act=act, residual=R)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / reps
    byts = 2 * (M + N) * K + M * N * out.element_size() * (2 if res else 1)
    print(f"fast={fast} path={_lib.load().octsam_gemm_last_path()} M={M} N={N} K={K} act={act} f32={f32} res={res}: "
          f"{us:.1f} us/launch, {2 * M * N * K / us / 1e6:.0f} TFLOP/s, {byts / us / 1e3:.0f} GB/s")


if __name__ == "__main__":
    main()
