#!/usr/bin/env python3
"""8-phase GEMM ablation (diagnostic): full kernel (path 1), main loop only (6: epilogue skipped),
epilogue only (7: main loop skipped), at M=32768 N=2048 over K. HIP events, random operands."""
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
    shapes = [(32768, 2048, 64), (32768, 2048, 768), (32768, 2304, 768), (32768, 3072, 768), (32768, 768, 3072),
              (688128, 256, 128), (688128, 384, 256)]
    for M, N, Kd in shapes:
        A = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        W = torch.randn(N, Kd, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        row = {"MNK": [M, N, Kd]}
        for v in (1, 10, 6, 7):
            lib.octsam_gemm_set_fast_path(v)
            ms = timeit(lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=out))
            row[f"v{v}_us"] = round(ms * 1e3, 1)
        row["tf"] = round(2 * M * N * Kd / row["v1_us"] / 1e6, 1)
        row["out_GBps"] = round(M * N * 2 / row["v1_us"] / 1e3, 1)
        print(json.dumps(row), flush=True)
    lib.octsam_gemm_set_fast_path(1)


if __name__ == "__main__":
    main()
