#!/usr/bin/env python3
"""Kernel micro-benchmarks (HIP events, same stream) for the hot kernels at the workload's shapes:
GEMM fast path vs generic path, ViT attention. Prints one JSON object per case."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
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
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    lib = _lib.load()
    for (M, N, Kd) in [(32768, 2304, 768), (32768, 3072, 768), (32768, 768, 3072), (32768, 768, 768),
                       (39200, 2304, 768), (688128, 384, 256), (688128, 256, 128)]:
        A = (torch.rand(M, Kd, generator=g) - 0.5).to(dev, torch.bfloat16)
        W = (torch.rand(N, Kd, generator=g) - 0.5).to(dev, torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {"case": "gemm_nt", "M": M, "N": N, "K": Kd}
        ref = A[-2048:].float() @ W.float().t()
        for fast in (1, 5, 0):
            lib.octsam_gemm_set_fast_path(fast)
            ms = timeit(lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=out))
            out.zero_()
            K.gemm(A, W, M=M, N=N, K=Kd, out=out)
            err = ((out[-2048:].float() - ref).abs().max() / ref.abs().max()).item()
            res[f"v{fast}"] = {"ms": round(ms, 4), "tflops": round(2 * M * N * Kd / ms / 1e9, 1),
                               "err": round(err, 5)}
        lib.octsam_gemm_set_fast_path(1)
        print(json.dumps(res), flush=True)
        del A, W, out
    for side, nseq, heads, hd, dt in [(64, 8, 12, 64, torch.bfloat16), (14, 200, 12, 64, torch.bfloat16),
                                      (64, 8, 16, 80, torch.bfloat16), (14, 200, 16, 80, torch.bfloat16),
                                      (64, 8, 16, 80, torch.float16), (14, 200, 16, 80, torch.float16)]:
        T = side * side
        qkv = torch.randn(nseq, T, 3 * heads * hd, generator=g).to(dev, dt)
        o = torch.empty(nseq, T, heads * hd, device=dev, dtype=dt)
        Rh = torch.randn(2 * side - 1, hd, device=dev) * 0.02
        fl = 4.0 * nseq * heads * T * T * hd
        byts = (qkv.numel() + o.numel()) * 2
        ms = timeit(lambda: K.vit_attention(qkv, o, Rh, Rh, nseq=nseq, side=side, heads=heads))
        print(json.dumps({"case": "vit_attention", "side": side, "nseq": nseq, "heads": heads, "head_dim": hd,
                          "dtype": str(dt).split(".")[-1], "us": round(ms * 1e3, 1),
                          "tflops": round(fl / ms / 1e9, 1), "gbs": round(byts / ms / 1e6, 1)}), flush=True)

if __name__ == "__main__":
    main()
