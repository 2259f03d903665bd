"""A/B of the encoder GEMM kernels at the workload shapes (B = 8 images): the two-workgroups-per-CU 256x128
kernel (gemm4w, fast path 1) against the one-workgroup 256x256 8-phase kernel (fast path 1 | 512), interleaved
rounds in one process (min of 5 rounds x 20 launches), outputs compared bitwise (the two accumulate the same K
chunks in the same order). Residual GEMMs update a copy of the same fp32 stream per variant. Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K  # noqa: E402

lib = _lib.load()
VARIANTS = {"gemm4w": 1, "gemm8": 1 | 512}


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


# (name, M, N, K, act, residual)
SHAPES = [("qkv", 32768, 2304, 768, 0, 0), ("proj", 32768, 768, 768, 0, 1), ("fc1", 32768, 3072, 768, 2, 0),
          ("fc2", 32768, 768, 3072, 0, 1), ("dec_up1", 688128, 256, 256, 0, 0)]
g = torch.Generator().manual_seed(0)
rows = []
for name, M, N, Kd, act, res in SHAPES:
    A = torch.randn(M, Kd, generator=g).to("cuda", torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to("cuda", torch.bfloat16)
    bias = torch.randn(N, generator=g).cuda()
    base = torch.randn(M, N, generator=g).cuda() if res else None
    outs = {}
    best = {}
    for _ in range(5):
        for v, fp in VARIANTS.items():
            lib.octsam_gemm_set_fast_path(fp)
            if res:
                o = base.clone()

                def fn(o=o):
                    K.gemm(A, W, M=M, N=N, K=Kd, out=o, bias=bias, residual=o)
                us = t(fn)
                o.copy_(base)
                fn()  # one application for the bitwise comparison
            else:
                o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

                def fn(o=o):
                    K.gemm(A, W, M=M, N=N, K=Kd, out=o, bias=bias, act=act)
                us = t(fn)
            outs[v] = o
            best[v] = min(best.get(v, 1e30), us)
    lib.octsam_gemm_set_fast_path(1)
    fl = 2.0 * M * N * Kd
    row = {"name": name, "M": M, "N": N, "K": Kd}
    for v in VARIANTS:
        row[v + "_us"] = round(best[v], 1)
        row[v + "_tf"] = round(fl / best[v] / 1e6, 1)
    row["bit_identical"] = bool(torch.equal(outs["gemm4w"], outs["gemm8"]))
    print(json.dumps(row), flush=True)
    del A, W, base, outs
    torch.cuda.empty_cache()
