"""Encoder residual GEMMs (proj, fc2 at B = 8) with the fp32 in-place residual epilogue vs a plain bf16 output (the
residual add moved elsewhere), and the LayerNorm pass, on the default kernel choice. Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import kernels as K  # noqa: E402


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


g = torch.Generator().manual_seed(0)
M, D = 32768, 768
x = torch.randn(M, D, generator=g).cuda()
for name, Kd in (("proj", 768), ("fc2", 3072)):
    A = torch.randn(M, Kd, generator=g).to("cuda", torch.bfloat16)
    W = (torch.randn(D, Kd, generator=g) / Kd ** 0.5).to("cuda", torch.bfloat16)
    bias = torch.randn(D, generator=g).cuda()
    o16 = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
    best = {}
    for _ in range(5):
        a = t(lambda: K.gemm(A, W, M=M, N=D, K=Kd, out=x, bias=bias, residual=x))
        b = t(lambda: K.gemm(A, W, M=M, N=D, K=Kd, out=o16, bias=bias))
        best["fp32_res"] = min(best.get("fp32_res", 1e9), a)
        best["bf16_out"] = min(best.get("bf16_out", 1e9), b)
    print(json.dumps({"gemm": name, **{k: round(v, 1) for k, v in best.items()}}), flush=True)
w = torch.ones(D, device="cuda")
bb = torch.zeros(D, device="cuda")
xn = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
print(json.dumps({"ln_fwd_768_us": round(min(t(lambda: K.layernorm_fwd(x, w, bb, 1e-6, xn)) for _ in range(5)), 1)}))
