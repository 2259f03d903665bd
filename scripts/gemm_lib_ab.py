"""Encoder GEMM times (8-phase kernel: fast path 1 | 512) of whichever liboctsam_hip.so build OCTSAM_LIB names, for
a same-box two-build A/B (alternate processes). Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K  # noqa: E402

lib = _lib.load()
lib.octsam_gemm_set_fast_path(1 | 512)


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
row = {"lib": os.path.basename(os.environ.get("OCTSAM_LIB", "default"))}
for name, M, N, Kd, act, res in (("qkv", 32768, 2304, 768, 0, 0), ("proj", 32768, 768, 768, 0, 1),
                                 ("fc1", 32768, 3072, 768, 2, 0), ("fc2", 32768, 768, 3072, 0, 1)):
    A = torch.randn(M, Kd, generator=g).to("cuda", torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to("cuda", torch.bfloat16)
    bias = torch.randn(N, generator=g).cuda()
    if res:
        o = torch.randn(M, N, generator=g).cuda()
        fn = lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=o, bias=bias, residual=o)  # noqa: E731
    else:
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fn = lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=o, bias=bias, act=act)  # noqa: E731
    row[name] = round(min(t(fn) for _ in range(3)), 1)
print(json.dumps(row), flush=True)
