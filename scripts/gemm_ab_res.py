"""A/B of the in-place fp32 residual epilogue (gemm8 FE 4: the encoder's MLP2 writing the fp32 residual stream):
residual through LDS quarters (default) vs the register form (fast path bit 4096), interleaved rounds in one
process (min of 5 rounds x 20 launches), outputs compared bitwise. proj runs on gemm8 here too (bit 512 turns the
two-workgroup kernel off) to see the epilogue on a K = 768 shape. Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K  # noqa: E402

lib = _lib.load()


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


SHAPES = [("fc2", 32768, 768, 3072, 1), ("proj", 32768, 768, 768, 1), ("proj_gemm8", 32768, 768, 768, 1 | 512),
          ("fc2_vith", 32768, 1280, 5120, 1)]
VAR = {"res_lds": 0, "res_reg": 4096}
g = torch.Generator().manual_seed(0)
for name, M, N, Kd, base_fp in SHAPES:
    A = torch.randn(M, Kd, generator=g).to("cuda", torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to("cuda", torch.bfloat16)
    bias = torch.randn(N, generator=g).cuda()
    base = torch.randn(M, N, generator=g).cuda()
    outs, best = {}, {}
    for _ in range(5):
        for v, bit in VAR.items():
            lib.octsam_gemm_set_fast_path(base_fp | bit)
            o = base.clone()

            def fn(o=o):
                K.gemm(A, W, M=M, N=N, K=Kd, out=o, bias=bias, residual=o)
            us = t(fn)
            o.copy_(base)
            fn()
            outs[v] = o
            best[v] = min(best.get(v, 1e30), us)
    lib.octsam_gemm_set_fast_path(1)
    ref = base + (A.float() @ W.float().t()) + bias
    fl = 2.0 * M * N * Kd
    row = {"name": name, "M": M, "N": N, "K": Kd}
    for v in VAR:
        row[v + "_us"] = round(best[v], 1)
        row[v + "_tf"] = round(fl / best[v] / 1e6, 1)
    row["bit_identical"] = bool(torch.equal(outs["res_lds"], outs["res_reg"]))
    row["max_err_vs_fp32"] = float((outs["res_lds"] - ref).abs().max())
    print(json.dumps(row), flush=True)
    del A, W, base, outs, ref
    torch.cuda.empty_cache()
