"""A/B of the ping-pong 8-wave GEMM (gemm8w, the default; fast path bit 8192 = the 8-phase kernel; bit 16384 also for
the shapes gemm4w takes; bit 262144 = the opt-in 256x192 tiles where they fill the waves better)
against the 8-phase / two-workgroup kernels on the encoder and decoder shapes (B = 8 images):
interleaved rounds in one process (min of 5 rounds x 20 launches), outputs compared bitwise against the native
default and in relative error against torch fp32. Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K  # noqa: E402

lib = _lib.load()
VARIANTS = {"native": 1, "n192": 1 | 262144, "gemm8": 1 | 8192, "w4": 1 | 16384,
            # diagnostics of the ping-pong loop (wrong results except dmac): no DMA / no fragment reads / no MFMAs
            "skipdma": 1 | (1 << 20), "skiprd": 1 | (2 << 20), "skipmfma": 1 | (4 << 20), "skipdmard": 1 | (3 << 20),
            "dmac": 1 | (5 << 20), "dmafirst": 1 | (6 << 20)}
if os.environ.get("VARIANTS"):
    VARIANTS = {k: VARIANTS[k] for k in os.environ["VARIANTS"].split(",")}


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
          ("fc2", 32768, 768, 3072, 0, 1), ("fc2e16", 32768, 768, 3072, 0, 0), ("neck1", 32768, 256, 768, 0, 0), ("dec_up1", 688128, 256, 256, 0, 0),
          ("ragged", 5000, 1000, 320, 0, 0), ("ragged_res", 3000, 520, 192, 0, 1)]
if os.environ.get("SHAPES"):
    SHAPES = [s for s in SHAPES if s[0] in os.environ["SHAPES"].split(",")]
g = torch.Generator().manual_seed(0)
for name, M, N, Kd, act, res in SHAPES:
    A = torch.randn(M, Kd, generator=g).to("cuda", torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to("cuda", torch.bfloat16)
    bias = torch.randn(N, generator=g).cuda()
    base = torch.randn(M, N, generator=g).cuda() if res else None
    outs, best, paths = {}, {}, {}
    for _ in range(5):
        for v, fp in VARIANTS.items():
            lib.octsam_gemm_set_fast_path(fp)
            if res:
                o = base.clone()

                def fn(o=o):
                    K.gemm(A, W, M=M, N=N, K=Kd, out=o, bias=bias, residual=o)
                us = t(fn)
                o.copy_(base)
                fn()
            else:
                o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

                def fn(o=o):
                    K.gemm(A, W, M=M, N=N, K=Kd, out=o, bias=bias, act=act)
                us = t(fn)
            torch.cuda.synchronize()
            paths[v] = int(lib.octsam_gemm_last_path())
            outs[v] = o
            best[v] = min(best.get(v, 1e30), us)
    lib.octsam_gemm_set_fast_path(1)
    ref = A.float() @ W.float().t() + bias
    if act == 2:
        ref = torch.nn.functional.gelu(ref)
    if res:
        ref = ref + base
    fl = 2.0 * M * N * Kd
    row = {"name": name, "M": M, "N": N, "K": Kd}
    for v in VARIANTS:
        row[v + "_us"] = round(best[v], 1)
        row[v + "_tf"] = round(fl / best[v] / 1e6, 1)
        row[v + "_path"] = paths[v]
        row[v + "_rel"] = float(f"{((outs[v].float() - ref).norm() / ref.norm()).item():.3g}")
        if "native" in outs:
            row[v + "_bitid"] = bool(torch.equal(outs[v], outs["native"]))
    print(json.dumps(row), flush=True)
    del A, W, base, outs, ref
    torch.cuda.empty_cache()
