"""Token-side (small-problem) GEMMs: device time per launch of the one-shot K <= 256 kernel (gemm_small_kernel,
default) against the chained 64x64 kernel (fast path bit 65536), 50 launches replayed in one hipGraph (no host launch
cost), min of 5 replays; outputs compared bitwise. Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K  # noqa: E402

lib = _lib.load()
VARIANTS = {"oneshot": 1, "chained": 1 | 65536}
# (M, N, K, b_mode, out dtype, act, beta, residual)
SHAPES = [(1176, 256, 256, 0, "f32", 0, 0.0, 0), (1176, 256, 256, 1, "f32", 0, 1.0, 0), (1176, 128, 256, 0, "f32", 0, 0.0, 0),
          (1176, 2048, 256, 0, "bf16", 1, 0.0, 0), (1176, 2048, 256, 1, "f32", 0, 0.0, 0),
          (1176, 256, 128, 0, "f32", 0, 0.0, 1), (1176, 256, 128, 1, "f32", 0, 1.0, 0), (168, 256, 256, 0, "bf16", 1, 0.0, 0),
          (4096, 256, 256, 0, "bf16", 0, 0.0, 0), (1176, 256, 2048, 0, "f32", 0, 0.0, 1)]
g = torch.Generator().manual_seed(0)
for M, N, Kd, bm, od, act, beta, res in SHAPES:
    A = torch.randn(M, Kd, generator=g).to("cuda", torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to("cuda", torch.bfloat16)
    Bop = W if bm == 0 else W.t().contiguous()
    bias = torch.randn(N, generator=g).cuda()
    R = torch.randn(M, N, generator=g).cuda() if res else None
    dt = torch.float32 if od == "f32" else torch.bfloat16
    outs, best = {}, {}
    for v, fp in VARIANTS.items():
        lib.octsam_gemm_set_fast_path(fp)
        out = torch.zeros(M, N, device="cuda", dtype=dt)

        def fn():
            K.gemm(A, Bop, M=M, N=N, K=Kd, out=out, b_mode=bm, bias=bias, act=act, beta=beta, residual=R)
        fn()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(50):
                fn()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 50)
        best[v] = min(ts)
        out.zero_()
        fn()
        torch.cuda.synchronize()
        outs[v] = out.clone()
        del gr
    lib.octsam_gemm_set_fast_path(1)
    print(json.dumps({"M": M, "N": N, "K": Kd, "b_mode": bm, "out": od, "act": act, "beta": beta, "res": res,
                      **{f"{v}_us": round(best[v], 2) for v in VARIANTS},
                      "bit_identical": bool(torch.equal(outs["oneshot"], outs["chained"]))}), flush=True)
