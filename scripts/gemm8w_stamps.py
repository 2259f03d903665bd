"""Phase timing of the ping-pong GEMM (gemm8w) against the 8-phase kernel (diagnostics): fast path 9 runs the
stamped kernels (octsam_gemm_debug_stamps: entry, main loop done, epilogue stores done; gemm8w: both wave rows'
loop ends). Prints per shape the median cycles of prologue+main loop and epilogue per tile and the spread of the
workgroups' start times (how many waves of tiles). Diagnostic only."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K  # noqa: E402

lib = _lib.load()
SHAPES = [("qkv", 32768, 2304, 768, 0, 0), ("fc1", 32768, 3072, 768, 2, 0), ("fc2", 32768, 768, 3072, 0, 1)]


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


for name, M, N, Kd, act, res in SHAPES:
    A = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    W = (torch.randn(N, Kd, device="cuda") / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    out = torch.randn(M, N, device="cuda") if res else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    R = out if res else None
    run = lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=out, bias=bias, act=act, residual=R)  # noqa: E731
    nwg = ((M + 255) // 256) * ((N + 255) // 256)
    for kname, fast_plain, fast_st in (("gemm8", 1 | 8192, 9 | 8192), ("gemm8w", 1, 9)):
        lib.octsam_gemm_set_fast_path(fast_plain)
        us = t(run)
        lib.octsam_gemm_set_fast_path(fast_st)
        us_st = t(run)
        run()
        torch.cuda.synchronize()
        buf = np.zeros(nwg * 4, dtype=np.int64)
        assert lib.octsam_gemm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), nwg) == 0
        st = buf.reshape(nwg, 4)
        t0 = st[:, 0]
        if kname == "gemm8":
            loop_end, t2 = st[:, 1], st[:, 2]
            loop_end0 = loop_end
        else:
            loop_end0, loop_end, t2 = st[:, 1], st[:, 2], st[:, 3]
        rel0 = (t0 - t0.min())
        span = int(t2.max() - t0.min())
        row = {"shape": name, "kernel": kname, "us": round(us, 1), "us_stamped": round(us_st, 1),
               "span_cycles": span, "clock_ghz_est": round(span / (us_st * 1e3), 3),
               "loop_cycles_med": int(np.median(loop_end - t0)), "loop0_cycles_med": int(np.median(loop_end0 - t0)),
               "epi_cycles_med": int(np.median(t2 - loop_end)),
               "tile_cycles_med": int(np.median(t2 - t0)),
               "start_quantiles": [int(np.quantile(rel0, q)) for q in (0.1, 0.5, 0.66, 0.9, 1.0)]}
        print(json.dumps(row), flush=True)
    lib.octsam_gemm_set_fast_path(1)
    del A, W, out
    torch.cuda.empty_cache()
