"""gemm8 variants on the encoder's GEMM shapes (bf16): the default dispatch (persistent gemm8p for bias /
activation epilogues), the one-tile-per-workgroup kernel (fast path 11), its no-epilogue (DBG 1) and
no-main-loop (DBG 2) builds, and torch.matmul (hipBLASLt) as a yardstick. Diagnostic only."""
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


# (name, M, N, K, act, residual): residual GEMMs write the fp32 residual stream in place, as the encoder does
# (the windowed projection through the window -> token row map)
SHAPES = [("qkv_win", 39200, 2304, 768, 0, 0), ("qkv_glob", 32768, 2304, 768, 0, 0),
          ("proj_win", 39200, 768, 768, 0, 2), ("proj", 32768, 768, 768, 0, 1), ("fc1", 32768, 3072, 768, 2, 0),
          ("fc2", 32768, 768, 3072, 0, 1), ("dec_out", 688128, 256, 128, 0, 3), ("dec_kqv", 688128, 384, 256, 0, 4),
          ("sq8k", 8192, 8192, 8192, 0, 0), ("deep", 32768, 2304, 6144, 0, 0)]
PICK = [x for x in os.environ.get("GEMM_SHAPES", "").split(",") if x]
VPICK = [x for x in os.environ.get("GEMM_VARIANTS", "").split(",") if x]
for name, M, N, Kd, act, res in SHAPES:
    if PICK and name not in PICK:
        continue
    A = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    W = (torch.randn(N, Kd, device="cuda") / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    Mo = 32768 if res == 2 else M
    out = torch.randn(Mo, N, device="cuda") if res in (1, 2) else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    R = out if res in (1, 2) else None
    rr = (0, 1)
    if res == 3:  # decoder: e16 residual stream (keys)
        R = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    if res == 4:  # decoder: per-prompt broadcast of the PE projection (4096 rows)
        R = torch.randn(4096, N, device="cuda").to(torch.bfloat16)
        rr = (4096, M // 4096)
    rm = None
    if res == 2:
        rm = torch.full((M,), -1, dtype=torch.int32)
        rm[torch.randperm(M)[:Mo]] = torch.arange(Mo, dtype=torch.int32)
        rm = rm.cuda()
    f = 2.0 * M * N * Kd
    ob = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    row = {"name": name, "M": M, "N": N, "K": Kd}
    variants = [("default", 1), ("single", 11), ("relax", 13), ("p1tile", 14), ("p_nostore", 16), ("p_tile0", 17),
                ("general", 18), ("nopersist", 20), ("no192", 21), ("noepi", 6), ("noloop", 7), ("blaslt", None)]
    if VPICK:
        variants = [v for v in variants if v[0] in VPICK]
    best = {}
    for rnd in range(3):  # round-robin, min over rounds: no variant always runs first after a clock ramp
        for tag, fast in variants:
            if fast is None:
                us = t(lambda: torch.matmul(A, W.t(), out=ob))
            else:
                lib.octsam_gemm_set_fast_path(fast)
                us = t(lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=out, bias=bias, act=act, residual=R, row_map=rm, r_remap=rr))
            best[tag] = min(best.get(tag, 1e30), us)
    lib.octsam_gemm_set_fast_path(1)
    for tag, us in best.items():
        row[tag + "_us"] = round(us, 1)
        row[tag + "_tf"] = round(f / us / 1e6)
    print(json.dumps(row), flush=True)
