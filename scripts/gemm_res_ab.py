"""A/B of the decoder's per-prompt image-side GEMMs (P = 168 prompts x 4096 rows, e16 output + e16 residual):
the two-workgroups-per-CU 256x128 kernel (gemm4w, fast path 1) against the 8-phase 256x256 kernels (fast path
1 | 1024: persistent gemm8p for the row-remapped broadcast addend, gemm8 for the plain residual), each with the
broadcast-residual tile order (rgroup_tm) and without it (| 2048). Interleaved rounds
in one process (min of 5 x 10 launches), outputs compared bitwise. Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K  # noqa: E402

lib = _lib.load()
VARIANTS = {"gemm4w": 1, "gemm8": 1 | 1024, "gemm4w_plain_order": 1 | 2048, "gemm8_plain_order": 1 | 1024 | 2048}
L, P = 4096, 168
M = L * P


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


# (name, N, K, remapped broadcast residual)
SHAPES = [("kqv_layer1", 384, 256, True), ("kv_final", 256, 256, True), ("dkeys_layer1", 256, 384, False),
          ("dkeys_final", 256, 256, False)]
g = torch.Generator().manual_seed(0)
for name, N, Kd, remap in SHAPES:
    A = torch.randn(M, Kd, generator=g).to("cuda", torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to("cuda", torch.bfloat16)
    R = (torch.randn(L, N, generator=g) if remap else torch.randn(M, N, generator=g)).to("cuda", torch.bfloat16)
    outs, best = {}, {}
    for _ in range(5):
        for v, fp in VARIANTS.items():
            lib.octsam_gemm_set_fast_path(fp)
            o = outs.setdefault(v, torch.empty(M, N, device="cuda", dtype=torch.bfloat16))
            kw = dict(residual=R, ldr=N, r_remap=(L, P)) if remap else dict(residual=R)
            fn = lambda o=o, kw=kw: K.gemm(A, W, M=M, N=N, K=Kd, out=o, **kw)  # noqa: E731
            best[v] = min(best.get(v, 1e30), t(fn))
            best[v + "_path"] = int(lib.octsam_gemm_last_path())
    lib.octsam_gemm_set_fast_path(1)
    ref = (A.float() @ W.float().t() + (R.float().repeat(P, 1) if remap else R.float()))
    row = {"name": name, "M": M, "N": N, "K": Kd, "gflop": round(2 * M * N * Kd / 1e9, 1)}
    for v in VARIANTS:
        row[v + "_us"] = round(best[v], 1)
        row[v + "_tf"] = round(2 * M * N * Kd / best[v] / 1e6, 1)
        row[v + "_rel"] = float((outs[v].float() - ref).norm() / ref.norm())
    row["same"] = all(torch.equal(outs["gemm4w"], o) for o in outs.values())
    print(json.dumps(row), flush=True)
