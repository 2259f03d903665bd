"""Timing of the decoder's image-side weight gradients (out[O, I] = dY[R, O]^T X[R, I] over R = P*4096 rows, k-major
operands) at the bench workload: the split-K LDS-DMA kernel (gemm_glds_kernel) at several split counts, with and
without the fused bias column sums, plus the split-K reduction, the whole-output-per-workgroup kernel (octsam_wgrad),
and torch.mm (hipBLASLt) of the same product. Min of 5 rounds x 10 launches, HIP events. Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import kernels as K  # noqa: E402

ROWS = int(os.environ.get("DW_ROWS", 688128))
SHAPES = [("kqv_pe", 384, 256), ("i2t_out", 256, 128), ("kv_final", 256, 256)]


def t(fn, it=10):
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
for name, O, I in SHAPES:
    dy = torch.randn(ROWS, O, generator=g).to("cuda", torch.bfloat16)
    x = torch.randn(ROWS, I, generator=g).to("cuda", torch.bfloat16)
    out = torch.empty(O, I, device="cuda")
    db = torch.empty(O, device="cuda")
    fns = {}
    for split in (32, 64, 128, 256):
        ks = ROWS // split
        if ks % 64 or split * (-(-O // 256)) * (-(-I // 128)) < 64:
            continue
        part = torch.empty(split, O, I, device="cuda")
        pa = torch.empty(split, O, device="cuda")

        def gemm_only(split=split, ks=ks, part=part):
            K.gemm(dy, x, M=O, N=I, K=ks, out=part, a_mode=1, b_mode=1, lda=O, ldb=I, batch=split,
                   stride_a=ks * O, stride_b=ks * I, stride_c=O * I)

        def full(split=split, ks=ks, part=part, pa=pa):
            K.gemm(dy, x, M=O, N=I, K=ks, out=part, a_mode=1, b_mode=1, lda=O, ldb=I, batch=split,
                   stride_a=ks * O, stride_b=ks * I, stride_c=O * I, a_colsum=pa)
            K.splitk_reduce(part.view(split, -1), out, split)
            K.splitk_reduce(pa, db, split)
        fns[f"s{split}_gemm"] = gemm_only
        fns[f"s{split}_full"] = full
    fns["wgrad_full"] = lambda: K.wgrad(dy, x, ROWS, out, db=db)
    fns["wgrad_nocs"] = lambda: K.wgrad(dy, x, ROWS, out)
    fns["torch_mm_bf16"] = lambda: torch.mm(dy.t(), x)
    best = {}
    for _ in range(5):
        for k, fn in fns.items():
            best[k] = min(best.get(k, 1e30), t(fn))
    byt = ROWS * (O + I) * 2
    row = {"name": name, "O": O, "I": I, "rows": ROWS, "compulsory_MB": round(byt / 1e6, 1)}
    for k, v in best.items():
        row[k] = round(v, 1)
    row["best_splitk_TBps"] = round(byt / min(v for k, v in best.items() if k.startswith("s")) / 1e6, 2)
    row["wgrad_TBps"] = round(byt / best["wgrad_full"] / 1e6, 2)
    ref = dy.float().t() @ x.float()
    K.wgrad(dy, x, ROWS, out, db=db)
    row["wgrad_rel_err"] = float((out - ref).abs().max() / ref.abs().max())
    print(json.dumps(row), flush=True)
    del dy, x, fns
    torch.cuda.empty_cache()
