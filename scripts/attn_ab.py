"""A/B of the ViT attention kernel variants (octsam_attention_set_variant) at the workload shapes: interleaved
rounds in one process (min of 5 rounds x 20 launches), outputs compared bitwise. Diagnostic only."""
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


VARIANTS = [int(v) for v in os.environ.get("ATTN_VARIANTS", "1,0").split(",")]
g = torch.Generator().manual_seed(0)
cases = [(64, 8, 12, 64, torch.bfloat16), (14, 200, 12, 64, torch.bfloat16), (64, 8, 16, 80, torch.float16),
         (14, 200, 16, 80, torch.float16)]
data = []
for side, nseq, heads, hd, dt in cases:
    tokens = nseq * side * side if side == 64 else 8 * 4096
    qkv = torch.randn(tokens, 3 * heads * hd, generator=g).to("cuda", dt)
    pad = torch.randn(3 * heads * hd, generator=g).to("cuda", dt) if side == 14 else None
    Rh = (torch.randn(2 * side - 1, hd, generator=g) * 0.02).cuda()
    outs = {v: torch.empty(tokens, heads * hd, device="cuda", dtype=dt) for v in VARIANTS}
    data.append((side, nseq, heads, hd, dt, qkv, outs, Rh, pad))
best = {(i, v): 1e30 for i in range(len(cases)) for v in VARIANTS}
for _ in range(5):
    for i, (side, nseq, heads, hd, dt, qkv, outs, Rh, pad) in enumerate(data):
        kw = dict(grid=64, pad_row=pad) if side == 14 else {}
        for v in VARIANTS:
            lib.octsam_attention_set_variant(v)
            best[i, v] = min(best[i, v], t(lambda: K.vit_attention(qkv, outs[v], Rh, Rh, nseq=nseq, side=side,
                                                                      heads=heads, **kw)))
lib.octsam_attention_set_variant(0)
for i, (side, nseq, heads, hd, dt, qkv, outs, *_) in enumerate(data):
    fl = 4.0 * nseq * heads * (side * side) ** 2 * hd
    ref = outs[VARIANTS[0]]
    row = {"side": side, "heads": heads, "hd": hd, "dtype": str(dt)[6:]}
    for v in VARIANTS:
        row[f"v{v}_us"] = round(best[i, v], 1)
        row[f"v{v}_tf"] = round(fl / best[i, v] / 1e6, 1)
        row[f"v{v}_same"] = bool(torch.equal(outs[v], ref))
        row[f"v{v}_rel"] = float((outs[v].float() - ref.float()).norm() / ref.float().norm())
    print(json.dumps(row), flush=True)
