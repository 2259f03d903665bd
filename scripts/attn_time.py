"""ViT attention launch times at the workload shapes (min over 3 rounds of 20 launches; diagnostic)."""
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
cases = [(64, 8, 12, 64, torch.bfloat16), (14, 200, 12, 64, torch.bfloat16), (64, 8, 16, 80, torch.float16),
         (14, 200, 16, 80, torch.float16)]
data = []
for side, nseq, heads, hd, dt in cases:
    # windowed layers as the encoder runs them: token-ordered qkv of 8 images (64 x 64 tokens) + the pad row
    tokens = nseq * side * side if side == 64 else 8 * 4096
    qkv = torch.randn(tokens, 3 * heads * hd, generator=g).to("cuda", dt)
    o = torch.empty(tokens, heads * hd, device="cuda", dtype=dt)
    pad = torch.randn(3 * heads * hd, generator=g).to("cuda", dt) if side == 14 else None
    Rh = (torch.randn(2 * side - 1, hd, generator=g) * 0.02).cuda()
    data.append((side, nseq, heads, hd, dt, qkv, o, Rh, pad))
best = [1e30] * len(cases)
for _ in range(3):
    for i, (side, nseq, heads, hd, dt, qkv, o, Rh, pad) in enumerate(data):
        kw = dict(grid=64, pad_row=pad) if side == 14 else {}
        best[i] = min(best[i], t(lambda: K.vit_attention(qkv, o, Rh, Rh, nseq=nseq, side=side, heads=heads, **kw)))
for (side, nseq, heads, hd, dt, *_), us in zip(data, best):
    fl = 4.0 * nseq * heads * (side * side) ** 2 * hd
    print(json.dumps({"side": side, "nseq": nseq, "heads": heads, "hd": hd, "dtype": str(dt)[6:], "us": round(us, 1),
                      "tflops": round(fl / us / 1e6, 1)}), flush=True)
