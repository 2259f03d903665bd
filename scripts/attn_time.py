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
    T = side * side
    qkv = torch.randn(nseq, T, 3 * heads * hd, generator=g).to("cuda", dt)
    o = torch.empty(nseq, T, heads * hd, device="cuda", dtype=dt)
    Rh = (torch.randn(2 * side - 1, hd, generator=g) * 0.02).cuda()
    data.append((side, nseq, heads, hd, dt, qkv, o, Rh))
best = [1e30] * len(cases)
for _ in range(3):
    for i, (side, nseq, heads, hd, dt, qkv, o, Rh) in enumerate(data):
        best[i] = min(best[i], t(lambda: K.vit_attention(qkv, o, Rh, Rh, nseq=nseq, side=side, heads=heads)))
for (side, nseq, heads, hd, dt, *_), us in zip(data, best):
    fl = 4.0 * nseq * heads * (side * side) ** 2 * hd
    print(json.dumps({"side": side, "nseq": nseq, "heads": heads, "hd": hd, "dtype": str(dt)[6:], "us": round(us, 1),
                      "tflops": round(fl / us / 1e6, 1)}), flush=True)
