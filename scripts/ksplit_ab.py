"""Kernel-level A/B of the last-wave K split (ABI 22) at the encoder's QKV and MLP2 shapes (B = 8, vit-b): min of
rounds x 20 launches with and without the workspace, outputs compared (diagnostics)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import kernels as K  # noqa: E402


def timed(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
ks = K.ksplit_workspace(dev)
shapes = {"qkv": (32768, 2304, 768, False), "fc2": (32768, 768, 3072, True), "fc1": (32768, 3072, 768, False)}
best = {}
outs = {}
for _ in range(4):
    for name, (M, N, Kd, res) in shapes.items():
        A = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
        W = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to(dev, torch.bfloat16)
        b = torch.randn(N, generator=g).to(dev)
        out = torch.zeros(M, N, device=dev, dtype=torch.float32 if res else torch.bfloat16)
        for use in (False, True):
            kw = dict(M=M, N=N, K=Kd, out=out, bias=b, ksplit=ks if use else None)
            if res:
                kw.update(residual=out)
            t = timed(lambda: K.gemm(A, W, **kw))
            best[name, use] = min(best.get((name, use), 1e30), t)
for name in shapes:
    print(json.dumps({"gemm": name, "unsplit_us": round(best[name, False], 1), "ksplit_us": round(best[name, True], 1)}),
          flush=True)
