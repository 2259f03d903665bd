"""Layout diagnostics for octsam_wgrad on structured inputs (one-hot rows of X pick one row of dY). Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import kernels as K  # noqa: E402

dev = "cuda"
for M, O, I in [(32, 128, 128), (96, 256, 128)]:
    mi = torch.arange(M, device=dev).view(M, 1).float()
    oi = torch.arange(O, device=dev).view(1, O).float()
    for name, dy in (("dy=o", oi.expand(M, O)), ("dy=m", mi.expand(M, O)), ("dy=(m%8)*16+o%16", (mi % 8) * 16 + oi % 16)):
        dyb = dy.contiguous().to(torch.bfloat16)
        for m0 in (0, 1, 5, 17):
            x = torch.zeros(M, I, device=dev)
            x[m0, :] = 1.0
            xb = x.to(torch.bfloat16)
            out = torch.zeros(O, I, device=dev)
            K.wgrad(dyb, xb, M, out)
            ref = dyb.float().t() @ xb.float()
            bad = (out != ref).nonzero()
            print(M, O, I, name, "m0", m0, "bad", bad.shape[0], "out[:6,0]", out[:6, 0].tolist(), "ref", ref[:6, 0].tolist(),
                  "out[0,:4]", out[0, :4].tolist(), flush=True)
