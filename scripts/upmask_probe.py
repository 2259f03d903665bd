#!/usr/bin/env python3
"""Fused upscaling tail timing at the bench size (diagnostic): octsam_upmask_fwd / _bwd for P prompts over
persistent-grid variants. usage: upmask_probe.py [P] [ntok]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dilabhelmholtzoct_amd import _lib, kernels
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 168
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    dev = torch.device("cuda", 0)
    up1 = torch.randn(P * 16384, 64, device=dev).to(torch.bfloat16)
    w2 = (0.15 * torch.randn(64, 128, device=dev)).to(torch.bfloat16)
    b2 = 0.2 * torch.randn(32, device=dev)
    hyper = torch.randn(P, ns, 32, device=dev)
    dmask = torch.randn(P, ns, 256, 256, device=dev)
    masks = torch.empty(P, ns, 256, 256, device=dev)
    dup1 = torch.empty_like(up1)
    dw2, db2, dh = torch.empty(64, 128, device=dev), torch.empty(32, device=dev), torch.empty(P, ns, 32, device=dev)
    lib = _lib.load()
    fb = up1.numel() * 2 + masks.numel() * 4
    bb = up1.numel() * 4 + dmask.numel() * 4
    for fg, bg in ((512, 512), (768, 256), (1024, 384), (2048, 512), (P * 128, 512)):
        lib.octsam_upmask_set_grid(fg, bg)
        res = []
        for fn in (lambda: kernels.upmask_fwd(up1, w2, b2, hyper, P, ns, masks),
                   lambda: kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, dup1, dw2, db2, dh)):
            for _ in range(2):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                fn()
            e.record()
            torch.cuda.synchronize()
            res.append(s.elapsed_time(e) * 1e3 / 5)
        print(f"grid fwd {fg:6d} bwd {bg:4d}: fwd {res[0]:7.1f} us ({fb / res[0] / 1e3:5.0f} GB/s)  "
              f"bwd {res[1]:7.1f} us ({bb / res[1] / 1e3:5.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
