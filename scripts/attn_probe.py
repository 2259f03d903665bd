#!/usr/bin/env python3
"""ViT attention kernel alone, launched repeatedly (rocprofv3 --pmc / timing; diagnostic).
usage: attn_probe.py side(64|14) [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dilabhelmholtzoct_amd import kernels
    side = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    heads, B = 12, 8
    nseq = B if side == 64 else B * 25
    T = side * side
    qkv = (torch.randn(nseq * T, 3 * heads * 64, device=dev) * 0.5).to(torch.bfloat16)
    out = torch.empty(nseq * T, heads * 64, device=dev, dtype=torch.bfloat16)
    rh = torch.randn(2 * side - 1, 64, device=dev) * 0.1
    rw = torch.randn(2 * side - 1, 64, device=dev) * 0.1
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(reps + 2):
        if i == 2:
            s.record()
        kernels.vit_attention(qkv, out, rh, rw, nseq=nseq, side=side, heads=heads)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / reps
    fl = 4.0 * T * T * 64 * heads * nseq
    print(f"side={side}: {us:.1f} us/launch, {fl / us / 1e6:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
