#!/usr/bin/env python3
"""Cubical-PH kernel latency vs map count and content (diagnostic)."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dilabhelmholtzoct_amd import kernels
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    noise = torch.randn(256, 1, 64, 64, generator=g)
    smooth = torch.sigmoid(F.interpolate(torch.randn(256, 1, 8, 8, generator=g) * 3, size=(50, 50), mode="bilinear",
                                         align_corners=True)).squeeze(1)
    rough = torch.sigmoid(F.interpolate(noise, size=(50, 50), mode="bilinear", align_corners=True) * 3).squeeze(1)
    binary = (smooth > 0.5).float()
    for name, maps in (("smooth", smooth), ("rough", rough), ("binary", binary)):
        for n in (1, 16, 256):
            x = maps[:n].contiguous().to(dev)
            kernels.cubical_ph(x)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                out = kernels.cubical_ph(x)
            e.record()
            torch.cuda.synchronize()
            cnt = out[3].cpu()
            print(f"{name:7s} n={n:4d}: {s.elapsed_time(e) / 5 * 1e3:8.1f} us/launch; pairs H0 mean {cnt[:, 0].float().mean():.0f}"
                  f" H1 mean {cnt[:, 1].float().mean():.0f}")


if __name__ == "__main__":
    main()
