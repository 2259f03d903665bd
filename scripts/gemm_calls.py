#!/usr/bin/env python3
"""Every octsam_gemm call of one eager training step (bench batch) with its shape, epilogue and HIP-event
time, sorted by time: where the GEMM family's time goes (diagnostic)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from dilabhelmholtzoct_amd import data, kernels
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(batch=8, prompt="bboxes")
    b = data.to_device_batch(bench.make_batch(args, 0, dev, data.make_processor()), dev)
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    step = FusedTrainStep(model, lr=1e-3, topological=True, graphs=False)
    for _ in range(2):
        step.step(b)
    step.flush()
    torch.cuda.synchronize()
    calls = []
    orig = kernels.gemm

    def wrapped(*a, **k):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = orig(*a, **k)
        e.record()
        out = k.get("out")
        calls.append((s, e, k.get("M"), k.get("N"), k.get("K"), k.get("batch", 1), k.get("a_mode", 0),
                      k.get("b_mode", 0), str(out.dtype).replace("torch.", "") if out is not None else "?",
                      k.get("residual") is not None, k.get("act", 0), k.get("beta", 0.0)))
        return r
    kernels.gemm = wrapped
    import dilabhelmholtzoct_amd.model as mm
    import dilabhelmholtzoct_amd.decoder as dm
    for mod in (mm, dm):
        if hasattr(mod, "K"):
            mod.K.gemm = wrapped
    step.step(b)
    step.flush()
    torch.cuda.synchronize()
    rows = []
    for s, e, M, N, Kk, bt, am, bm, dt, res, act, beta in calls:
        us = s.elapsed_time(e) * 1e3
        fl = 2.0 * M * N * Kk * bt
        rows.append((us, M, N, Kk, bt, am, bm, dt, res, act, beta, fl / us / 1e6))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    print(f"{len(rows)} gemm calls, {tot:.0f} us")
    for r in rows[:int(os.environ.get("TOP", "40"))]:
        print(f"{r[0]:8.1f} us  M={r[1]:7d} N={r[2]:5d} K={r[3]:6d} b={r[4]:3d} am={r[5]} bm={r[6]} out={r[7]:8s} "
              f"res={int(r[8])} act={r[9]} beta={r[10]} {r[11]:6.0f} TF/s")


if __name__ == "__main__":
    main()
