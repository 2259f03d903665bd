#!/usr/bin/env python3
"""Per-shape GEMM timing of one eager training step (diagnostic): every kernels.gemm call is bracketed by HIP
events; calls are grouped by (M, N, K, batch, a_mode, b_mode, path) and sorted by total time."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dilabhelmholtzoct_amd import _lib, data, kernels
    import dilabhelmholtzoct_amd.decoder as dmod
    import dilabhelmholtzoct_amd.model as mmod
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep

    dev = torch.device("cuda", 0)
    B = int(os.environ.get("B", "8"))
    sd = data.SAMDataset(data.synthetic_oct(seed=0, n=B), {"prompt_type": "bboxes"}, epoch_seed=0)
    batch = data.to_device_batch(data.process_batch(data.make_processor(), data.custom_collate([sd[i] for i in range(B)]),
                                                    "bboxes"), dev)
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    step = FusedTrainStep(model, topological=True)
    for _ in range(2):
        step.step(batch)
    torch.cuda.synchronize()
    lib = _lib.load()
    orig = kernels.gemm
    rec = []

    def wrapped(A, B_, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig(A, B_, **kw)
        e.record()
        rec.append(((kw["M"], kw["N"], kw["K"], kw.get("batch", 1), kw.get("a_mode", 0), kw.get("b_mode", 0),
                     lib.octsam_gemm_last_path(), kw.get("residual") is not None, out.dtype == torch.float32), s, e))
        return out

    kernels.gemm = mmod.K.gemm = dmod.K.gemm = wrapped
    step.step(batch)
    torch.cuda.synchronize()
    kernels.gemm = mmod.K.gemm = dmod.K.gemm = orig
    agg = collections.defaultdict(list)
    for key, s, e in rec:
        agg[key].append(s.elapsed_time(e) * 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{len(rec)} GEMM calls, {tot / 1e3:.2f} ms")
    print("   total_us  n    avg_us  TF/s   M       N     K     bat am bm path res f32")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        M, N, K, b = k[:4]
        tf = 2.0 * M * N * K * b * len(v) / (sum(v) * 1e-6) / 1e12
        print(f"{sum(v):10.1f} {len(v):3d} {sum(v) / len(v):8.1f} {tf:6.0f}  {M:7d} {N:5d} {K:5d} {b:4d} {k[4]:2d} {k[5]:2d} "
              f"{k[6]:3d} {int(k[7]):3d} {int(k[8]):3d}")


if __name__ == "__main__":
    main()
