#!/usr/bin/env python3
"""Per-call-site GEMM census of one training step (bench workload): shape, modes, epilogue options,
which kernel ran (octsam_gemm_last_path) and its time (HIP events, synchronised per call). Prints a
table sorted by total time. Diagnostic only."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from dilabhelmholtzoct_amd import _lib, data, kernels
    import dilabhelmholtzoct_amd.decoder as dmod
    import dilabhelmholtzoct_amd.model as mmod
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    ds = data.synthetic_oct(seed=1000, n=8)
    sd = data.SAMDataset(ds, {"prompt_type": "bboxes"}, epoch_seed=0)
    b = data.process_batch(data.make_processor(), data.custom_collate([sd[i] for i in range(8)]), "bboxes")
    bd = data.to_device_batch(b, dev)
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    step = FusedTrainStep(model, topological=True)
    step.step(bd)
    orig = kernels.gemm
    stats = collections.defaultdict(lambda: [0, 0.0])

    def wrapped(A, B, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig(A, B, **kw)
        e.record()
        torch.cuda.synchronize()
        site = [f for f in traceback.extract_stack()[:-1] if "dilabhelmholtzoct_amd" in f.filename][-1]
        key = (f"{os.path.basename(site.filename)}:{site.lineno}", kw["M"], kw["N"], kw["K"], kw.get("batch", 1),
               kw.get("a_mode", 0), kw.get("b_mode", 0), kw["out"].dtype == torch.float32,
               kw.get("beta", 0.0) != 0.0, kw.get("residual") is not None and kw["residual"].dtype == torch.float32,
               kw.get("residual") is not None, kw.get("pre_out") is not None, kw.get("row_map") is not None,
               lib.octsam_gemm_last_path())
        stats[key][0] += 1
        stats[key][1] += s.elapsed_time(e)
        return out

    kernels.gemm = mmod.K.gemm = dmod.K.gemm = wrapped
    step.step(bd)
    kernels.gemm = mmod.K.gemm = dmod.K.gemm = orig
    print("site M N K batch am bm c_f32 beta r_f32 R pre rowmap fast | calls ms TF/s")
    tot = 0.0
    for k, (n, ms) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        tot += ms
        fl = 2.0 * k[1] * k[2] * k[3] * k[4] * n
        print(*k, "|", n, round(ms, 3), round(fl / ms / 1e9, 1))
    print("total gemm ms", round(tot, 3))


if __name__ == "__main__":
    main()
