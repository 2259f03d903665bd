"""Same-process A/B of the fused training step (bench.py's default workload, hipGraph replay) under GEMM fast-path
settings: every variant re-captures its graphs, variants alternate over rounds, min ms/step per variant.
Devices differ by several percent, so step changes are compared here, inside one process. Diagnostic only.
usage: python scripts/step_ab.py 1 513   (octsam_gemm_set_fast_path values)"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dilabhelmholtzoct_amd import _lib, data  # noqa: E402
from dilabhelmholtzoct_amd.model import SamModel  # noqa: E402
from dilabhelmholtzoct_amd.train import FusedTrainStep  # noqa: E402

variants = [int(v) for v in sys.argv[1:]] or [1]
device = torch.device("cuda", 0)
lib = _lib.load()
args = argparse.Namespace(batch=8, prompt="bboxes")
batch = data.to_device_batch(bench.make_batch(args, 0, device, data.make_processor()), device)
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(device)
best = {v: 1e30 for v in variants}
for rnd in range(3):
    for v in variants:
        lib.octsam_gemm_set_fast_path(v)
        st = FusedTrainStep(model, lr=0.0, topological=True, graphs=True)
        for _ in range(3):
            st.step(batch)
        st.flush()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            st.step(batch)
        st.flush()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 100.0
        best[v] = min(best[v], ms)
        print(f"round {rnd} fast_path {v}: {ms:.3f} ms/step", flush=True)
        del st
lib.octsam_gemm_set_fast_path(1)
print({v: round(ms, 3) for v, ms in best.items()})
