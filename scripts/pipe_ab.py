"""Same-process A/B: bench.py's default workload (graph replay) with and without the encoder lookahead
(FusedTrainStep(pipeline=True)); every timed run does exactly its K encoders (the last step passes no
next batch). Min ms/step per variant over alternating rounds. Diagnostic only."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dilabhelmholtzoct_amd import data  # noqa: E402
from dilabhelmholtzoct_amd.model import SamModel  # noqa: E402
from dilabhelmholtzoct_amd.train import FusedTrainStep  # noqa: E402

device = torch.device("cuda", 0)
args = argparse.Namespace(batch=int(os.environ.get("B", "8")), prompt="bboxes")
batch = data.to_device_batch(bench.make_batch(args, 0, device, data.make_processor()), device)
model = SamModel.from_pretrained(os.environ.get("MODEL", "facebook/sam-vit-base"), seed=0).to(device)
K = 10
steps = {p: FusedTrainStep(model, lr=0.0, topological=True, graphs=True, pipeline=p) for p in (False, True)}
best = {}
for rnd in range(3):
    for p, st in steps.items():
        for _ in range(3):
            st.step(batch, next_batch=batch)
        st.step(batch)
        st.flush()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            st.step(batch, next_batch=batch if k + 1 < K else None)
        st.flush()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / K
        best[p] = min(best.get(p, 1e30), ms)
        print(f"round {rnd} pipeline={p}: {ms:.3f} ms/step ({8000 / ms:.1f} imgs/s)", flush=True)
print({str(p): round(v, 3) for p, v in best.items()})
