"""Same-process A/B of stream priorities under the encoder lookahead: variant 0 = both default, 1 = the step
(decoder phases) on a high-priority stream, lookahead at default. Diagnostic only."""
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

print("priority range", torch.cuda.Stream.priority_range(), flush=True)
device = torch.device("cuda", 0)
args = argparse.Namespace(batch=8, prompt="bboxes")
batch = data.to_device_batch(bench.make_batch(args, 0, device, data.make_processor()), device)
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(device)
K = 10
steps = {}
hi = torch.cuda.Stream(device=device, priority=-1)
VARS = [tuple(int(x) for x in v.split(":")) for v in os.environ.get("VARS", "2:0,3:0,3:-1").split(",")]
for sets, eprio in VARS:
    st = FusedTrainStep(model, lr=0.0, topological=True, graphs=True, pipeline=True)
    st.pipeline_sets, st.enc_priority = sets, eprio
    steps[(sets, eprio)] = st
best = {}
for rnd in range(4):
    for prio, st in steps.items():
      with torch.cuda.stream(torch.cuda.default_stream(device)):
        for i in range(4):
            st.step(batch, next_batch=batch if i < 3 else None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            st.step(batch, next_batch=batch if k + 1 < K else None)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / K
        best[prio] = min(best.get(prio, 1e30), ms)
        print(f"round {rnd} sets:priority {prio}: {ms:.3f} ms/step", flush=True)
print(best)
