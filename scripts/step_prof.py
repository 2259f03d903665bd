"""K steps of the bench's training step (B = 8, boxes, --top=True, hipGraphs), sequential (PIPE=0) or with the encoder
lookahead (PIPE=1), nothing else in the process: the program profiled for the per-kernel tables. Diagnostic only."""
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
pipe = os.environ.get("PIPE", "0") == "1"
K = int(os.environ.get("STEPS", "10"))
args = argparse.Namespace(batch=8, prompt="bboxes")
batch = data.to_device_batch(bench.make_batch(args, 0, device, data.make_processor()), device)
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(device)
st = FusedTrainStep(model, lr=1e-3, topological=True, graphs=True, pipeline=pipe)
for i in range(4):
    st.step(batch, next_batch=batch if i < 3 else None)
st.flush()
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(K):
    st.step(batch, next_batch=batch if k + 1 < K else None)
st.flush()
torch.cuda.synchronize()
print(f"pipeline={pipe}: {(time.perf_counter() - t0) * 1e3 / K:.3f} ms/step over {K} steps", flush=True)
