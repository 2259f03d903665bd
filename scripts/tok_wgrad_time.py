"""Token-side weight-gradient launches timed alone (device time per launch from 20 replays in one hipGraph): one
problem at a time and the decoder block's group (M = 1176 rows: MLP lin1 / lin2, the attention projections).
Diagnostic only; OCTSAM_LIB selects another build."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import kernels as K  # noqa: E402

g = torch.Generator().manual_seed(0)
M = 1176
SHAPES = {"lin1": (2048, 256), "lin2": (256, 2048), "proj256": (256, 256), "q128": (128, 256), "o128": (256, 128)}
probs = {}
for name, (O, I) in SHAPES.items():
    dy = (torch.randn(M, O, generator=g) * 0.1).to("cuda", torch.bfloat16)
    x = torch.randn(M, I, generator=g).to("cuda", torch.bfloat16)
    out = torch.zeros(O, I, device="cuda")
    db = torch.zeros(O, device="cuda")
    probs[name] = (dy, x, M, out, None, None, 0.0, db)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return round(best, 2)


row = {}
for name, p in probs.items():
    row[name] = timed(lambda p=p: K.wgrad_tok_group([p]))
row["block_group"] = timed(lambda: K.wgrad_tok_group([probs[k] for k in SHAPES] + [probs["proj256"]] * 0))
print(json.dumps(row), flush=True)
