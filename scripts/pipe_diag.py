"""Diagnostic: per-step losses of the plain graph step vs the pipelined step (two graph sets), with the
lookahead on and off, to separate set alternation from concurrency."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_pipeline import _batch  # noqa: E402
from dilabhelmholtzoct_amd.model import SamModel  # noqa: E402
from dilabhelmholtzoct_amd.train import FusedTrainStep  # noqa: E402

cuda = torch.device("cuda", 0)
a, b = _batch(cuda, 3), _batch(cuda, 3, epoch=1)
seq = [a, b, a, a, b, b, a]
hints = seq[1:] + [None]


def run(pipeline, look):
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(cuda)
    st = FusedTrainStep(model, topological=True, graphs=True, pipeline=pipeline)
    out = []
    for i, x in enumerate(seq):
        out.append(st.step(x, next_batch=hints[i] if look else None).clone())
        torch.cuda.synchronize()
        out[-1] = (out[-1], model.mask_decoder.flat_grad.detach().clone(), model.mask_decoder.flat.detach().clone())
    return out


ref = run(False, False)
for name, p, lk in (("two sets, no lookahead", True, False), ("lookahead", True, True)):
    got = run(p, lk)
    for i, (r, g) in enumerate(zip(ref, got)):
        print(name, "step", i, "loss eq", torch.equal(r[0], g[0]), "grad eq", torch.equal(r[1], g[1]),
              "param eq", torch.equal(r[2], g[2]), "loss diff", (r[0] - g[0]).abs().max().item(),
              "grad maxdiff", (r[1] - g[1]).abs().max().item(), flush=True)
