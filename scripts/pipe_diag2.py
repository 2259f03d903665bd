"""Diagnostic: is the prefetched encoder output (E of step 2, replayed on the encoder stream during step 1) the
same as the encoder output of step 0 (same batch)?"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_pipeline import _batch  # noqa: E402
from dilabhelmholtzoct_amd.model import SamModel  # noqa: E402
from dilabhelmholtzoct_amd.train import FusedTrainStep  # noqa: E402

cuda = torch.device("cuda", 0)
a, b = _batch(cuda, 3), _batch(cuda, 3, epoch=1)
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(cuda)
st = FusedTrainStep(model, topological=True, graphs=True, pipeline=True)
st.step(a, next_batch=b)
torch.cuda.synchronize()
g0 = [g for k, g in st._graphs.items()][0]
emb0, tok0 = g0["st"].emb.clone(), g0["st"].tokens.clone()
saved0 = None
st.step(b, next_batch=a)   # captures set 1, prefetches E(a) into set 0 on the encoder stream
torch.cuda.synchronize()
print("sets", len(st._graphs), "prefetch set0", st._prefetch[0] is g0)
print("emb equal", torch.equal(emb0, g0["st"].emb), "tokens equal", torch.equal(tok0, g0["st"].tokens),
      "maxdiff", (emb0 - g0["st"].emb).abs().max().item(), flush=True)
# run E(a) again on the main stream alone and compare
g0["graphs"][0].replay()
torch.cuda.synchronize()
print("emb (main replay) equal", torch.equal(emb0, g0["st"].emb), flush=True)
