import argparse, sys, time, os
sys.path.insert(0, os.getcwd())
import torch, bench
from dilabhelmholtzoct_amd import data
from dilabhelmholtzoct_amd.model import SamModel
from dilabhelmholtzoct_amd.train import FusedTrainStep
dev = torch.device("cuda", 0)
b = data.to_device_batch(bench.make_batch(argparse.Namespace(batch=8, prompt="bboxes"), 0, dev, data.make_processor()), dev)
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
step = FusedTrainStep(model, lr=1e-3, topological=True, graphs=True)
ts = []
orig = step._topo_host
def timed(st, backward):
    t = time.perf_counter(); r = orig(st, backward); ts.append(time.perf_counter() - t); return r
step._topo_host = timed
for _ in range(8): step.step(b)
step.flush(); torch.cuda.synchronize()
print("topo_host us per call:", [round(x * 1e6) for x in ts[-5:]])
st = next(iter(step._graphs.values()))["st"]
print("h1 counts", st.pinned[1].numpy()[:, 1].tolist())
