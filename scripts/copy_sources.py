"""Diagnostic: which torch-level copies / fills / elementwise launches the eager training step issues, with the
Python line that issued each (torch.profiler, CPU stacks). The graph-replayed step runs the same launches."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    sys.argv = ["bench.py"]
    args = bench.parse()
    device = torch.device("cuda", 0)
    batch = data.to_device_batch(bench.make_batch(args, 0, device, data.make_processor()), device)
    model = SamModel.from_pretrained(args.model, seed=0).to(device)
    step = FusedTrainStep(model, lr=1e-3, topological=True, graphs=False, pipeline=False)
    step.step(batch)
    torch.cuda.synchronize()
    import traceback
    from torch.overrides import TorchFunctionMode
    names = {"copy_", "clone", "contiguous", "to", "zero_", "fill_", "cat", "repeat", "zeros", "zeros_like", "full",
             "t", "float"}
    cnt = collections.Counter()

    class Mode(TorchFunctionMode):
        def __torch_function__(self, func, types, args=(), kwargs=None):
            nm = getattr(func, "__name__", str(func))
            if nm in names:
                fr = [f for f in traceback.extract_stack()[:-1] if "dilabhelmholtzoct_amd" in f.filename]
                where = f"{os.path.basename(fr[-1].filename)}:{fr[-1].lineno} {fr[-1].line}" if fr else "?"
                cnt[(nm, where)] += 1
            return func(*args, **(kwargs or {}))

    with Mode():
        step.step(batch)
    torch.cuda.synchronize()
    for (name, where), n in cnt.most_common(80):
        print(f"{n:4d}  {name:10s} {where[:150]}")


if __name__ == "__main__":
    main()
