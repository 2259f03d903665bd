"""Same-process A/B of the training step with the encoder lookahead under GEMM fast-path settings.
usage: python scripts/step_ab2.py 1:1 11:1 1:0   (fast_path:pipeline). Min ms/step over alternating rounds."""
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

variants = [tuple(int(x) for x in v.split(":")) for v in sys.argv[1:]] or [(1, 1)]
device = torch.device("cuda", 0)
lib = _lib.load()
args = argparse.Namespace(batch=8, prompt="bboxes")
batch = data.to_device_batch(bench.make_batch(args, 0, device, data.make_processor()), device)
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(device)
# DEC_ATTRS="name=value,..." sets mask-decoder attributes (A/B across processes, e.g. tok_flush_block=0)
for kv in filter(None, os.environ.get("DEC_ATTRS", "").split(",")):
    k, v = kv.split("=")
    setattr(model.mask_decoder, k, bool(int(v)))
K = 10
best = {}
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for fp, pipe in variants:
        lib.octsam_gemm_set_fast_path(fp)
        st = FusedTrainStep(model, lr=0.0, topological=True, graphs=True, pipeline=bool(pipe))
        for kv in filter(None, os.environ.get("STEP_ATTRS", "").split(",")):  # FusedTrainStep attributes, as DEC_ATTRS
            k, v = kv.split("=")
            setattr(st, k, bool(int(v)))
        for i in range(4):
            st.step(batch, next_batch=batch if i < 3 else None)
        st.flush()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            st.step(batch, next_batch=batch if k + 1 < K else None)
        st.flush()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / K
        best[(fp, pipe)] = min(best.get((fp, pipe), 1e30), ms)
        print(f"round {rnd} fast_path {fp} pipeline {pipe}: {ms:.3f} ms/step", flush=True)
        del st
lib.octsam_gemm_set_fast_path(1)
print({f"{k[0]}:{k[1]}": round(v, 3) for k, v in best.items()})
