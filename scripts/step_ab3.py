"""Same-process A/B of the pipelined training step (bench.py's loop: hipGraphs + encoder lookahead, B = 8 boxes,
--top=True) for: the topological forward (resampling, persistence, W2) forked beside the DiceCE backward (default),
only the W2 forked (persistence in F), the W2 on the host between the graphs (w2_host), and the token-side weight
gradients as one GEMM each instead of split-K + reduction (device_tok_dw_1pass). Interleaved rounds,
median of 5 rounds x 20 steps. Diagnostic only."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    dev = torch.device("cuda", 0)
    sd = data.SAMDataset(data.synthetic_oct(seed=1000, n=8), {"prompt_type": "bboxes"}, epoch_seed=0)
    batch = data.to_device_batch(data.process_batch(data.make_processor(), data.custom_collate(
        [sd[i] for i in range(8)]), "bboxes"), dev)
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    variants = {}
    dec = model.mask_decoder
    for name, w2, fork, tok_split in (("device", "device", True, True), ("device_ph_in_F", "device", False, True),
                                      ("w2_host", "host", True, True), ("device_tok_dw_1pass", "device", True, False)):
        st = FusedTrainStep(model, lr=1e-3, topological=True, graphs=True, pipeline=True, w2=w2)
        st.fork_topo = fork
        dec.token_dw_split = tok_split  # read while the graphs are captured
        for i in range(3):  # capture + warm
            st.step(batch, next_batch=batch if i < 2 else None)
        st.flush()
        dec.token_dw_split = True
        variants[name] = st
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    n = 20
    for _ in range(5):
        for name, st in variants.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                st.step(batch, next_batch=batch if i + 1 < n else None)
            st.flush()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) * 1e3 / n)
    print(json.dumps({k: {"median_ms": round(statistics.median(v), 3), "all": [round(x, 3) for x in v]}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
