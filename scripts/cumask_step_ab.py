"""Same-process A/B of the pipelined training step (bench.py's loop, B = 8 boxes, --top=True) with the encoder
lookahead stream and the step's own (decoder) stream created by hipExtStreamCreateWithCUMask: does partitioning the
CUs between the MFMA-bound encoder and the HBM-bound decoder beat letting them contend for every CU? Variants
"enc:dec" name each stream's CU set: all, even / odd (alternate CUs), q1 (every 4th CU), q3 (the other three of
four), h1 (every 8th CU), def (an ordinary stream). Median of 5 interleaved rounds x 20 steps. Diagnostic only."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(dev, sel):
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (n_cu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(n_cu):
        if sel(c):
            mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


SETS = {"all": lambda c: True, "even": lambda c: c % 2 == 0, "odd": lambda c: c % 2 == 1,
        "q1": lambda c: c % 4 == 0, "q3": lambda c: c % 4 != 0, "h1": lambda c: c % 8 == 0,
        "t3": lambda c: c % 8 != 0}


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
    for name in os.environ.get("CU_VARIANTS", "default,all:all,q3:all,all:q1,q3:q1,even:odd").split(","):
        st = FusedTrainStep(model, lr=1e-3, topological=True, graphs=True, pipeline=True)
        main_s = torch.cuda.current_stream(dev)
        if name != "default":  # "def" keeps that stream an ordinary one (torch's current / a torch.cuda.Stream)
            e, d = name.split(":")
            if e != "def":
                st._enc_stream = masked_stream(dev, SETS[e])
            if d != "def":
                main_s = masked_stream(dev, SETS[d])
        with torch.cuda.stream(main_s):
            for i in range(3):
                st.step(batch, next_batch=batch if i < 2 else None)
            st.flush()
        torch.cuda.synchronize()
        variants[name] = (st, main_s)
    res = {k: [] for k in variants}
    n = 20
    for _ in range(5):
        for name, (st, main_s) in variants.items():
            with torch.cuda.stream(main_s):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(n):
                    st.step(batch, next_batch=batch if i + 1 < n else None)
                st.flush()
                torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) * 1e3 / n)
    print(json.dumps({k: {"median_ms": round(statistics.median(v), 3), "all": [round(x, 3) for x in v]}
                      for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
