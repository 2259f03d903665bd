"""Same-process A/B of how the pipelined step's two streams share the chip (bench batch, B = 8, boxes, --top=True):
stream priorities and CU masks (hipExtStreamCreateWithCUMask) for the step (decoder phases, main stream) and the
encoder lookahead stream. Masks: 'all', 'q<k>' = CUs i with i % 4 in a set of k residues (k/4 of the CUs), 'nq<k>'
= its complement. Interleaved rounds, best of 4 x 10 steps. Diagnostic only.
VARS="name:main_mask:enc_mask:enc_prio,..." """
import argparse
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dilabhelmholtzoct_amd import data  # noqa: E402
from dilabhelmholtzoct_amd.model import SamModel  # noqa: E402
from dilabhelmholtzoct_amd.train import FusedTrainStep  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
device = torch.device("cuda", 0)
n_cu = torch.cuda.get_device_properties(device).multi_processor_count


def mask_words(spec):
    if spec == "all":
        sel = set(range(n_cu))
    else:
        neg = spec.startswith("n")
        k = int(spec.lstrip("nq"))
        sel = {i for i in range(n_cu) if i % 4 < k}
        if neg:
            sel = set(range(n_cu)) - sel
    words = [0] * ((n_cu + 31) // 32)
    for i in sel:
        words[i // 32] |= 1 << (i % 32)
    return words, len(sel)


def make_stream(spec, prio):
    if spec == "all":
        return torch.cuda.Stream(device=device, priority=prio), n_cu
    words, n = mask_words(spec)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value, device=device), n


args = argparse.Namespace(batch=8, prompt="bboxes")
batch = data.to_device_batch(bench.make_batch(args, 0, device, data.make_processor()), device)
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(device)
K = 10
VARS = os.environ.get("VARS", "base:all:all:0,encprio:all:all:-1,dec3q:q3:all:0,dec2q:q2:all:0,split1q:q1:nq1:0,"
                      "dec1q:q1:all:0")
steps = {}
for v in VARS.split(","):
    name, mm, em, ep = v.split(":")
    main, nm = make_stream(mm, 0)
    enc, ne = make_stream(em, int(ep))
    st = FusedTrainStep(model, lr=0.0, topological=True, graphs=True, pipeline=True)
    st._enc_stream = enc
    steps[name] = (st, main)
    print(f"{name}: main {mm} ({nm} CUs), encoder {em} ({ne} CUs) priority {ep}", flush=True)
best = {}
for rnd in range(4):
    for name, (st, main) in steps.items():
        with torch.cuda.stream(main):
            for i in range(4):
                st.step(batch, next_batch=batch if i < 3 else None)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                st.step(batch, next_batch=batch if k + 1 < K else None)
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / K
        best[name] = min(best.get(name, 1e30), ms)
        print(f"round {rnd} {name}: {ms:.3f} ms/step", flush=True)
print({k: round(v, 3) for k, v in best.items()})
