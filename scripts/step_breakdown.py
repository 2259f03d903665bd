#!/usr/bin/env python3
"""Per-call GPU time of one eager training step (BASELINE configs[2]: vit-b, B = 8, boxes, --top=True), by
phase (encoder / decoder forward / losses / decoder backward) and by call site: every kernels.* wrapper and
every _lib.call entry point is bracketed with HIP events on the launch stream. Prints the top call sites with
their shapes, total ms per phase, and the HBM bytes each GEMM moves compulsorily. Diagnostic only."""
from __future__ import annotations

import collections
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from dilabhelmholtzoct_amd import _lib, data
    from dilabhelmholtzoct_amd import kernels as Kmod
    from dilabhelmholtzoct_amd.decoder import MaskDecoder
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    dev = torch.device("cuda", 0)
    B = int(os.environ.get("BATCH", "8"))
    sd = data.SAMDataset(data.synthetic_oct(seed=1000, n=B), {"prompt_type": "bboxes"}, epoch_seed=0)
    batch = data.to_device_batch(data.process_batch(data.make_processor(), data.custom_collate(
        [sd[i] for i in range(B)]), "bboxes"), dev)
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    step = FusedTrainStep(model, topological=True)
    for _ in range(2):
        step.step(batch)
    torch.cuda.synchronize()

    phase = ["other"]
    recs = []
    active = [False]
    orig_call = _lib.call

    def site():
        for fr in reversed(traceback.extract_stack()[:-3]):
            if "dilabhelmholtzoct_amd" in fr.filename and "kernels.py" not in fr.filename and "_lib.py" not in fr.filename:
                return f"{os.path.basename(fr.filename)}:{fr.lineno}"
        return "?"

    def call(name, *a):
        if not active[0] or name in ("octsam_gemm", "octsam_gemm_f16"):  # timed by the gemm wrapper
            return orig_call(name, *a)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig_call(name, *a)
        e.record()
        recs.append((phase[0], name, site(), s, e))
        return out

    _lib.call = call
    # gemm goes through ctypes directly: wrap the python function
    orig_gemm = Kmod.gemm

    def gemm(A, Bm, **kw):
        if not active[0]:
            return orig_gemm(A, Bm, **kw)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig_gemm(A, Bm, **kw)
        e.record()
        shape = f"gemm M={kw['M']} N={kw['N']} K={kw['K']} b={kw.get('batch', 1)} am={kw.get('a_mode', 0)} bm={kw.get('b_mode', 0)}"
        recs.append((phase[0], shape, site(), s, e))
        return out

    Kmod.gemm = gemm
    import dilabhelmholtzoct_amd.model as mm
    import dilabhelmholtzoct_amd.decoder as dd
    mm.K.gemm = gemm
    dd.K.gemm = gemm

    def wrap_phase(owner, name, label):
        f = getattr(owner, name)

        def g(*a, **k):
            old = phase[0]
            phase[0] = label
            try:
                return f(*a, **k)
            finally:
                phase[0] = old
        setattr(owner, name, g)

    wrap_phase(MaskDecoder, "forward_impl", "dec_fwd")
    wrap_phase(MaskDecoder, "backward_impl", "dec_bwd")
    enc = model.vision_encoder
    f_enc = enc.forward_nhwc

    def enc_fwd(*a, **k):
        phase[0] = "encoder"
        try:
            return f_enc(*a, **k)
        finally:
            phase[0] = "loss"
    enc.forward_nhwc = enc_fwd
    active[0] = True
    step.step(batch)
    step.flush()
    active[0] = False
    torch.cuda.synchronize()
    per_phase = collections.defaultdict(float)
    per_site = collections.defaultdict(lambda: [0.0, 0])
    for ph, name, st, s, e in recs:
        ms = s.elapsed_time(e)
        per_phase[ph] += ms
        key = (ph, name, st)
        per_site[key][0] += ms
        per_site[key][1] += 1
    print(json.dumps({k: round(v, 3) for k, v in per_phase.items()}))
    rows = sorted(per_site.items(), key=lambda kv: -kv[1][0])
    for (ph, name, st), (ms, n) in rows[:70]:
        print(f"{ph:8s} {ms * 1e3:9.1f} us  x{n:3d}  {st:22s} {name}")


if __name__ == "__main__":
    main()
