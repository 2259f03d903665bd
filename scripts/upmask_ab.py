#!/usr/bin/env python3
"""Same-box A/B of two builds of the fused mask-head kernels (OCTSAM_LIB selects the library; diagnostics only).

  python scripts/upmask_ab.py run TAG     time octsam_upmask_fwd / _bwd / _bwd with the LayerNorm2d + GELU (the
                                          step's form) at P prompts, save times + output hashes
  python scripts/upmask_ab.py cmp A B     times side by side, outputs bitwise
env P (default 168, the bench step's prompts)."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")


def sha(*ts):
    h = hashlib.sha1()
    for t in ts:
        h.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()


def timed(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


def run(tag):
    from dilabhelmholtzoct_amd import kernels
    P = int(os.environ.get("P", "168"))
    ns = 1
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    up1 = torch.randn(P * 16384, 64, generator=g).to(dev, torch.bfloat16)
    x = torch.randn(P * 16384, 64, generator=g).to(dev, torch.bfloat16)  # ConvT1 output (LayerNorm input)
    xf = x.float()
    mean, rstd = xf.mean(1), torch.rsqrt(xf.var(1, unbiased=False) + 1e-6)
    lw, lb = (1 + 0.1 * torch.randn(64, generator=g)).to(dev), (0.1 * torch.randn(64, generator=g)).to(dev)
    w2 = (0.15 * torch.randn(64, 128, generator=g)).to(dev, torch.bfloat16)
    b2 = (0.2 * torch.randn(32, generator=g)).to(dev)
    hyper = torch.randn(P, ns, 32, generator=g).to(dev)
    dmask = torch.randn(P, ns, 256, 256, generator=g).to(dev)
    masks = torch.empty(P, ns, 256, 256, device=dev)
    dup1 = torch.empty_like(up1)
    dx = torch.empty_like(up1)
    dw2, db2, dh = torch.empty(64, 128, device=dev), torch.empty(32, device=dev), torch.empty(P, ns, 32, device=dev)
    dlw, dlb = torch.empty(64, device=dev), torch.empty(64, device=dev)
    fns = {"fwd": lambda: kernels.upmask_fwd(up1, w2, b2, hyper, P, ns, masks),
           "bwd": lambda: kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, dup1, dw2, db2, dh),
           "bwd_ln": lambda: kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, dx, dw2, db2, dh,
                                                ln=(x, mean, rstd, lw, lb, dlw, dlb))}
    best = {}
    for _ in range(3):
        for k, fn in fns.items():
            best[k] = min(best.get(k, 1e30), timed(fn))
    hashes = {}
    fns["fwd"]()
    hashes["fwd"] = sha(masks)
    fns["bwd"]()
    hashes["bwd"] = sha(dup1, dw2, db2, dh)
    fns["bwd_ln"]()
    hashes["bwd_ln"] = sha(dx, dw2, db2, dh, dlw, dlb)
    torch.cuda.synchronize()
    res = {"tag": tag, "lib": os.environ.get("OCTSAM_LIB", "default"), "P": P,
           "us": {k: round(v, 1) for k, v in best.items()}, "sha": hashes}
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"upmask_ab_{tag}.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps(res), flush=True)


def cmp(a, b):
    ra = json.load(open(os.path.join(OUT, f"upmask_ab_{a}.json")))
    rb = json.load(open(os.path.join(OUT, f"upmask_ab_{b}.json")))
    for k in ra["us"]:
        print(json.dumps({"kernel": k, a: ra["us"][k], b: rb["us"].get(k),
                          "identical": ra["sha"][k] == rb["sha"].get(k)}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
