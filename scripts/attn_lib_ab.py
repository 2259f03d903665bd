"""Same-box A/B of two builds of the ViT attention kernels (OCTSAM_LIB selects the library; diagnostics only).

  python scripts/attn_lib_ab.py run TAG      time the variants at the workload shapes, save outputs + times
  python scripts/attn_lib_ab.py cmp A B      compare two runs: times side by side, outputs bitwise

Variants (octsam_attention_set_variant): global -1 (default), 2 (4-wave, two per CU), 1 (plain 8-wave); windowed 100
(one unit per workgroup), 101 (persistent; only where the library has it: ATTN_WIN="100,101")."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")


def timed(fn, it=20):
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
    from dilabhelmholtzoct_amd import _lib, kernels as K
    lib = _lib.load()
    glob = [int(v) for v in os.environ.get("ATTN_GLOB", "-1,2,1").split(",")]
    win = [int(v) for v in os.environ.get("ATTN_WIN", "100").split(",")]
    g = torch.Generator().manual_seed(0)
    cases = [(64, 8, 12, 64, torch.bfloat16), (14, 200, 12, 64, torch.bfloat16), (64, 8, 16, 80, torch.float16),
             (14, 200, 16, 80, torch.float16)]
    data = []
    for side, nseq, heads, hd, dt in cases:
        tokens = nseq * side * side if side == 64 else 8 * 4096
        qkv = torch.randn(tokens, 3 * heads * hd, generator=g).to("cuda", dt)
        pad = torch.randn(3 * heads * hd, generator=g).to("cuda", dt) if side == 14 else None
        Rh = (torch.randn(2 * side - 1, hd, generator=g) * 0.02).cuda()
        vs = glob if side == 64 else win
        outs = {v: torch.empty(tokens, heads * hd, device="cuda", dtype=dt) for v in vs}
        data.append((side, nseq, heads, hd, dt, qkv, outs, Rh, pad))
    best = {}
    for _ in range(5):
        for i, (side, nseq, heads, hd, dt, qkv, outs, Rh, pad) in enumerate(data):
            kw = dict(grid=64, pad_row=pad) if side == 14 else {}
            for v in outs:
                lib.octsam_attention_set_variant(v)
                t = timed(lambda: K.vit_attention(qkv, outs[v], Rh, Rh, nseq=nseq, side=side, heads=heads, **kw))
                best[i, v] = min(best.get((i, v), 1e30), t)
    lib.octsam_attention_set_variant(-1)
    lib.octsam_attention_set_variant(100)
    res, saved = [], {}
    for i, (side, nseq, heads, hd, dt, qkv, outs, *_) in enumerate(data):
        fl = 4.0 * nseq * heads * (side * side) ** 2 * hd
        for v, o in outs.items():
            res.append({"case": i, "side": side, "hd": hd, "variant": v, "us": round(best[i, v], 1),
                        "tflops": round(fl / best[i, v] / 1e6, 1)})
            saved[f"{i}_{v}"] = hashlib.sha1(o.view(torch.uint8).cpu().numpy().tobytes()).hexdigest()

    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"attn_lib_ab_{tag}.sha.json"), "w") as f:
        json.dump(saved, f)
    with open(os.path.join(OUT, f"attn_lib_ab_{tag}.json"), "w") as f:
        json.dump(res, f)
    for r in res:
        print(json.dumps(r), flush=True)


def cmp(a, b):
    ta = {(r["case"], r["variant"]): r for r in json.load(open(os.path.join(OUT, f"attn_lib_ab_{a}.json")))}
    tb = {(r["case"], r["variant"]): r for r in json.load(open(os.path.join(OUT, f"attn_lib_ab_{b}.json")))}
    oa = json.load(open(os.path.join(OUT, f"attn_lib_ab_{a}.sha.json")))
    ob = json.load(open(os.path.join(OUT, f"attn_lib_ab_{b}.sha.json")))
    ref = {}
    for k in sorted(set(ta) | set(tb)):
        row = {"case": k[0], "variant": k[1], a: ta.get(k, {}).get("us"), b: tb.get(k, {}).get("us")}
        key = f"{k[0]}_{k[1]}"
        if key in oa and key in ob:
            row["identical"] = oa[key] == ob[key]
        # windowed variants of one library against the other library's first windowed variant
        base = ref.setdefault(k[0], oa.get(key))
        if key in ob and base is not None:
            row["identical_to_base"] = ob[key] == base
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
