"""Same-box A/B of two builds of the mask-decoder attention kernels at the vit-b step's shapes (OCTSAM_LIB selects the
library; diagnostics only). B = 8 images x N = 21 prompts, T = 7 tokens, L = 4096 keys.

  python scripts/dec_attn_ab.py run TAG      time each call (min over rounds), hash the outputs -> gpurun_out/
  python scripts/dec_attn_ab.py cmp A B      times side by side, outputs bitwise (sha1 of the bytes)"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
B, N, T, L, CI = 8, 21, 7, 4096, 128
P = B * N


def timed(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


def sha(*ts):
    h = hashlib.sha1()
    for t in ts:
        h.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def run(tag):
    from dilabhelmholtzoct_amd import kernels as K
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)

    def rn(*shape, s=1.0, dt=torch.float32):
        return (torch.randn(*shape, generator=g) * s).to(dev, dt)

    img = rn(B * L, 3 * CI, s=1.5, dt=torch.bfloat16)      # layer 0: [K | Q' | V] per image
    per = rn(P * L, 3 * CI, s=1.5, dt=torch.bfloat16)      # layer 1: per prompt
    fin = rn(P * L, 2 * CI, s=1.5, dt=torch.bfloat16)      # final attention: [K | V] per prompt
    q = rn(P, T, CI, s=2.0)
    dout = rn(P, T, CI)
    kt, vt = rn(P, T, CI, s=2.0), rn(P, T, CI)
    dio = rn(P * L, CI, dt=torch.bfloat16)
    cases = {}

    def t2i_case(name, buf, ld, rep, bwd_sum):
        out = torch.empty(P, T, CI, device=dev, dtype=torch.bfloat16)
        of = torch.empty(P, T, CI, device=dev)
        lse = torch.empty(P, 8, T, device=dev)
        vcol = ld - CI
        fwd = lambda: K.t2i_fwd(q, buf, buf[:, vcol:], ld, rep, P, T, L, out, lse, out_f32=of)  # noqa: E731
        fwd()
        dq = torch.empty(P, T, CI, device=dev, dtype=torch.bfloat16)
        if bwd_sum:
            dkv = torch.empty((P // rep) * L, 2 * CI, device=dev, dtype=torch.bfloat16)
            bwd = lambda: K.t2i_bwd_sum(q, buf, buf[:, vcol:], ld, rep, P, T, L, out, dout, lse, dq, dkv,  # noqa
                                        dkv[:, CI:], 2 * CI, out_f32=of)
        else:
            dkv = torch.empty(P * L, 2 * CI, device=dev, dtype=torch.bfloat16)
            bwd = lambda: K.t2i_bwd(q, buf, buf[:, vcol:], ld, rep, P, T, L, out, dout, lse, dq, dkv, dkv[:, CI:],  # noqa
                                    2 * CI, out_f32=of)
        cases[name + "_fwd"] = (fwd, (out, of, lse))
        cases[name + "_bwd"] = (bwd, (dq, dkv))

    t2i_case("t2i0", img, 3 * CI, N, True)
    t2i_case("t2i1", per, 3 * CI, 1, False)
    t2i_case("t2if", fin, 2 * CI, 1, False)
    o0 = torch.empty(P * L, CI, device=dev, dtype=torch.bfloat16)
    cases["i2t0_fwd"] = (lambda: K.i2t_fwd(img[:, CI:], 3 * CI, N, kt, vt, P, T, L, o0, CI), (o0,))
    dqi = torch.empty(B * L, CI, device=dev, dtype=torch.bfloat16)
    res0 = {}

    def i2t0_bwd():
        res0["kv"] = K.i2t_bwd_sum(img[:, CI:], 3 * CI, N, kt, vt, P, T, L, dio, CI, dqi, CI)
    cases["i2t0_bwd"] = (i2t0_bwd, (dqi,))
    dq1 = torch.empty(P * L, CI, device=dev, dtype=torch.bfloat16)
    res1 = {}

    def i2t1_bwd():
        res1["kv"] = K.i2t_bwd(per[:, CI:], 3 * CI, 1, kt, vt, P, T, L, dio, CI, dq1, CI)
    cases["i2t1_bwd"] = (i2t1_bwd, (dq1,))
    best = {}
    for _ in range(3):
        for name, (fn, _) in cases.items():
            best[name] = min(best.get(name, 1e30), timed(fn))
    res = []
    for name, (fn, outs) in cases.items():
        fn()
        torch.cuda.synchronize()
        extra = res0["kv"] if name == "i2t0_bwd" else res1["kv"] if name == "i2t1_bwd" else ()
        res.append({"call": name, "us": round(best[name], 1), "sha": sha(*outs, *extra)})
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"dec_attn_ab_{tag}.json"), "w") as f:
        json.dump(res, f)
    for r in res:
        print(json.dumps(r), flush=True)


def cmp(a, b):
    ra = {r["call"]: r for r in json.load(open(os.path.join(OUT, f"dec_attn_ab_{a}.json")))}
    rb = {r["call"]: r for r in json.load(open(os.path.join(OUT, f"dec_attn_ab_{b}.json")))}
    for k in ra:
        print(json.dumps({"call": k, a: ra[k]["us"], b: rb.get(k, {}).get("us"),
                          "identical": ra[k]["sha"] == rb.get(k, {}).get("sha")}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
