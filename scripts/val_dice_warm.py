#!/usr/bin/env python3
"""Val-Dice protocol diagnostics for tests/test_gpu_val_dice.py (128 synthetic training scans,
32 held-out, B = 8, box prompts, --top=True, lr 1e-3; ref:octsam/models/training_utils.py:27-80, 113-156, 246).

--mode spread   the round-3 protocol (start decoder tests/golden/valdice_start_decoder.safetensors with a COLD
                Adam): the fp32 oracle from the start and from perturbed copies of it (each weight times
                1 + 2^-8 u, u ~ U(-1, 1), i.e. bf16-rounding-sized noise; and the oracle fed bf16-rounded image
                embeddings, the HIP encoder's operand precision), plus the HIP step; val Dice every --every steps.
                The spread of the oracle runs at a checkpoint is the noise floor of a HIP-vs-oracle comparison there.
--mode warm     continue the oracle from the same start with a cold Adam on the start's own training set (seed
                2000) for --steps steps and save decoder weights + Adam moments + step (bf16 tensors) to --save.
--mode traj     both sides from a warm start (--warm: weights + Adam state), --epochs epochs on the test's set
                (seed 2001), val (seed 3001) every --every steps: HIP (hipGraphs + lookahead, as bench.py) vs oracle.
One JSON line per checkpoint on stdout and in --out."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

NAME = "facebook/sam-vit-base"
START = os.path.join(ROOT, "tests", "golden", "valdice_start_decoder.safetensors")


def batches(seed, n, bs, epoch):
    from dilabhelmholtzoct_amd import data
    proc = data.make_processor()
    sd = data.SAMDataset(data.synthetic_oct(seed=seed, n=n), {"prompt_type": "bboxes"}, epoch_seed=seed)
    sd.epoch = epoch
    return [data.process_batch(proc, data.custom_collate([sd[i] for i in range(s, min(n, s + bs))]), "bboxes")
            for s in range(0, n, bs)]


def oracle_adam_state(ref) -> dict:
    """torch Adam state by HF name; parameters that never received a gradient (the IoU head: the loss does not use
    it) have no state in torch and zero moments in the fused Adam, so they are exported as zeros."""
    out = {}
    step = None
    for name, p in ref.model.mask_decoder.named_parameters():
        st = ref.opt.state.get(p, {})
        if "step" in st:
            step = float(st["step"])
        out[f"exp_avg.mask_decoder.{name}"] = st["exp_avg"].detach().cpu() if st else torch.zeros_like(p).cpu()
        out[f"exp_avg_sq.mask_decoder.{name}"] = st["exp_avg_sq"].detach().cpu() if st else torch.zeros_like(p).cpu()
    out["step"] = torch.tensor(step)
    return out


def load_oracle_adam(ref, state):
    for name, p in ref.model.mask_decoder.named_parameters():
        if not bool(state[f"exp_avg_sq.mask_decoder.{name}"].any()):
            continue  # no state in torch for a parameter that never had a gradient
        ref.opt.state[p] = {"step": torch.tensor(float(state["step"])),
                            "exp_avg": state[f"exp_avg.mask_decoder.{name}"].to(p.device, torch.float32).clone(),
                            "exp_avg_sq": state[f"exp_avg_sq.mask_decoder.{name}"].to(p.device, torch.float32).clone()}


def split_warm(path):
    from safetensors.torch import load_file
    raw = load_file(path)
    weights = {k: v.float() for k, v in raw.items() if k.startswith("mask_decoder.")}
    adam = {k: v.float() for k, v in raw.items() if k.startswith("exp_avg")}
    adam["step"] = raw["step"].float()
    return weights, adam


class Runner:
    def __init__(self, dev, bs):
        from dilabhelmholtzoct_amd import data
        from oracle.step_ref import synthetic_state_dict
        self.dev, self.bs = dev, bs
        self.base_state = synthetic_state_dict(NAME, seed=0)
        self.data = data
        self._emb = {}

    def state_from(self, weights):
        st = dict(self.base_state)
        for k, v in weights.items():
            assert k in st and st[k].shape == v.shape, k
            st[k] = v.float()
        return st

    def val(self, seed):
        vc = batches(seed, 32, self.bs, 0)
        return vc, [self.data.to_device_batch(v, self.dev) for v in vc]

    def emb(self, ref, key, batch, bf16=False):
        if key not in self._emb:
            self._emb[key] = ref.embed(batch)
        e = self._emb[key]
        return e.bfloat16().float() if bf16 else e


def oracle_conf(ref, runner, val_cpu, tag, bf16_emb=False):
    from oracle.eval_ref import pooled_confusion_ref
    c = torch.zeros(14, 4, dtype=torch.int64)
    with torch.no_grad():
        for i, v in enumerate(val_cpu):
            c += pooled_confusion_ref(ref.predict(v, runner.emb(ref, (tag, i), v, bf16_emb)), v["gt_u8"],
                                      v["mask_values"])
    return c


def hip_conf(step, model, val):
    from dilabhelmholtzoct_amd.train import class_confusion, predict_masks
    step.flush()
    c = torch.zeros(14, 3, dtype=torch.int64)
    for v in val:
        c += class_confusion(predict_masks(model, v), v["gt_u8"], v["mask_values"])
    return torch.cat([c, torch.zeros(14, 1, dtype=c.dtype)], 1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", choices=["spread", "warm", "traj"], required=True)
    p.add_argument("--variants", default="base,ulp1,ulp2,ulp3,emb_bf16,hip")
    p.add_argument("--epochs", type=int, default=2)
    p.add_argument("--steps", type=int, default=64)
    p.add_argument("--every", type=int, default=4)
    p.add_argument("--bs", type=int, default=8)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--warm", default=None)
    p.add_argument("--save", default=None)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    from safetensors.torch import load_file, save_file
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    from oracle.eval_ref import mean_dice_ref, mean_specificity_ref
    from oracle.step_ref import CpuReferenceStep
    dev = torch.device("cuda", 0)
    t0 = time.time()
    fo = open(a.out, "a") if a.out else None
    R = Runner(dev, a.bs)

    def emit(rec):
        rec["t"] = round(time.time() - t0, 1)
        print(json.dumps(rec), flush=True)
        if fo:
            fo.write(json.dumps(rec) + "\n")
            fo.flush()

    start_w = {k: v.float() for k, v in load_file(START).items()}
    warm_adam = None
    if a.warm and a.mode == "spread":  # the spread along the warm-start trajectory (weights + Adam state)
        start_w, warm_adam = split_warm(a.warm)
    if a.mode == "spread":
        val_cpu, val = R.val(3001)
        tr_by_ep = {ep: batches(2001, 128, a.bs, ep) for ep in range(a.epochs)}
        for var in a.variants.split(","):
            w = dict(start_w)
            if var.startswith("ulp"):
                g = torch.Generator().manual_seed(int(var[3:]))
                w = {k: v * (1 + 2.0 ** -8 * (2 * torch.rand(v.shape, generator=g) - 1)) for k, v in w.items()}
            state = R.state_from(w)
            bf = var == "emb_bf16"
            if var == "hip":
                model = SamModel(NAME)
                model.load_state_dict(state)
                model = model.to(dev)
                st = FusedTrainStep(model, lr=a.lr, topological=True, graphs=True, pipeline=True)
                if warm_adam is not None:
                    st.load_optimizer_state(warm_adam)
                conf = lambda: hip_conf(st, model, val)  # noqa: E731
            else:
                ref = CpuReferenceStep(NAME, topological=True, lr=a.lr, state_dict=state, device=dev, loss_device=dev)
                if warm_adam is not None:
                    load_oracle_adam(ref, warm_adam)
                conf = lambda: oracle_conf(ref, R, val_cpu, "v3001", bf)  # noqa: E731
            k = 0
            c = conf()
            emit({"variant": var, "step": k, "dice": round(mean_dice_ref(c), 5),
                  "spec": round(mean_specificity_ref(c), 4)})
            for ep in range(a.epochs):
                tr_cpu = tr_by_ep[ep]
                tr = [R.data.to_device_batch(b, dev) for b in tr_cpu] if var == "hip" else None
                for i in range(len(tr_cpu)):
                    if var == "hip":
                        st.step(tr[i], next_batch=tr[i + 1] if i + 1 < len(tr) else None)
                    else:
                        ref.step(tr_cpu[i], R.emb(ref, ("t2001", i), tr_cpu[i], bf))
                    k += 1
                    if k % a.every == 0:
                        c = conf()
                        emit({"variant": var, "step": k, "dice": round(mean_dice_ref(c), 5),
                              "spec": round(mean_specificity_ref(c), 4)})
            del conf
        return

    if a.mode == "warm":
        val_cpu, _ = R.val(3000)
        ref = CpuReferenceStep(NAME, topological=True, lr=a.lr, state_dict=R.state_from(start_w), device=dev,
                               loss_device=dev)
        k = 0
        c = oracle_conf(ref, R, val_cpu, "v3000")
        emit({"mode": "warm", "step": k, "dice": round(mean_dice_ref(c), 5), "spec": round(mean_specificity_ref(c), 4)})
        ep = 0
        while k < a.steps:
            tr_cpu = batches(2000, 128, a.bs, ep)
            for i in range(len(tr_cpu)):
                ref.step(tr_cpu[i], R.emb(ref, ("t2000", i), tr_cpu[i]))
                k += 1
                if k % a.every == 0:
                    c = oracle_conf(ref, R, val_cpu, "v3000")
                    emit({"mode": "warm", "step": k, "dice": round(mean_dice_ref(c), 5),
                          "spec": round(mean_specificity_ref(c), 4)})
                if k >= a.steps:
                    break
            ep += 1
        sd = {"mask_decoder." + n: t.detach().to(torch.bfloat16).cpu().contiguous()
              for n, t in ref.model.mask_decoder.state_dict().items()}
        for kk, v in oracle_adam_state(ref).items():
            sd[kk] = v.to(torch.bfloat16).contiguous() if kk != "step" else v.float().reshape(1)
        os.makedirs(os.path.dirname(os.path.abspath(a.save)), exist_ok=True)
        save_file(sd, a.save)
        emit({"mode": "warm", "saved": a.save, "epochs_seen": ep})
        return

    # traj: both sides from the warm start, bf16-stored weights + Adam moments loaded on both
    weights, adam = split_warm(a.warm)
    state = R.state_from(weights)
    val_cpu, val = R.val(3001)
    ref = CpuReferenceStep(NAME, topological=True, lr=a.lr, state_dict=state, device=dev, loss_device=dev)
    load_oracle_adam(ref, adam)
    model = SamModel(NAME)
    model.load_state_dict(state)
    model = model.to(dev)
    st = FusedTrainStep(model, lr=a.lr, topological=True, graphs=True, pipeline=True)
    st.load_optimizer_state(adam)

    def both(k):
        co = hip_conf(st, model, val)
        cr = oracle_conf(ref, R, val_cpu, "v3001")
        dh, dr = mean_dice_ref(co), mean_dice_ref(cr)
        emit({"mode": "traj", "step": k, "dice_hip": round(dh, 5), "dice_ref": round(dr, 5),
              "diff": round(dh - dr, 5), "spec_hip": round(mean_specificity_ref(co), 4),
              "spec_ref": round(mean_specificity_ref(cr), 4)})

    k = 0
    both(0)
    for ep in range(a.epochs):
        tr_cpu = batches(2001, 128, a.bs, ep)
        tr = [R.data.to_device_batch(b, dev) for b in tr_cpu]
        for i in range(len(tr)):
            st.step(tr[i], next_batch=tr[i + 1] if i + 1 < len(tr) else None)
            ref.step(tr_cpu[i], R.emb(ref, ("t2001", i), tr_cpu[i]))
            k += 1
            if k % a.every == 0:
                both(k)


if __name__ == "__main__":
    main()
