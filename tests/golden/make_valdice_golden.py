#!/usr/bin/env python3
"""Makes the val-Dice protocol's committed fixtures (tests/valdice_protocol.py) with the fp32 ORACLE only, on an
MI355X (the oracle's SamModel runs on the GPU to keep this short; oracle_mode makes it run-to-run reproducible):

  --warm    tests/golden/valdice_warm_oracle.safetensors: the committed start decoder continued by the oracle for
            WARM_STEPS steps (cold Adam) on synthetic_oct(seed=2000); decoder weights and Adam moments rounded to bf16
            for storage, the step count as fp32. This file is the protocol's start state on both sides.
  --oracle  tests/golden/valdice_oracle.json: for every (training, held-out) seed pair the oracle's held-out Dice at
            every checkpoint from that start state, plus the oracle's own spread per checkpoint (the same run from
            N_PERTURB copies of the start with each decoder weight times 1 + 2^-8 u): the protocol's noise floor.

Test infrastructure: imports oracle/ (and nothing of it reaches the product path)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import valdice_protocol as P  # noqa: E402

N_PERTURB = 1


def make_warm(cuda, out):
    from safetensors.torch import load_file, save_file
    state = P.base_state()
    for k, v in load_file(P.START).items():
        assert k in state and state[k].shape == v.shape, k
        state[k] = v.float()
    runner = P.OracleRunner(cuda)
    ref = runner.make(state)
    k, ep = 0, 0
    while k < P.WARM_STEPS:
        k += runner.train_steps(ref, P.WARM_SEED, ep, limit=P.WARM_STEPS - k)
        ep += 1
    d = P.dice_of(runner.conf(ref, P.WARM_VAL_SEED))
    sd = {"mask_decoder." + n: t.detach().to(torch.bfloat16).cpu().contiguous()
          for n, t in ref.model.mask_decoder.state_dict().items()}
    step = None
    for name, p in ref.model.mask_decoder.named_parameters():
        st = ref.opt.state.get(p, {})
        if "step" in st:
            step = float(st["step"])
        for key in ("exp_avg", "exp_avg_sq"):
            t = st[key] if st else torch.zeros_like(p)
            sd[f"{key}.mask_decoder.{name}"] = t.detach().to(torch.bfloat16).cpu().contiguous()
    sd["step"] = torch.tensor([step], dtype=torch.float32)
    save_file(sd, out)
    print(json.dumps({"warm": out, "steps": k, "epochs_started": ep, "adam_step": step,
                      "val_dice_seed3000": round(d, 5)}), flush=True)


def _doc(pairs, t0):
    n = len(pairs)
    mean = [round(sum(p["oracle_dice"][i] for p in pairs) / n, 5) for i in range(len(P.CHECKPOINTS))]
    return {"protocol": "tests/valdice_protocol.py: sam-vit-base synthetic weights (seed 0); start state "
                        "tests/golden/valdice_warm_oracle.safetensors (the fp32 oracle: the committed start decoder + "
                        f"{P.WARM_STEPS} oracle steps on synthetic_oct(seed={P.WARM_SEED}), bf16-stored); per seed "
                        f"pair {P.EPOCHS} epochs on synthetic_oct(train seed, n={P.N_TRAIN}), B={P.BS}, box prompts, "
                        f"--top=True, lr {P.LR}; held-out synthetic_oct(val seed, n={P.N_VAL}), epoch-0 prompts; mean "
                        "per-class Dice after every epoch",
            "made_by": "tests/golden/make_valdice_golden.py --oracle on MI355X (oracle/step_ref.py in oracle_mode: "
                       "MIOpen off, torch deterministic algorithms); depends on no HIP kernel",
            "steps": P.CHECKPOINTS, "pairs": pairs, "oracle_mean_dice": mean,
            "noise_floor": "per pair, perturbed_dice = the oracle's Dice from the start state with every decoder weight "
                           "times (1 + 2^-8 u), u ~ U(-1, 1) (perturbation seeds 100, 101, ...; at least one run per "
                           "pair); spread = max - min over the base run and the perturbed runs; the mean over pairs of "
                           "perturbed_dice[0] - oracle_dice is the protocol's noise floor beside HIP's mean difference",
            "seconds": round(time.time() - t0, 1)}


def make_oracle(cuda, out, keep=False, n_perturb=N_PERTURB, fill=0, deadline=None):
    """keep: pairs already in `out` are kept (only the missing ones are run); n_perturb: perturbed runs per new pair;
    fill: kept pairs with fewer than `fill` perturbed runs get the missing ones. The file is rewritten after every
    pair, so a run stopped at `deadline` (seconds) keeps what it made (rerun with keep to continue)."""
    from oracle.eval_ref import mean_specificity_ref
    state, adam = P.load_warm()
    runner = P.OracleRunner(cuda)
    old = {}
    if keep and os.path.exists(out):
        old = {(g["train_seed"], g["val_seed"]): g for g in json.load(open(out))["pairs"]}
    t0 = time.time()
    done = dict(old)

    def save():
        pairs = [done[sp] for sp in P.SEEDS if sp in done] + [g for sp, g in done.items() if sp not in P.SEEDS]
        with open(out + ".tmp", "w") as f:
            json.dump(_doc(pairs, t0), f, indent=1)
        os.replace(out + ".tmp", out)

    def spread_of(rec):
        runs = [rec["oracle_dice"]] + rec["perturbed_dice"]
        return ([round(max(r[i] for r in runs) - min(r[i] for r in runs), 5) for i in range(len(rec["oracle_dice"]))]
                if rec["perturbed_dice"] else None)

    for tr, va in P.SEEDS:
        if deadline is not None and time.time() - t0 > deadline:
            print(json.dumps({"stopped_at_deadline": deadline, "pairs_done": len(done)}), flush=True)
            break
        rec = done.get((tr, va))
        if rec is None:
            base, moved = runner.run(state, adam, tr, va)
            rec = {"train_seed": tr, "val_seed": va, "steps": [k for k, _ in base],
                   "oracle_dice": [round(P.dice_of(c), 5) for _, c in base],
                   "oracle_specificity": round(mean_specificity_ref(base[-1][1]), 4), "oracle_moved": round(moved, 4),
                   "perturbed_dice": []}
            want = n_perturb
        else:
            rec = dict(rec)
            rec["perturbed_dice"] = list(rec.get("perturbed_dice") or [])
            want = max(0, fill - len(rec["perturbed_dice"]))
            if want == 0:
                continue
        for j in range(len(rec["perturbed_dice"]), len(rec["perturbed_dice"]) + want):
            pert, _ = runner.run(P.perturbed(state, 100 + j), adam, tr, va)
            rec["perturbed_dice"].append([round(P.dice_of(c), 5) for _, c in pert])
        rec["spread"] = spread_of(rec)
        done[tr, va] = rec
        runner.forget(tr, va)
        save()
        print(json.dumps({"pair": [tr, va], "oracle_dice": rec["oracle_dice"], "perturbed": rec["perturbed_dice"],
                          "t": round(time.time() - t0, 1)}), flush=True)
    save()
    d = json.load(open(out))
    print(json.dumps({"pairs": len(d["pairs"]), "oracle_mean_dice": d["oracle_mean_dice"]}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--warm", action="store_true")
    p.add_argument("--oracle", action="store_true")
    p.add_argument("--warm-out", default=P.WARM)
    p.add_argument("--oracle-out", default=P.ORACLE_JSON)
    p.add_argument("--keep", action="store_true", help="--oracle: keep the pairs already in --oracle-out")
    p.add_argument("--perturb", type=int, default=N_PERTURB, help="--oracle: perturbed runs per new pair")
    p.add_argument("--fill", type=int, default=0, help="--oracle --keep: perturbed runs every kept pair should have")
    p.add_argument("--deadline", type=float, default=None, help="--oracle: stop starting new pairs after this many s")
    a = p.parse_args()
    cuda = torch.device("cuda", 0)
    if a.warm:
        make_warm(cuda, a.warm_out)
    if a.oracle:
        make_oracle(cuda, a.oracle_out, keep=a.keep, n_perturb=a.perturb, fill=a.fill, deadline=a.deadline)


if __name__ == "__main__":
    main()
