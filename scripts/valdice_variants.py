#!/usr/bin/env python3
"""The HIP side of the val-Dice protocol (tests/valdice_protocol.py) under step variants, against the committed
oracle values (tests/golden/valdice_oracle.json): per variant the per-pair differences and their mean per checkpoint
(diagnostics). Variants (comma list, argv[1]): base, dkeys (decoder.fuse_dkeys on), fp16 (the fp16 encoder)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import valdice_protocol as P  # noqa: E402

ENV = {"base": {}, "dkeys": {"OCTSAM_FUSE_DKEYS": "1"}, "fp16": {"OCTSAM_ENCODER_DTYPE": "fp16"}}


def main():
    cuda = torch.device("cuda", 0)
    variants = (sys.argv[1] if len(sys.argv) > 1 else "base,dkeys").split(",")
    gold = {(g["train_seed"], g["val_seed"]): g for g in json.load(open(P.ORACLE_JSON))["pairs"]}
    state, adam = P.load_warm()
    batches = P.device_batches(cuda)
    for var in variants:
        t0 = time.time()
        for k in ("OCTSAM_FUSE_DKEYS", "OCTSAM_ENCODER_DTYPE"):
            os.environ.pop(k, None)
        os.environ.update(ENV[var])
        diffs = []
        for tr, va in P.SEEDS:
            hip = [P.dice_of(c) for _, c in P.hip_run(cuda, state, adam, tr, va, epoch_batches=batches,
                                                        val_batches=batches(va, P.N_VAL, 0))]
            d = [round(h - o, 5) for h, o in zip(hip, gold[(tr, va)]["oracle_dice"])]
            diffs.append(d)
            print(json.dumps({"variant": var, "pair": [tr, va], "diff": d}), flush=True)
        mean = [round(sum(d[i] for d in diffs) / len(diffs), 5) for i in range(len(P.CHECKPOINTS))]
        print(json.dumps({"variant": var, "mean_diff": mean, "max_abs": max(abs(x) for x in mean),
                          "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
