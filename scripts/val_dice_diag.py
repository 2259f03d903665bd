#!/usr/bin/env python3
"""Where the HIP-vs-oracle val-Dice difference of tests/valdice_protocol.py comes from (diagnostics, test
infrastructure: uses the oracle). Per seed pair, from the oracle-made warm start:

  hip_fp16     the HIP step with the fp16 encoder (octsam_gemm_f16 etc.: 8x smaller embedding error than bf16)
  ora_hipemb   the fp32 ORACLE decoder / losses / Adam fed the HIP encoder's bf16-GEMM image embeddings: isolates
               the encoder's precision from the decoder path (if this tracks the HIP run, the decoder path agrees)
  ora_emb16    the fp32 oracle with its own embeddings rounded to bf16 (the operand precision alone)

One JSON line per (variant, pair) with the held-out Dice at every checkpoint."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import valdice_protocol as P  # noqa: E402


def main():
    cuda = torch.device("cuda", 0)
    variants = (sys.argv[1] if len(sys.argv) > 1 else "hip_fp16,ora_hipemb,ora_emb16").split(",")
    state, adam = P.load_warm()
    t0 = time.time()
    from dilabhelmholtzoct_amd.model import SamModel
    enc = None
    if "ora_hipemb" in variants:
        enc = SamModel(P.NAME)
        enc.load_state_dict(state)
        enc = enc.to(cuda)

    def hip_embed(batch):
        with torch.no_grad():
            e = enc.vision_encoder.forward_nhwc(batch["pixel_values"].to(cuda).float())
        B = e.shape[0]
        return e.view(B, 64, 64, 256).permute(0, 3, 1, 2).contiguous().float()

    for tr, va in P.SEEDS:
        for var in variants:
            if var == "hip_fp16":
                os.environ["OCTSAM_ENCODER_DTYPE"] = "fp16"
                out = [round(P.dice_of(c), 5) for _, c in P.hip_run(cuda, state, adam, tr, va)]
                os.environ.pop("OCTSAM_ENCODER_DTYPE")
            else:
                runner = P.OracleRunner(cuda)
                if var == "ora_hipemb":
                    runner.embed_fn = hip_embed
                else:
                    runner.round_emb = True
                confs, _ = runner.run(state, adam, tr, va)
                out = [round(P.dice_of(c), 5) for _, c in confs]
                del runner
                torch.cuda.empty_cache()
            print(json.dumps({"variant": var, "train_seed": tr, "val_seed": va, "steps": P.CHECKPOINTS, "dice": out,
                              "t": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
