#!/usr/bin/env python3
"""Val-Dice trajectory of the HIP training step vs the fp32 oracle on SURVEY.md §8(d)'s protocol
(synthetic 128 train / 32 val OCT-like images, B = 8, box prompts, --top=True, lr 1e-3, same seeds on both
sides). Diagnostic for tests/test_gpu_val_dice.py: prints one JSON line per checkpoint with the pooled
per-class "Mean dice" of both sides (ref:octsam/models/training_utils.py:153-156,246) and the oracle's
mean specificity / sensitivity, so the non-degenerate regime (specificity > 0.5) can be read off.

The oracle (oracle/step_ref.py, transformers SamModel fp32) runs on the GPU only to keep this short; its
frozen encoder's embeddings are computed once per batch (the encoder has no trainable weight)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def batches(seed, n, bs, epoch, prompt="bboxes"):
    from dilabhelmholtzoct_amd import data
    proc = data.make_processor()
    ds = data.synthetic_oct(seed=seed, n=n)
    sd = data.SAMDataset(ds, {"prompt_type": prompt}, epoch_seed=seed)
    sd.epoch = epoch
    out = []
    for s in range(0, n, bs):
        out.append(data.process_batch(proc, data.custom_collate([sd[i] for i in range(s, min(n, s + bs))]), prompt))
    return out


def conf_counts(masks, gt_u8, mask_values, C=14):
    """Pooled per-class (tp, fp, fn, tn) with the reference's break quirk (training_utils.py:126-134),
    sigmoid(x) > 0.5 as the reference thresholds; plain torch (oracle side)."""
    from dilabhelmholtzoct_amd.metrics import included_prompts
    B, N = masks.shape[:2]
    pred = torch.sigmoid(masks.float()) > 0.5
    g = gt_u8.to(pred.device).bool()
    tp = (pred & g).sum((2, 3)).cpu()
    fp = (pred & ~g).sum((2, 3)).cpu()
    fn = (~pred & g).sum((2, 3)).cpu()
    tn = (~pred & ~g).sum((2, 3)).cpu()
    out = torch.zeros(C, 4, dtype=torch.int64)
    for b, c in included_prompts(mask_values):
        v = int(mask_values[b, c])
        out[v] += torch.tensor([tp[b, c], fp[b, c], fn[b, c], tn[b, c]])
    return out


def summarize(conf):
    d, sp, se = [], [], []
    for tp, fp, fn, tn in conf.tolist():
        d.append(2 * tp / (2 * tp + fp + fn) if 2 * tp + fp + fn else 0.0)
        sp.append(tn / (tn + fp) if tn + fp else 0.0)
        se.append(tp / (tp + fn) if tp + fn else 0.0)
    return float(np.mean(d)), float(np.mean(sp)), float(np.mean(se))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--epochs", type=int, default=8)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--seed", type=int, default=0, help="data seed (train = 2000+seed, val = 3000+seed)")
    p.add_argument("--wseed", type=int, default=0, help="weight seed")
    p.add_argument("--ntrain", type=int, default=128)
    p.add_argument("--nval", type=int, default=32)
    p.add_argument("--bs", type=int, default=8)
    p.add_argument("--every", type=int, default=16)
    p.add_argument("--top", type=int, default=1)
    p.add_argument("--no-oracle", action="store_true")
    p.add_argument("--no-hip", action="store_true")
    p.add_argument("--ref-autocast", action="store_true", help="oracle under torch.autocast(bfloat16)")
    p.add_argument("--init", default=None, help="safetensors mask-decoder weights both sides start from")
    p.add_argument("--save-at", default="", help="comma-separated steps at which to save the oracle's decoder")
    p.add_argument("--save-dir", default=None)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep, predict_masks
    from oracle.step_ref import CpuReferenceStep, synthetic_state_dict
    name = "facebook/sam-vit-base"
    state = synthetic_state_dict(name, seed=a.wseed)
    if a.init:
        from safetensors.torch import load_file
        for kk, vv in load_file(a.init).items():
            assert kk in state and state[kk].shape == vv.shape, kk
            state[kk] = vv.float()
    save_at = {int(x) for x in a.save_at.split(",") if x}
    t0 = time.time()
    val_cpu = batches(3000 + a.seed, a.nval, a.bs, 0)
    val = [data.to_device_batch(v, dev) for v in val_cpu]
    ours = SamModel(name)
    ours.load_state_dict(state)
    ours = ours.to(dev)
    step = FusedTrainStep(ours, lr=a.lr, topological=bool(a.top), graphs=True)
    ref = None
    if not a.no_oracle:
        ref = CpuReferenceStep(name, topological=bool(a.top), lr=a.lr, state_dict=state, device=dev, loss_device=dev)
        if a.ref_autocast:  # a plain bf16 model: transformers SamModel under torch.autocast(bfloat16)
            orig_predict = ref.predict

            def predict_bf16(batch, image_embeddings=None):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    return orig_predict(batch, image_embeddings).float()
            ref.predict = predict_bf16
        val_emb = [ref.embed(v) for v in val_cpu]
    print(f"setup {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    fo = open(a.out, "w") if a.out else None

    def evaluate(k):
        step.flush()
        co = torch.zeros(14, 4, dtype=torch.int64)
        cr = torch.zeros(14, 4, dtype=torch.int64)
        for i, v in enumerate(val):
            if not a.no_hip:
                co += conf_counts(predict_masks(ours, v), v["gt_u8"], val_cpu[i]["mask_values"])
            if ref is not None:
                with torch.no_grad():
                    cr += conf_counts(ref.predict(val_cpu[i], val_emb[i]), v["gt_u8"], val_cpu[i]["mask_values"])
        d_o, sp_o, se_o = summarize(co)
        rec = {"step": k, "dice_hip": round(d_o, 5), "spec_hip": round(sp_o, 4), "sens_hip": round(se_o, 4)}
        if ref is not None:
            d_r, sp_r, se_r = summarize(cr)
            rec.update({"dice_ref": round(d_r, 5), "spec_ref": round(sp_r, 4), "sens_ref": round(se_r, 4),
                        "diff": round(d_o - d_r, 5)})
        rec["t"] = round(time.time() - t0, 1)
        print(json.dumps(rec), flush=True)
        if fo:
            fo.write(json.dumps(rec) + "\n")
            fo.flush()

    k = 0
    emb_cache = {}
    evaluate(0)
    for ep in range(a.epochs):
        tr_cpu = batches(2000 + a.seed, a.ntrain, a.bs, ep)
        tr = [data.to_device_batch(b, dev) for b in tr_cpu]
        for i, b in enumerate(tr):
            if not a.no_hip:
                step.step(b)
            if ref is not None:
                if i not in emb_cache:  # same images every epoch (no shuffle): the frozen encoder's output
                    emb_cache[i] = ref.embed(tr_cpu[i])
                ref.step(tr_cpu[i], emb_cache[i])
            k += 1
            if k % a.every == 0:
                evaluate(k)
            if k in save_at and ref is not None:
                from safetensors.torch import save_file
                sd = {"mask_decoder." + n: t.detach().to(torch.bfloat16).cpu().contiguous()  # 8 MB
                      for n, t in ref.model.mask_decoder.state_dict().items()}
                os.makedirs(a.save_dir, exist_ok=True)
                save_file(sd, os.path.join(a.save_dir, f"decoder_step{k}.safetensors"))
        del tr


if __name__ == "__main__":
    main()
