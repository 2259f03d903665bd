"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

CPU restatement of the reference's evaluation, ref:octsam/models/training_utils.py:82-270 (evaluate_metrics),
from the post-processed mask logits on: the per-image loop with sigmoid > 0.5 and the ``break`` when a
background-valued prompt follows the first one (:113-134), then per class the pooled metrics (:136-156) and
the per-sample means (:158-192), and the means over classes (:236-270).

Third-party pieces: ``evaluate.load("mean_iou")`` (hub metric, not installed) is restated from its published
algorithm (intersect / union and intersect / label area per category, numpy division -> NaN on 0/0,
category 1 of num_labels=2); sklearn (installed here, 1.7) is called directly for f1_score,
average_precision_score and confusion_matrix exactly as the reference calls them.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch


def _mean_iou_cat1(preds: list, refs: list):
    """evaluate mean_iou(num_labels=2, ignore_index=255, reduce_labels=False): (iou[1], accuracy[1])."""
    inter = union = label = 0
    for p, r in zip(preds, refs):
        p = np.asarray(p).astype(np.int64)
        r = np.asarray(r).astype(np.int64)
        keep = r != 255
        p, r = p[keep], r[keep]
        i1 = int(np.sum((p == r) & (r == 1)))
        a_p, a_l = int(np.sum(p == 1)), int(np.sum(r == 1))
        inter += i1
        union += a_p + a_l - i1
        label += a_l
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.float64(inter) / np.float64(union)), float(np.float64(inter) / np.float64(label))


def evaluate_metrics_ref(mask_logits: list, gt_masks: list, mask_values: list, num_classes: int = 14) -> dict:
    """mask_logits[i]: [N_i, H, W] post-processed logits of test image i (its own prompts, unpadded or
    zero-padded), gt_masks[i]: [N_i, H, W] 0/1, mask_values[i]: [N_i]. Same output layout as
    dilabhelmholtzoct_amd.metrics.EvalAccumulator.compute()."""
    import sklearn.metrics as skm
    seg = [[] for _ in range(num_classes)]
    prob = [[] for _ in range(num_classes)]
    gts = [[] for _ in range(num_classes)]
    for x, g, mv in zip(mask_logits, gt_masks, mask_values):
        masks = torch.sigmoid(torch.as_tensor(x).float()).numpy()
        binary = (masks > 0.5).astype(np.uint8)
        for c in range(len(mv)):
            if mv[c] == 0 and c > 0:
                break
            seg[int(mv[c])].append(binary[c])
            prob[int(mv[c])].append(masks[c])
            gts[int(mv[c])].append(np.asarray(g[c]))
    keys = ("accuracy", "iou", "specificity", "sensitivity", "f1", "dice", "ap")
    # the reference's result arrays start as np.zeros(14) (:94-107); a class without samples keeps 0 (the
    # reference itself would stop in sklearn's confusion_matrix unpacking there)
    cat = {k: [0.0] * num_classes for k in keys}
    smp = {k: [0.0] * num_classes for k in keys}

    def conf(gt_flat, seg_flat):
        return skm.confusion_matrix(gt_flat, seg_flat, labels=[0, 1]).ravel()

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i in range(num_classes):
            if not seg[i]:
                continue
            iou, acc = _mean_iou_cat1(seg[i], gts[i])
            cat["accuracy"][i], cat["iou"][i] = acc, iou
            fg = np.array(gts[i]).reshape(-1)
            fs = np.array(seg[i]).reshape(-1)
            fp_ = np.array(prob[i]).reshape(-1)
            cat["f1"][i] = float(skm.f1_score(fg, fs))
            cat["ap"][i] = float(skm.average_precision_score(fg, fp_))
            tn, fp, fn, tp = conf(fg, fs)
            cat["sensitivity"][i] = tp / (tp + fn) if (tp + fn) != 0 else 0.0
            cat["specificity"][i] = tn / (tn + fp) if (tn + fp) != 0 else 0.0
            cat["dice"][i] = 2 * tp / (2 * tp + fp + fn) if (2 * tp + fp + fn) != 0 else 0.0
            per = {k: [] for k in keys}
            for j in range(len(seg[i])):
                iou_j, acc_j = _mean_iou_cat1([seg[i][j]], [gts[i][j]])
                fg = np.array(gts[i][j]).reshape(-1)
                fs = np.array(seg[i][j]).reshape(-1)
                fp_ = np.array(prob[i][j]).reshape(-1)
                tn, fp, fn, tp = conf(fg, fs)
                per["iou"].append(iou_j)
                per["accuracy"].append(acc_j)
                per["specificity"].append(tn / (tn + fp) if (tn + fp) != 0 else 0.0)
                per["sensitivity"].append(tp / (tp + fn) if (tp + fn) != 0 else 0.0)
                per["f1"].append(float(skm.f1_score(fg, fs)))
                per["dice"].append(2 * tp / (2 * tp + fp + fn) if (2 * tp + fp + fn) != 0 else 0.0)
                per["ap"].append(float(skm.average_precision_score(fg, fp_)))
            for k in keys:
                smp[k][i] = float(np.mean(per[k]))
    mean = {k: float(np.mean(cat[k])) for k in keys}
    smean = {k: float(np.mean(smp[k])) for k in keys}
    return {"category": cat, "sample": smp, "mean": mean, "sample_mean": smean}


def pooled_confusion_ref(mask_logits: torch.Tensor, gt_u8: torch.Tensor, mask_values, num_classes: int = 14):
    """Per-class pooled (tp, fp, fn, tn) int64 [C, 4] of sigmoid(logits) > 0.5 (:126-127) against the 0/1 gt, with
    the break quirk (:128-130): the counts evaluate_metrics_ref's confusion_matrix calls pool, in plain torch (any
    device) for the long val-Dice parity test. mask_logits / gt_u8 [B, N, H, W], mask_values [B, N]."""
    mv = np.asarray(mask_values.cpu() if isinstance(mask_values, torch.Tensor) else mask_values)
    pred = torch.sigmoid(mask_logits.float()) > 0.5
    g = gt_u8.to(pred.device).bool()
    cnt = torch.stack([(pred & g).sum((2, 3)), (pred & ~g).sum((2, 3)), (~pred & g).sum((2, 3)),
                       (~pred & ~g).sum((2, 3))], -1).cpu()
    out = torch.zeros(num_classes, 4, dtype=torch.int64)
    for b in range(mv.shape[0]):
        for c in range(mv.shape[1]):
            if mv[b, c] == 0 and c > 0:
                break
            out[int(mv[b, c])] += cnt[b, c]
    return out


def mean_dice_ref(pooled: torch.Tensor) -> float:
    """"Mean dice" (:156, :246): mean over the classes of 2tp / (2tp + fp + fn), 0 for an empty class."""
    d = [2 * tp / (2 * tp + fp + fn) if (2 * tp + fp + fn) else 0.0 for tp, fp, fn, _ in pooled.tolist()]
    return float(np.mean(d))


def mean_specificity_ref(pooled: torch.Tensor) -> float:
    """Mean over the classes of tn / (tn + fp) (:150-153), 0 for an empty class."""
    d = [tn / (tn + fp) if (tn + fp) else 0.0 for tp, fp, fn, tn in pooled.tolist()]
    return float(np.mean(d))
