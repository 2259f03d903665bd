"""Evaluation metrics of the OCT-SAM reference on the GPU.

``evaluate_metrics`` (ref:octsam/models/training_utils.py:82-270) runs the model per test image, thresholds
sigmoid(mask) > 0.5 (:126-127) and pools the prompts of every class with an early ``break`` when a
background-valued prompt follows the first one (:128-134). Per class it reports, pooled over all the class's
pixels (:136-156) and as the mean over the class's samples (:158-192):

  * IoU and accuracy of category 1 from ``evaluate.load("mean_iou")`` (num_labels=2): tp/(tp+fp+fn) and
    tp/(tp+fn), NaN when the denominator is 0 (numpy division, as that metric computes them);
  * F1 = sklearn.metrics.f1_score (binary, zero_division -> 0);
  * sensitivity tp/(tp+fn), specificity tn/(tn+fp), Dice 2tp/(2tp+fp+fn), each 0 on an empty denominator;
  * AP = sklearn.metrics.average_precision_score(gt, sigmoid(mask)) — step-wise precision-recall area
    over the distinct scores (no positives: recall is set to one, AP = 0);

and the mean of each over the 14 classes ("Mean dice" :246,251 is the north_star's val-Dice metric).

Here the confusion counts of every prompt come from one HIP kernel (``octsam_confusion``: 16 B of logits and
4 B of gt per lane, integer atomics, exact); the AP needs the scores in order, which is a device sort
(torch.sort, rocPRIM) + cumulative sums. evaluate and sklearn are not needed (evaluate is not installed).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

NUM_CLASSES = 14
METRICS = ("accuracy", "iou", "specificity", "sensitivity", "f1", "dice", "ap")


def prompt_confusion(masks: torch.Tensor, gt_u8: torch.Tensor) -> torch.Tensor:
    """masks fp32 [..., H, W] logits, gt uint8 of the same shape (device) -> int64 [M, 4] (tp, fp, fn, tn)
    on the device, M = prod of the leading dims."""
    if masks.shape != gt_u8.shape or masks.dim() < 2:
        raise ValueError(f"masks {tuple(masks.shape)} and gt {tuple(gt_u8.shape)} must match")
    if not masks.is_cuda or not gt_u8.is_cuda:
        raise ValueError("prompt_confusion needs device tensors (liboctsam_hip.so)")
    x = masks.float().contiguous()
    g = gt_u8.to(torch.uint8).contiguous()
    HW = x.shape[-1] * x.shape[-2]
    M = x.numel() // HW
    out = torch.empty(M, 4, device=x.device, dtype=torch.int64)
    for m0 in range(0, M, 65535):
        m1 = min(M, m0 + 65535)
        _lib.call("octsam_confusion", _lib.ptr(x.view(M, HW)[m0:m1]), _lib.ptr(g.view(M, HW)[m0:m1]), m1 - m0, HW,
                  _lib.ptr(out[m0:m1]))
    return out


def included_prompts(mask_values) -> list:
    """(b, c) pairs evaluate_metrics keeps: per image, prompts in order until a background-valued prompt at
    c > 0 (:128-130; the collate's zero padding ends the list the same way)."""
    mv = np.asarray(mask_values.cpu() if isinstance(mask_values, torch.Tensor) else mask_values)
    out = []
    for b in range(mv.shape[0]):
        for c in range(mv.shape[1]):
            if int(mv[b, c]) == 0 and c > 0:
                break
            out.append((b, c))
    return out


def _div_nan(a, b):
    return a / b if b else float("nan")


def _div_zero(a, b):
    return a / b if b else 0.0


def confusion_metrics(tp, fp, fn, tn) -> dict:
    """The per-class / per-sample scalar metrics of :145-156 / :177-183 from one confusion count."""
    tp, fp, fn, tn = (int(v) for v in (tp, fp, fn, tn))
    return {"accuracy": _div_nan(tp, tp + fn), "iou": _div_nan(tp, tp + fp + fn),
            "specificity": _div_zero(tn, tn + fp), "sensitivity": _div_zero(tp, tp + fn),
            "f1": _div_zero(2 * tp, 2 * tp + fp + fn), "dice": _div_zero(2 * tp, 2 * tp + fp + fn)}


@torch.no_grad()
def average_precision(scores: torch.Tensor, labels: torch.Tensor) -> float:
    """sklearn.metrics.average_precision_score(labels, scores) on the device: sum over distinct score
    thresholds (descending) of (R_k - R_{k-1}) * P_k."""
    s = scores.reshape(-1).float()
    y = labels.reshape(-1).to(torch.int64)
    n = s.numel()
    if n == 0:
        return float("nan")
    s_sorted, order = torch.sort(s, descending=True, stable=True)
    tps = torch.cumsum(y[order], 0)
    last = torch.ones(n, dtype=torch.bool, device=s.device)
    last[:-1] = s_sorted[1:] != s_sorted[:-1]
    idx = torch.nonzero(last).view(-1)
    tp_k = tps[idx].double()
    fp_k = (idx + 1).double() - tp_k
    P = float(tps[-1])
    prec = tp_k / (tp_k + fp_k)
    if P == 0:  # sklearn: "No positive class found in y_true, recall is set to one for all thresholds"
        rec = torch.ones_like(tp_k)
    else:
        rec = tp_k / P
    prev = torch.cat([torch.zeros(1, dtype=rec.dtype, device=rec.device), rec[:-1]])
    return float(((rec - prev) * prec).sum())


class EvalAccumulator:
    """Collects evaluate_metrics' per-class samples batch by batch (device), then computes every metric.

    add(masks, gt_u8, mask_values): masks fp32 [B, N, H, W] post-processed logits, gt uint8 [B, N, H, W]
    (device), mask_values [B, N]. keep_scores=False skips the AP (no logits kept)."""

    def __init__(self, num_classes: int = NUM_CLASSES, keep_scores: bool = True):
        self.C = num_classes
        self.keep_scores = keep_scores
        self.counts = [[] for _ in range(num_classes)]  # per class: list of (tp, fp, fn, tn)
        self.scores = [[] for _ in range(num_classes)]  # per class: list of (logits row, gt row), host memory
        self.samples = [[] for _ in range(num_classes)]  # per class: image index of each sample (:134)
        self.n_images = 0
        self.device = torch.device("cpu")

    def add(self, masks: torch.Tensor, gt_u8: torch.Tensor, mask_values, image_index=None):
        B, N = masks.shape[:2]
        conf = prompt_confusion(masks, gt_u8).view(B, N, 4).cpu().numpy()
        mv = np.asarray(mask_values.cpu() if isinstance(mask_values, torch.Tensor) else mask_values)
        for b, c in included_prompts(mv):
            v = int(mv[b, c])
            self.counts[v].append(tuple(int(t) for t in conf[b, c]))
            self.samples[v].append(self.n_images + b if image_index is None else image_index[b])
            if self.keep_scores:  # host memory, as the reference keeps its arrays (HBM stays free)
                self.scores[v].append((masks[b, c].float().cpu(), gt_u8[b, c].cpu()))
        self.n_images += B
        self.device = masks.device

    def pooled_confusion(self) -> torch.Tensor:
        """int64 [C, 4] pooled (tp, fp, fn, tn) per class."""
        out = torch.zeros(self.C, 4, dtype=torch.int64)
        for v in range(self.C):
            if self.counts[v]:
                out[v] = torch.tensor(self.counts[v], dtype=torch.int64).sum(0)
        return out

    def compute(self) -> dict:
        """{"category": {metric: [C]}, "sample": {metric: [C]}, "mean": {metric}, "sample_mean": {metric}}."""
        # np.zeros(14) result arrays (:94-107): a class without samples reports 0
        cat = {k: [0.0] * self.C for k in METRICS}
        smp = {k: [0.0] * self.C for k in METRICS}
        pooled = self.pooled_confusion()
        for v in range(self.C):
            if not self.counts[v]:
                continue
            m = confusion_metrics(*pooled[v].tolist())
            for k in m:
                cat[k][v] = m[k]
            per = [confusion_metrics(*c) for c in self.counts[v]]
            for k in per[0]:
                smp[k][v] = float(np.mean([p[k] for p in per]))
            if self.keep_scores:  # one class's scores on the device at a time
                dev = self.device
                xs = torch.cat([x.reshape(-1) for x, _ in self.scores[v]]).to(dev)
                ys = torch.cat([y.reshape(-1) for _, y in self.scores[v]]).to(dev)
                cat["ap"][v] = average_precision(torch.sigmoid(xs), ys)
                del xs, ys
                smp["ap"][v] = float(np.mean([average_precision(torch.sigmoid(x.to(dev)), y.to(dev))
                                              for x, y in self.scores[v]]))
        mean = {k: float(np.mean(cat[k])) for k in METRICS}
        smean = {k: float(np.mean(smp[k])) for k in METRICS}
        return {"category": cat, "sample": smp, "mean": mean, "sample_mean": smean}


def mean_dice_from_counts(pooled: torch.Tensor) -> float:
    """'Mean dice' (:156,246): mean over classes of 2tp/(2tp+fp+fn), 0 on an empty denominator."""
    d = [_div_zero(2 * tp, 2 * tp + fp + fn) for tp, fp, fn, _ in pooled.tolist()]
    return sum(d) / len(d)
