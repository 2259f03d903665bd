"""Evaluation (A20 / §8(f)3): the package's assembly of evaluate_metrics' outputs (metrics.EvalAccumulator,
train.class_confusion's break rule) against oracle/eval_ref.py — a restatement of the reference's per-image
loop (ref:octsam/models/training_utils.py:113-134, incl. the ``break`` when a background-valued prompt
follows the first one), pooled per-class metrics (:136-156) and per-sample means (:158-192), with sklearn
for F1 / AP / confusion as the reference calls it. The per-prompt counts normally come from the HIP kernel
(tests/test_gpu_metrics.py); here a numpy count stands in so the host logic is checked on CPU."""
import math

import numpy as np
import pytest
import torch

from dilabhelmholtzoct_amd import metrics
from oracle.eval_ref import evaluate_metrics_ref


def _cpu_confusion(masks, gt):
    p = masks.float() > 0
    t = gt.bool()
    c = torch.stack([(p & t).sum((-1, -2)), (p & ~t).sum((-1, -2)), (~p & t).sum((-1, -2)),
                     (~p & ~t).sum((-1, -2))], -1)
    return c.reshape(-1, 4).long()


def eval_batches(seed=0):
    """3 batches of 2 images (H, W = 40, 48, N <= 5 with zero padding). Image 1 of batch 0 has a second
    background component at c = 1, so everything after it is dropped (the quirk); class 7 never occurs;
    class 9's gt is all-negative (AP with no positives)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    vals = [[[0, 2, 3, 5, 0], [0, 0, 3, 6, 0]], [[0, 1, 9, 0, 0], [0, 4, 5, 11, 13]],
            [[0, 2, 8, 10, 12], [0, 3, 0, 0, 0]]]
    for b in range(3):
        mv = torch.tensor(vals[b], dtype=torch.uint8)
        x = torch.randn(2, 5, 40, 48, generator=g) * 2
        gt = (torch.randn(2, 5, 40, 48, generator=g) + x * 0.7 > 0.3).to(torch.uint8)
        gt[mv == 9] = 0
        gt[mv == 0] = gt[mv == 0] * 0  # padded / background prompts: empty gt is allowed
        gt[:, 0] = (x[:, 0] > -0.5).to(torch.uint8)
        x[0, 0, :3, :3] = 40.0  # saturated scores: ties at 1.0 in the AP
        out.append((x, gt, mv))
    return out


def _assert_metrics_equal(got, want, tol=1e-9):
    for part in ("category", "sample"):
        for k in metrics.METRICS:
            for i, (a, b) in enumerate(zip(got[part][k], want[part][k])):
                if math.isnan(b):
                    assert math.isnan(a), (part, k, i, a, b)
                else:
                    assert abs(a - b) <= tol * max(1.0, abs(b)), (part, k, i, a, b)
    for part in ("mean", "sample_mean"):
        for k in metrics.METRICS:
            a, b = got[part][k], want[part][k]
            assert (math.isnan(a) and math.isnan(b)) or abs(a - b) <= tol * max(1.0, abs(b)), (part, k, a, b)


def test_eval_accumulator_matches_reference_loop(monkeypatch):
    monkeypatch.setattr(metrics, "prompt_confusion", _cpu_confusion)
    acc = metrics.EvalAccumulator()
    logits, gts, mvs = [], [], []
    for x, gt, mv in eval_batches():
        acc.add(x, gt, mv)
        for b in range(2):
            logits.append(x[b]), gts.append(gt[b]), mvs.append(mv[b].tolist())
    got = acc.compute()
    want = evaluate_metrics_ref(logits, gts, mvs)
    _assert_metrics_equal(got, want)
    assert got["category"]["iou"][7] == 0.0 and got["category"]["ap"][9] == want["category"]["ap"][9]
    # the break quirk: image 1 of batch 0 keeps only its first prompt
    assert [p for p in metrics.included_prompts(eval_batches()[0][2]) if p[0] == 1] == [(1, 0)]


def test_class_confusion_and_mean_dice_match_reference(monkeypatch):
    """train.class_confusion / mean_dice (the bench's and the val-Dice test's metric) = the reference's
    per-class pooled Dice and its mean over the 14 classes (:156, :246)."""
    from dilabhelmholtzoct_amd import train
    monkeypatch.setattr(metrics, "prompt_confusion", _cpu_confusion)
    conf = torch.zeros(14, 3, dtype=torch.int64)
    logits, gts, mvs = [], [], []
    for x, gt, mv in eval_batches(1):
        conf += train.class_confusion(x, gt, mv)
        for b in range(2):
            logits.append(x[b]), gts.append(gt[b]), mvs.append(mv[b].tolist())
    want = evaluate_metrics_ref(logits, gts, mvs)
    assert abs(train.mean_dice(conf) - float(np.mean(want["category"]["dice"]))) < 1e-12
    assert train.class_dice(conf) == pytest.approx(want["category"]["dice"], abs=1e-12)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_average_precision_matches_sklearn(seed):
    from sklearn.metrics import average_precision_score
    rng = np.random.default_rng(seed)
    s = rng.random(5000).astype(np.float32)
    s[:800] = np.round(s[:800] * 10) / 10  # ties
    y = (rng.random(5000) < s).astype(np.uint8)
    got = metrics.average_precision(torch.from_numpy(s), torch.from_numpy(y))
    assert abs(got - average_precision_score(y, s)) < 1e-12
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want0 = average_precision_score(np.zeros(100), s[:100])
    assert metrics.average_precision(torch.from_numpy(s[:100]), torch.zeros(100)) == want0
