"""§8(f)3 on the GPU: octsam_confusion per-prompt counts exact vs torch, and the whole evaluate_metrics
output (metrics.EvalAccumulator: HIP counts + device AP) vs oracle/eval_ref.py (the reference's loop with
sklearn). AP: the device sigmoid may differ from the CPU one in the last ulp -> 1e-6."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_prompt_confusion_exact(cuda):
    from dilabhelmholtzoct_amd.metrics import prompt_confusion
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 14, 496, 512, generator=g)
    x[0, 0] = 0.0  # x == 0 is not > 0 (sigmoid(0) = 0.5 is not > 0.5)
    gt = (torch.rand(3, 14, 496, 512, generator=g) > 0.5).to(torch.uint8)
    got = prompt_confusion(x.to(cuda), gt.to(cuda)).cpu()
    p, t = x > 0, gt.bool()
    want = torch.stack([(p & t).sum((2, 3)), (p & ~t).sum((2, 3)), (~p & t).sum((2, 3)),
                        (~p & ~t).sum((2, 3))], -1).view(-1, 4)
    assert torch.equal(got, want)
    odd = torch.randn(5, 37, 53, generator=g)
    godd = (torch.rand(5, 37, 53, generator=g) > 0.3).to(torch.uint8)
    got = prompt_confusion(odd.to(cuda), godd.to(cuda)).cpu()
    assert int(got.sum()) == odd.numel() and int(got[:, 0].sum()) == int(((odd > 0) & godd.bool()).sum())


def test_eval_metrics_match_reference(cuda):
    import math
    from dilabhelmholtzoct_amd import metrics
    from oracle.eval_ref import evaluate_metrics_ref
    from test_eval_cpu import _assert_metrics_equal, eval_batches
    acc = metrics.EvalAccumulator()
    logits, gts, mvs = [], [], []
    for x, gt, mv in eval_batches(3):
        acc.add(x.to(cuda), gt.to(cuda), mv)
        for b in range(2):
            logits.append(x[b]), gts.append(gt[b]), mvs.append(mv[b].tolist())
    got = acc.compute()
    want = evaluate_metrics_ref(logits, gts, mvs)
    ap_got = {p: got[p].pop("ap") for p in ("category", "sample")}
    ap_want = {p: want[p].pop("ap") for p in ("category", "sample")}
    for p in ("mean", "sample_mean"):
        got[p].pop("ap"), want[p].pop("ap")
    keep = metrics.METRICS
    metrics.METRICS = tuple(k for k in keep if k != "ap")
    try:
        _assert_metrics_equal(got, want)
    finally:
        metrics.METRICS = keep
    for p in ap_got:
        for a, b in zip(ap_got[p], ap_want[p]):
            assert (math.isnan(a) and math.isnan(b)) or abs(a - b) < 1e-6, (p, a, b)
