"""Host-side logic of the product path, checked on CPU:
* the post-processing interpolation tables (losses._composite_1d / _pp_tables_host) against torch's own
  F.interpolate chain (ref:octsam/models/training_utils.py:56-58 via HF post_process_masks);
* the host exact Wasserstein solver (octsam_w2_host, C-ABI, CPU) against the oracle's
  diagonal-augmented linear_sum_assignment + torch autograd restatement of torch_topological's
  WassersteinDistance(q=2, p=inf);
* the oracle's DiceCE restatement (monai 1.3.0 DiceCELoss(sigmoid=True)) on closed-form cases;
* topo_entries (batch_iter nesting) and the training-loop reductions."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from dilabhelmholtzoct_amd import kernels as K
from dilabhelmholtzoct_amd import losses
from oracle.losses_ref import _wasserstein_ref, dicece_ref, topo_entries as topo_entries_ref


@pytest.mark.parametrize("crop,orig", [((992, 1024), (496, 512)), ((853, 1024), (160, 192)), ((1024, 768), (1024, 768))])
def test_postproc_tables_match_interpolate(crop, orig):
    S = 256
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, 1, S, S, generator=g, dtype=torch.float32)
    ref = F.interpolate(x, (1024, 1024), mode="bilinear", align_corners=False)[..., : crop[0], : crop[1]]
    ref = F.interpolate(ref, orig, mode="bilinear", align_corners=False)[0, 0].double()
    Wy = torch.from_numpy(losses._composite_1d(S, 1024, crop[0], orig[0])).double()
    Wx = torch.from_numpy(losses._composite_1d(S, 1024, crop[1], orig[1])).double()
    got = Wy @ x[0, 0].double() @ Wx.T
    assert (got - ref).abs().max().item() < 2e-5
    (cptr, cidx, cw), (rptr, ridx, rw) = losses._pp_tables_host(S, 1024, crop[0], crop[1], orig[0], orig[1])
    assert cptr[-1] == len(cidx) == len(cw) and rptr[-1] == len(ridx)
    dense = np.zeros((orig[1], S), np.float32)
    for a in range(S):
        dense[cidx[cptr[a]:cptr[a + 1]], a] = cw[cptr[a]:cptr[a + 1]]
    assert np.array_equal(dense, losses._composite_1d(S, 1024, crop[1], orig[1]))


def _diag(rng, n, lo=0.0, hi=1.0):
    b = rng.uniform(lo, hi, n)
    d = b + rng.uniform(0.01, 0.5, n)
    return np.stack([b, d], 1).astype(np.float32)


@pytest.mark.parametrize("n,m", [(0, 0), (0, 3), (4, 0), (1, 1), (5, 7), (9, 2), (30, 41), (120, 3)])
def test_w2_host_matches_oracle(n, m):
    rng = np.random.default_rng(n * 100 + m)
    d1, d2 = _diag(rng, n), _diag(rng, m)
    cost, grad = K.w2_host(d1, d2, 2.0)
    D1 = torch.tensor(d1, dtype=torch.float64, requires_grad=True)
    ref = _wasserstein_ref(D1, torch.tensor(d2, dtype=torch.float64), 2.0)
    assert math.isclose(cost, float(ref.detach()), rel_tol=1e-5, abs_tol=1e-7)
    if n:
        ref.backward()
        np.testing.assert_allclose(grad, D1.grad.numpy(), rtol=1e-4, atol=1e-5)


def test_w2_host_symmetric_cost_and_diagonal_only():
    d1 = np.array([[0.1, 0.9], [0.2, 0.25]], np.float32)
    cost, grad = K.w2_host(d1, np.zeros((0, 2), np.float32), 2.0)
    # every point to the diagonal: (death - birth)/2 under p = inf, squared
    assert math.isclose(cost, 0.4 ** 2 + 0.025 ** 2, rel_tol=1e-5)
    np.testing.assert_allclose(grad, [[-0.4, 0.4], [-0.025, 0.025]], rtol=1e-4)
    rng = np.random.default_rng(3)
    a, b = _diag(rng, 6), _diag(rng, 8)
    assert math.isclose(K.w2_host(a, b)[0], K.w2_host(b, a)[0], rel_tol=1e-5)


def test_dicece_ref_closed_form():
    # logits 0 -> p = 1/2 everywhere; one prompt (N = 1): CE over a single class is exactly 0
    x = torch.zeros(2, 1, 4, 5, dtype=torch.float64)
    t = torch.zeros_like(x)
    t[:, :, :2] = 1.0  # 10 of 20 pixels
    inter, g, pr = 0.5 * 10, 10.0, 10.0
    dice = 1 - (2 * inter + 1e-5) / (g + pr + 1e-5)
    assert math.isclose(float(dicece_ref(x, t)), dice, rel_tol=1e-12)
    # two prompts with probability targets: CE = -sum_c t_c log softmax(x)_c averaged over pixels and batch
    x = torch.tensor([[[[2.0]], [[0.0]]]], dtype=torch.float64)
    t = torch.tensor([[[[1.0]], [[0.0]]]], dtype=torch.float64)
    ce = -math.log(math.exp(2) / (math.exp(2) + 1))
    p0, p1 = 1 / (1 + math.exp(-2)), 0.5
    dice = ((1 - (2 * p0 + 1e-5) / (1 + p0 + 1e-5)) + (1 - 1e-5 / (p1 + 1e-5))) / 2
    assert math.isclose(float(dicece_ref(x, t)), dice + ce, rel_tol=1e-12)


@pytest.mark.parametrize("B,N", [(1, 5), (4, 1), (3, 4), (1, 1)])
@pytest.mark.parametrize("mode", ["first", "all"])
def test_topo_entries(B, N, mode):
    assert losses.topo_entries(B, N, mode) == topo_entries_ref(B, N, mode)
    ent = losses.topo_entries(B, N, mode)
    flat = [k for e in ent for k in e]
    assert len(set(flat)) == len(flat) and all(0 <= k < B * N for k in flat)
    if B == 1:
        assert len(ent) == N
    elif N == 1 or mode == "first":
        assert len(ent) == B


def test_dicece_pp_rows_supported_limits():
    """The fused DiceCE / row-pass kernel's limits as the host checks them before choosing it (train._dicece falls back
    to the two-kernel path outside them): N <= 32 prompts, W % 4 == 0, W <= 1024."""
    from dilabhelmholtzoct_amd.losses import dicece_pp_rows_supported
    assert dicece_pp_rows_supported(8, 21, 496, 512)
    assert dicece_pp_rows_supported(8, 32, 496, 512)
    assert not dicece_pp_rows_supported(8, 33, 496, 512)
    assert not dicece_pp_rows_supported(8, 21, 496, 510)
    assert not dicece_pp_rows_supported(1, 2, 100, 2048)
    assert not dicece_pp_rows_supported(8, 0, 496, 512)
