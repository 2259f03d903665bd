"""Post-processing (training_utils.py:57-59: bilinear 256->1024, crop, bilinear -> original size) and DiceCE
(training_utils.py:32,62; monai 1.3.0 DiceCELoss restated in oracle/losses_ref.py) on the GPU kernels:
forward against torch F.interpolate on the same fp32 input, backward against autograd of that chain, the
fused Dice partial sums and the DiceCE loss / gradient against the oracle. fp32 throughout: tolerance 1e-5
relative (1e-9 on the loss, accumulated in double)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _chain(low, crop, orig):
    up = F.interpolate(low, size=(1024, 1024), mode="bilinear", align_corners=False)
    return F.interpolate(up[..., :crop[0], :crop[1]], size=orig, mode="bilinear", align_corners=False)


@pytest.mark.parametrize("crop,orig", [((1024, 992), (496, 512)), ((700, 1024), (350, 513)), ((1024, 1024), (300, 300))])
def test_postproc_fwd_bwd(cuda, crop, orig):
    from dilabhelmholtzoct_amd.losses import postproc_backward, postproc_forward
    g = torch.Generator().manual_seed(crop[0] + orig[1])
    M = 5
    low = torch.randn(M, 256, 256, generator=g).to(cuda)
    gt = (torch.rand(M, *orig, generator=g) > 0.6).to(cuda, torch.uint8)
    out, part = postproc_forward(low, crop, orig, gt)
    lr = low.clone().requires_grad_()
    ref = _chain(lr[:, None], crop, orig)[:, 0]
    scale = ref.abs().max().item()
    assert (out - ref).abs().max().item() < 1e-5 * scale
    p, t = torch.sigmoid(ref.detach()), gt.float()
    sums = torch.stack([(p * t).sum((1, 2)), t.sum((1, 2)), p.sum((1, 2))], 1)
    assert torch.allclose(part.sum(1), sums, rtol=1e-4)
    dout = torch.randn(M, *orig, generator=g).to(cuda)
    ref.backward(dout)
    dlow = postproc_backward(dout, 256, crop, orig)
    assert (dlow - lr.grad).abs().max().item() < 1e-5 * lr.grad.abs().max().item()


def test_dicece_matches_oracle(cuda):
    from dilabhelmholtzoct_amd.losses import dicece_forward_backward, postproc_forward
    from oracle.losses_ref import dicece_ref
    g = torch.Generator().manual_seed(7)
    B, N, crop, orig = 2, 5, (1024, 992), (496, 512)
    low = torch.randn(B * N, 256, 256, generator=g).to(cuda)
    gt = (torch.rand(B, N, *orig, generator=g) > 0.7).to(cuda, torch.uint8)
    masks, part = postproc_forward(low, crop, orig, gt.view(B * N, *orig))
    masks = masks.view(B, N, *orig)
    loss, dmask = dicece_forward_backward(masks, gt, part)
    x = masks.detach().double().cpu().requires_grad_()
    ref = dicece_ref(x, gt.double().cpu())
    ref.backward()
    r = float(ref.detach())
    assert abs(float(loss[2]) - r) < 1e-9 + 1e-6 * abs(r)
    assert (dmask.double().cpu() - x.grad).abs().max().item() < 1e-5 * x.grad.abs().max().item()


# ------------------------------------------------------------------------------ topological loss
# ref:octsam/models/topological_loss.py:11-96 vs oracle.losses_ref.topo_loss_ref (+ torch autograd).
# Exact-grid inputs: 99x99 maps resampled to 50x50 with align_corners=True sample every other pixel
# exactly (scale 98/49 = 2, zero fractional weights), so both sides see bit-identical 50x50 maps and the
# persistence pairs must agree; only the fp32 / fp64 summation order of W2 differs -> rtol 1e-5.
def _prob_maps(B, N, S, seed, plateaus=True):
    g = torch.Generator().manual_seed(seed)
    low = torch.randn(B * N, 1, 12, 12, generator=g)
    f = F.interpolate(low, (S, S), mode="bicubic", align_corners=True)[:, 0]
    f = f + 0.05 * torch.randn(B * N, S, S, generator=g)
    p = torch.sigmoid(20.0 * f + 3.0)  # saturated regions: exact 1.0 plateaus
    if plateaus:  # exact 0 / 1 rectangles (sigmoid of +-120 in fp32)
        p[:, 10:30, 10:31] = 1.0
        p[:, 60:82, 50:90] = 0.0
    gt = (F.interpolate(torch.randn(B * N, 1, 8, 8, generator=g), (S, S), mode="bilinear",
                        align_corners=True)[:, 0] > 0.3)
    return p.reshape(B, N, S, S).contiguous(), gt.reshape(B, N, S, S).to(torch.uint8)


def _assert_grad_close(got, want, rtol=1e-5):
    scale = want.abs().max().item()
    assert scale > 0
    err = (got - want).abs().max().item()
    assert err <= rtol * scale, (err, scale)


@pytest.mark.parametrize("B,N,mode", [(1, 5, "first"), (4, 3, "first"), (4, 3, "all"), (1, 1, "first"),
                                      (3, 1, "first")])
def test_topo_loss_matches_oracle(cuda, B, N, mode):
    """Drop-in losses.topo_loss (autograd) vs the oracle: value and d loss / d pred, B == 1 per-prompt
    nesting and B > 1 per-image nesting ("first" / "all" readings of batch_iter), exact 0/1 plateaus."""
    from dilabhelmholtzoct_amd import losses
    from oracle.losses_ref import topo_loss_ref
    pred, gt = _prob_maps(B, N, 99, seed=B * 10 + N)
    x = pred.to(cuda).requires_grad_()
    got = losses.topo_loss(x, gt.to(cuda), 0.1, interp=50, feat_d=1, mode=mode)
    got.backward()
    xr = pred.clone().requires_grad_()
    want = topo_loss_ref(xr, gt.float(), 0.1, interp=50, feat_d=1, mode=mode)
    want.backward()
    assert float(want.detach()) > 0
    assert abs(float(got) - float(want.detach())) <= 1e-5 * abs(float(want.detach()))
    _assert_grad_close(x.grad.cpu(), xr.grad)


@pytest.mark.parametrize("feat_d,loss_r", [(0, False), (1, True), (0, True)])
def test_topo_loss_dims_and_regulariser(cuda, feat_d, loss_r):
    """H0 diagrams (with the essential class paired to the argmax, torch_topological's CubicalComplex) and
    the total-persistence regulariser loss_r (topological_loss.py:88-94), vs the oracle."""
    from dilabhelmholtzoct_amd import losses
    from oracle.losses_ref import topo_loss_ref
    pred, gt = _prob_maps(2, 3, 99, seed=5 + feat_d)
    x = pred.to(cuda).requires_grad_()
    got = losses.topo_loss(x, gt.to(cuda), 0.1, interp=50, feat_d=feat_d, loss_r=loss_r)
    got.backward()
    xr = pred.clone().requires_grad_()
    want = topo_loss_ref(xr, gt.float(), 0.1, interp=50, feat_d=feat_d, loss_r=loss_r)
    want.backward()
    assert abs(float(got) - float(want)) <= 1e-5 * abs(float(want))
    _assert_grad_close(x.grad.cpu(), xr.grad)


def test_topo_loss_interp0_and_feat_d2(cuda):
    """interp=0 (no resampling, :48-52) on maps the kernel accepts; feat_d=2 (the signature default) selects
    no pairs of a 2-D map, so the loss is 0 like gudhi's empty H2 diagrams."""
    from dilabhelmholtzoct_amd import losses
    from oracle.losses_ref import topo_loss_ref
    pred, gt = _prob_maps(1, 3, 40, seed=9, plateaus=False)
    x = pred.to(cuda).requires_grad_()
    got = losses.topo_loss(x, gt.to(cuda), 0.1, interp=0, feat_d=1)
    got.backward()
    xr = pred.clone().requires_grad_()
    want = topo_loss_ref(xr, gt.float(), 0.1, interp=0, feat_d=1)
    want.backward()
    assert abs(float(got) - float(want)) <= 1e-5 * abs(float(want))
    _assert_grad_close(x.grad.cpu(), xr.grad)
    assert float(losses.topo_loss(x, gt.to(cuda), 0.1, interp=50)) == 0.0  # feat_d=2 default
    with pytest.raises(NotImplementedError):
        losses.topo_loss(torch.rand(1, 1, 128, 128, device=cuda), torch.zeros(1, 1, 128, 128, device=cuda), 0.1,
                         feat_d=1)


def test_topo_checkerboard_does_not_overflow(cuda):
    """Verdict r1: a 50x50 checkerboard-like map (~1150 H1 pairs) raised mid-training with 1024 records."""
    from dilabhelmholtzoct_amd import losses
    yy, xx = torch.meshgrid(torch.arange(99), torch.arange(99), indexing="ij")
    cb = ((yy // 2 + xx // 2) % 2).float()  # 2x2 cells -> a 50x50 checkerboard after the exact resampling
    pred = (0.2 + 0.6 * cb + 0.01 * torch.rand(99, 99, generator=torch.Generator().manual_seed(0)))[None, None]
    gt = torch.zeros(1, 1, 99, 99, dtype=torch.uint8)
    loss = losses.topo_forward_backward(pred.to(cuda), gt.to(cuda), None, interp=50, logits=False)
    assert loss > 0


@pytest.mark.parametrize("B,N,mode", [(1, 6, "first"), (4, 5, "first"), (4, 5, "all")])
def test_topo_training_path_matches_oracle(cuda, B, N, mode):
    """The training step's form (logits, sigmoid fused, 496x512 -> 50x50, training_utils.py:64), staged:
    (a) the resampled sigmoid maps vs F.interpolate(torch.sigmoid) (the HIP sigmoid differs in the last
    ulp); (b) from the SAME 50x50 maps, loss and d loss / d map vs the oracle's PH + W2 + autograd;
    (c) the scatter back through the resampling and the sigmoid vs autograd of that chain; (d) the end-to-end
    loss value vs the oracle from the logits (continuous in the maps: rtol 1e-4)."""
    from dilabhelmholtzoct_amd import losses
    from oracle.losses_ref import topo_loss_ref
    g = torch.Generator().manual_seed(B * 7 + N)
    low = torch.randn(B * N, 1, 16, 16, generator=g) * 6.0
    masks = F.interpolate(low, (496, 512), mode="bilinear", align_corners=False).reshape(B, N, 496, 512)
    masks = masks + 0.3 * torch.randn(B, N, 496, 512, generator=g)
    gt = (F.interpolate(torch.randn(B * N, 1, 10, 10, generator=g), (496, 512), mode="bilinear",
                        align_corners=False) > 0.2).reshape(B, N, 496, 512).to(torch.uint8)
    mc, gc = masks.to(cuda).contiguous(), gt.to(cuda).contiguous()
    entries, maps, midx = losses.topo_index(B, N, mode, None, cuda)
    pairs, cnt, both = losses.topo_device_forward(mc, gc, midx, interp=50)
    Kn = len(maps)
    flat = masks.reshape(B * N, 1, 496, 512)
    ref_p = F.interpolate(torch.sigmoid(flat[maps]), (50, 50), mode="bilinear", align_corners=True)[:, 0]
    ref_t = F.interpolate(gt.reshape(B * N, 1, 496, 512)[maps].float(), (50, 50), mode="bilinear",
                          align_corners=True)[:, 0]
    bh = both.cpu().view(2 * Kn, 50, 50)
    assert (bh[:Kn] - ref_p).abs().max().item() < 1e-6                              # (a)
    assert (bh[Kn:] - ref_t).abs().max().item() < 1e-6
    loss, dpred = losses.topo_host(pairs.cpu().numpy(), cnt.cpu().numpy(), both.cpu().numpy(), entries, maps)
    # (b) oracle on the same 50x50 maps: place them at their (b, n) slots, interp=0
    pm = torch.zeros(B * N, 50, 50)
    tm = torch.zeros(B * N, 50, 50)
    pm[maps], tm[maps] = bh[:Kn], bh[Kn:]
    pm.requires_grad_()
    want = topo_loss_ref(pm.view(B, N, 50, 50), tm.view(B, N, 50, 50), 0.1, interp=0, feat_d=1, mode=mode)
    want.backward()
    assert abs(loss - float(want)) <= 1e-5 * abs(float(want))
    _assert_grad_close(torch.from_numpy(dpred).view(Kn, 50, 50), pm.grad[maps])
    # (c) scatter through resampling + sigmoid
    dmask = torch.zeros_like(mc)
    dp = torch.from_numpy(dpred).to(cuda)
    losses.topo_device_backward(mc, midx, dp, dmask)
    xr = flat[maps].clone().requires_grad_()
    F.interpolate(torch.sigmoid(xr), (50, 50), mode="bilinear", align_corners=True)[:, 0].backward(
        torch.from_numpy(dpred).view(Kn, 50, 50))
    want_dm = torch.zeros(B * N, 496, 512)
    want_dm[maps] = xr.grad[:, 0]
    _assert_grad_close(dmask.cpu().view(B * N, 496, 512), want_dm)
    # (d) end to end from the logits: the maps differ by the sigmoid's last-ulp rounding (bounded in (a)),
    # which moves diagram points by ~1e-7 each; the loss is Lipschitz in them -> rtol 1e-4
    e2e = losses.topo_forward_backward(mc, gc, None, interp=50, mode=mode)
    ref = topo_loss_ref(torch.sigmoid(masks), gt.float(), 0.1, interp=50, feat_d=1, mode=mode)
    assert abs(e2e - float(ref)) <= 1e-4 * abs(float(ref))


def test_dicece_dropin_autograd(cuda):
    """losses.DiceCELoss()(input, target) through autograd (HIP Dice partials + CE/Dice backward) vs the
    oracle's monai restatement; soft targets are rejected rather than rounded."""
    from dilabhelmholtzoct_amd.losses import DiceCELoss
    from oracle.losses_ref import dicece_ref
    g = torch.Generator().manual_seed(3)
    for B, N in ((2, 5), (1, 1), (3, 2)):
        x = (torch.randn(B, N, 96, 80, generator=g) * 3).to(cuda).requires_grad_()
        t = (torch.rand(B, N, 96, 80, generator=g) > 0.6).double()
        loss = DiceCELoss(sigmoid=True)(x, t.to(cuda))
        assert loss.dtype == torch.float64
        loss.backward()
        xr = x.detach().double().cpu().requires_grad_()
        ref = dicece_ref(xr, t)
        ref.backward()
        assert abs(float(loss) - float(ref)) <= 1e-6 * abs(float(ref)) + 1e-9
        _assert_grad_close(x.grad.double().cpu(), xr.grad, rtol=2e-5)
    with pytest.raises(ValueError):
        DiceCELoss(sigmoid=True)(x.detach(), torch.full(x.shape, 0.5, device=cuda))
