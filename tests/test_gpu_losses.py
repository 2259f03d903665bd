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
