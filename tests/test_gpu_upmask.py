"""Fused upscaling tail + mask head (csrc/upmask.hip; SamMaskDecoder, hf:modeling_sam.py:519-542: second
ConvTranspose2d, GELU, masks = hyper_in @ upscaled_embedding) vs a plain PyTorch fp32 reference on the
same bf16 inputs, forward and backward (autograd), ntok 1 and 3.

Tolerances: the forward keeps fp32 everywhere after the bf16 MFMA inputs (1e-4 of the max |mask|);
the backward feeds d pre-activation to the d up1 / d W2 products as bf16 (rel. 2^-9 per element), so
d up1, d W2, d b2 and d hyper are checked at 1e-2 of each tensor's max magnitude."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


def _inputs(cuda, P, ns, seed):
    g = torch.Generator().manual_seed(seed)
    up1 = torch.randn(P * 16384, 64, generator=g).to(cuda, torch.bfloat16)
    w2 = (0.15 * torch.randn(64, 128, generator=g)).to(cuda, torch.bfloat16)
    b2 = (0.2 * torch.randn(32, generator=g)).to(cuda)
    hyper = torch.randn(P, ns, 32, generator=g).to(cuda)
    dmask = torch.randn(P, ns, 256, 256, generator=g).to(cuda)
    return up1, w2, b2, hyper, dmask


def _ref(up1, w2, b2, hyper, P):
    """fp32: rows (p, y1, x1, dy1, dx1) x columns (dy2, dx2, c) -> image [P, 32, 256, 256] -> masks."""
    pre = up1 @ w2 + b2.repeat(4)
    up2 = F.gelu(pre).view(P, 64, 64, 2, 2, 2, 2, 32)  # p y1 x1 dy1 dx1 dy2 dx2 c
    img = up2.permute(0, 7, 1, 3, 5, 2, 4, 6).reshape(P, 32, 256, 256)
    return torch.einsum("ptc,pcyx->ptyx", hyper, img)


@pytest.mark.parametrize("P,ns", [(3, 1), (2, 3), (5, 1)])
def test_upmask_fwd_bwd(cuda, P, ns):
    from dilabhelmholtzoct_amd import kernels
    up1, w2, b2, hyper, dmask = _inputs(cuda, P, ns, 10 * P + ns)
    masks = torch.empty(P, ns, 256, 256, device=cuda)
    kernels.upmask_fwd(up1, w2, b2, hyper, P, ns, masks)
    u = up1.float().requires_grad_()
    w = w2.float().requires_grad_()
    b = b2.clone().requires_grad_()
    h = hyper.clone().requires_grad_()
    ref = _ref(u, w, b, h, P)
    assert _rel(masks, ref) < 1e-4, _rel(masks, ref)
    (ref * dmask).sum().backward()
    dup1 = torch.empty_like(up1)
    dw2 = torch.full((64, 128), float("nan"), device=cuda)
    db2 = torch.full((32,), float("nan"), device=cuda)
    dh = torch.full((P, ns, 32), float("nan"), device=cuda)
    kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, dup1, dw2, db2, dh)
    assert _rel(dup1, u.grad) < 1e-2, _rel(dup1, u.grad)
    assert _rel(dw2, w.grad) < 1e-2, _rel(dw2, w.grad)
    assert _rel(db2, b.grad) < 1e-2, _rel(db2, b.grad)
    assert _rel(dh, h.grad) < 1e-2, _rel(dh, h.grad)


def test_upmask_deterministic(cuda):
    from dilabhelmholtzoct_amd import kernels
    P, ns = 4, 1
    up1, w2, b2, hyper, dmask = _inputs(cuda, P, ns, 99)
    res = []
    for _ in range(2):
        masks = torch.empty(P, ns, 256, 256, device=cuda)
        kernels.upmask_fwd(up1, w2, b2, hyper, P, ns, masks)
        dup1 = torch.empty_like(up1)
        dw2, db2, dh = (torch.empty(64, 128, device=cuda), torch.empty(32, device=cuda),
                        torch.empty(P, ns, 32, device=cuda))
        kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, dup1, dw2, db2, dh)
        res.append((masks, dup1, dw2, db2, dh))
    for a, b in zip(*res):
        assert torch.equal(a, b)
