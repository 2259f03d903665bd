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


@pytest.mark.parametrize("P,ns", [(3, 1), (2, 3)])
def test_upmask_ln_bwd(cuda, P, ns):
    """octsam_upmask_ln_bwd: the LayerNorm2d(eps 1e-6) + GELU in front of up1 differentiated in the mask-head
    backward, vs fp32 autograd through LN + GELU + ConvT2 + mask head on the same bf16 x (the kernel's up1 is the
    bf16 LN forward output, as in the step). d x at 1e-2 of its max (the d pre-activation feeds the MFMAs as bf16),
    d LN weight / bias at 1e-2; and the fused path against octsam_upmask_bwd + octsam_layernorm_bwd (which rounds
    d up1 to bf16 in between) at 2e-2."""
    from dilabhelmholtzoct_amd import kernels
    _, w2, b2, hyper, dmask = _inputs(cuda, P, ns, 7 * P + ns)
    g = torch.Generator().manual_seed(5 + P)
    x = (torch.randn(P * 16384, 64, generator=g) * 0.8 + 0.3).to(cuda, torch.bfloat16)
    lw = (1.0 + 0.3 * torch.randn(64, generator=g)).to(cuda)
    lb = (0.2 * torch.randn(64, generator=g)).to(cuda)
    up1 = torch.empty_like(x)
    mean = torch.empty(P * 16384, device=cuda)
    rstd = torch.empty(P * 16384, device=cuda)
    kernels.layernorm_fwd(x, lw, lb, 1e-6, up1, act=2, mean=mean, rstd=rstd)
    xr = x.float().requires_grad_()
    wr, br = lw.clone().requires_grad_(), lb.clone().requires_grad_()
    u = F.gelu(F.layer_norm(xr, (64,), wr, br, eps=1e-6))
    ref = _ref(u, w2.float(), b2, hyper, P)
    (ref * dmask).sum().backward()
    dx = torch.empty_like(x)
    dw2, db2, dh = torch.empty(64, 128, device=cuda), torch.empty(32, device=cuda), torch.empty(P, ns, 32, device=cuda)
    dlw, dlb = torch.full((64,), float("nan"), device=cuda), torch.full((64,), float("nan"), device=cuda)
    kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, dx, dw2, db2, dh, ln=(x, mean, rstd, lw, lb, dlw, dlb))
    assert _rel(dx, xr.grad) < 1e-2, _rel(dx, xr.grad)
    assert _rel(dlw, wr.grad) < 1e-2, _rel(dlw, wr.grad)
    assert _rel(dlb, br.grad) < 1e-2, _rel(dlb, br.grad)
    # the two-kernel path
    dup1 = torch.empty_like(x)
    dw2b, db2b, dhb = torch.empty_like(dw2), torch.empty_like(db2), torch.empty_like(dh)
    kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, dup1, dw2b, db2b, dhb)
    dx2 = torch.empty_like(x)
    _, dlw2, dlb2 = kernels.layernorm_bwd(dup1, x, mean, rstd, lw, lb, dx2, act=2)
    assert torch.equal(dw2, dw2b) and torch.equal(db2, db2b) and torch.equal(dh, dhb)
    assert _rel(dx, dx2) < 2e-2 and _rel(dlw, dlw2) < 2e-2 and _rel(dlb, dlb2) < 2e-2
    # deterministic
    dx3, dlw3, dlb3 = torch.empty_like(x), torch.empty_like(dlw), torch.empty_like(dlb)
    kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, dx3, dw2b, db2b, dhb, ln=(x, mean, rstd, lw, lb, dlw3, dlb3))
    assert torch.equal(dx, dx3) and torch.equal(dlw, dlw3) and torch.equal(dlb, dlb3)
    # d x at a row stride (octsam_upmask_ln_bwd_strided: the left half of a [P * 4096, 512] operand), the right half
    # untouched
    wide = torch.full((P * 4096, 512), 7.0, device=cuda, dtype=torch.bfloat16)
    dlw4, dlb4 = torch.empty_like(dlw), torch.empty_like(dlb)
    kernels.upmask_bwd(up1, w2, b2, hyper, dmask, P, ns, wide, dw2b, db2b, dhb, ln=(x, mean, rstd, lw, lb, dlw4, dlb4),
                       ldd=512)
    assert torch.equal(wide[:, :256].reshape(P * 16384, 64), dx) and bool((wide[:, 256:] == 7.0).all())
    assert torch.equal(dlw4, dlw) and torch.equal(dlb4, dlb)
