"""octsam_adam (fused Adam + bf16 weight mirror, ref:octsam/models/training_utils.py:31,68) against
torch.optim.Adam on the same fp32 parameters and gradients, with weight_decay != 0 and several steps
(bias corrections change per step). fp32 arithmetic on both sides; the orders of operations match
torch's single-tensor formula up to fused multiply-adds -> 1e-6 of the parameter scale."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wd", [0.0, 1e-4, 0.05])
def test_adam_matches_torch(cuda, wd):
    from dilabhelmholtzoct_amd import kernels as K
    g = torch.Generator().manual_seed(int(wd * 1e4) + 1)
    n = 1_000_003  # odd tail
    p0 = torch.randn(n, generator=g).to(cuda)
    ours = p0.clone()
    ref = p0.clone().requires_grad_()
    m = torch.zeros_like(ours)
    v = torch.zeros_like(ours)
    mirror = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    lr, b1, b2, eps = 1e-3, 0.9, 0.999, 1e-8
    opt = torch.optim.Adam([ref], lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd, foreach=False)
    for t in range(1, 6):
        grad = (torch.randn(n, generator=g) * (0.1 * t)).to(cuda)
        ref.grad = grad.clone()
        opt.step()
        K.adam(ours, grad, m, v, beta1=b1, beta2=b2, eps=eps, weight_decay=wd, step_size=lr / (1 - b1 ** t),
               bc2_sqrt=math.sqrt(1 - b2 ** t), params_bf16=mirror)
        err = (ours - ref.detach()).abs().max().item()
        assert err <= 1e-6 * max(1.0, p0.abs().max().item()), (t, err)
        st = opt.state[ref]
        assert (m - st["exp_avg"]).abs().max().item() <= 1e-6 * st["exp_avg"].abs().max().item()
        assert (v - st["exp_avg_sq"]).abs().max().item() <= 1e-6 * st["exp_avg_sq"].abs().max().item()
    assert torch.equal(mirror, ours.to(torch.bfloat16))
