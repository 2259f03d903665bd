"""DiceCE backward fused with the post-processing adjoint's row pass (octsam_dicece_pp_rows + octsam_pp_bwd_rows_maps +
octsam_pp_bwd_cols, ABI 19) against the two-kernel path it replaces (octsam_dicece_bwd's d-mask, then
octsam_postproc_bwd): the same per-pixel arithmetic and the same CSR row / column sums, so the d low-res masks and the
loss agree to rounding (the CE partials are summed per (image, row) instead of per grid-stride block). With kept maps
(the topological loss's), their d-mask goes through the compact topo backward and the per-map row pass."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(cuda, B, N, seed, crop=(1024, 993), orig=(496, 512)):
    from dilabhelmholtzoct_amd.losses import postproc_forward
    g = torch.Generator().manual_seed(seed)
    low = (3.0 * torch.randn(B * N, 256, 256, generator=g)).to(cuda)
    gt = (torch.rand(B * N, *orig, generator=g) > 0.7).to(torch.uint8).to(cuda)
    masks, part = postproc_forward(low, crop, orig, gt)
    return masks.view(B, N, *orig), gt.view(B, N, *orig), part, crop, orig


@pytest.mark.parametrize("B,N,maps", [(2, 5, ()), (2, 5, (0, 5)), (1, 21, (0,)), (3, 1, (0, 1, 2)),
                                     (1, 28, (0,)), (2, 32, (0, 32))])
def test_fused_pp_matches_two_kernel_path(cuda, B, N, maps):
    from dilabhelmholtzoct_amd.losses import (dicece_forward_backward, dicece_pp_rows, postproc_backward,
                                              pp_rows_finish, topo_device_backward)
    masks, gt, part, crop, orig = _case(cuda, B, N, 7 * B + N)
    H, W = orig
    loss_a, dmask = dicece_forward_backward(masks, gt, part)
    midx = torch.tensor(list(maps), dtype=torch.int32, device=cuda) if maps else None
    dp = None
    if maps:
        g = torch.Generator().manual_seed(11)
        dp = torch.randn(len(maps), 50 * 50, generator=g).to(cuda)
        topo_device_backward(masks, midx, dp, dmask, interp=50)
    dlow_a = postproc_backward(dmask.view(B * N, H, W), 256, crop, orig)

    loss_b, tmp, dkeep = dicece_pp_rows(masks, gt, part, crop, maps=maps)
    if maps:
        topo_device_backward(masks, midx, dp, dkeep, interp=50, compact=True)
    dlow_b = pp_rows_finish(tmp, crop, orig, dkeep=dkeep, midx=midx)
    torch.cuda.synchronize()
    assert torch.allclose(loss_a, loss_b, rtol=1e-12, atol=0.0), (loss_a, loss_b)
    scale = dlow_a.abs().max().item()
    err = (dlow_a - dlow_b).abs().max().item()
    assert err <= 1e-6 * scale, (err, scale)
    if maps:  # the kept maps' d-mask equals the two-kernel d-mask rows of those maps
        assert torch.allclose(dkeep, dmask.view(B * N, H, W)[list(maps)], rtol=1e-6, atol=1e-12)


def test_train_step_fused_pp_matches_unfused(cuda):
    """Two graph-replayed training steps with the fused and the two-kernel loss backward: the same losses and updated
    decoder weights to rounding."""
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    sd = data.SAMDataset(data.synthetic_oct(seed=3, n=2), {"prompt_type": "bboxes"}, epoch_seed=0)
    batch = data.to_device_batch(data.process_batch(data.make_processor(), data.custom_collate([sd[0], sd[1]]),
                                                    "bboxes"), cuda)
    runs = []
    for fused in (True, False):
        model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(cuda)
        step = FusedTrainStep(model, topological=True, graphs=True)
        step.fused_pp = fused
        losses = [step.step(batch).clone() for _ in range(2)]
        step.flush()
        torch.cuda.synchronize()
        runs.append((losses, model.mask_decoder.flat.detach().clone()))
    (la, fa), (lb, fb) = runs
    for a, b in zip(la, lb):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-9), (a, b)
    assert (fa - fb).abs().max().item() <= 1e-5 * fa.abs().max().item()


def _wide_batch(cuda, reps):
    """A real two-image batch whose prompt dimension is repeated `reps` times (N = 21 * reps > 32 for reps >= 2):
    more components than the fused DiceCE / row-pass kernel takes (the reference caps neither)."""
    from dilabhelmholtzoct_amd import data
    sd = data.SAMDataset(data.synthetic_oct(seed=3, n=2), {"prompt_type": "bboxes"}, epoch_seed=0)
    b = data.process_batch(data.make_processor(), data.custom_collate([sd[0], sd[1]]), "bboxes")
    for k in ("input_boxes", "gt_u8", "mask_values"):
        b[k] = torch.cat([b[k]] * reps, 1)
    return data.to_device_batch(b, cuda)


def test_train_step_over_32_prompts_falls_back(cuda):
    """N > 32 prompts: FusedTrainStep (fused_pp on by default) takes the two-kernel DiceCE + post-processing backward
    instead of raising in octsam_dicece_pp_rows, so its steps equal those with fused_pp off bit for bit."""
    from dilabhelmholtzoct_amd.losses import dicece_pp_rows_supported
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    batch = _wide_batch(cuda, 2)
    B, N = batch["gt_u8"].shape[:2]
    assert N > 32 and not dicece_pp_rows_supported(B, N, *batch["gt_u8"].shape[2:])
    runs = []
    for fused in (True, False):
        model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(cuda)
        step = FusedTrainStep(model, topological=True, graphs=True)
        step.fused_pp = fused
        losses = [step.step(batch).clone() for _ in range(2)]
        step.flush()
        torch.cuda.synchronize()
        runs.append((losses, model.mask_decoder.flat.detach().clone()))
    (la, fa), (lb, fb) = runs
    for a, b in zip(la, lb):
        assert torch.isfinite(a).all() and torch.equal(a, b), (a, b)
    assert torch.equal(fa, fb)
