"""BASELINE configs[4] model (sam-vit-huge: D = 1280, 32 layers, 16 heads of head_dim 80, global layers
7/15/23/31) with its prompt mode (a box and a point per component, --prompt=both) on the HIP path vs
transformers' SamModel in fp32 on the same weights: encoder output and mixed-prompt decoder masks (the
tolerances of tests/test_gpu_model.py: relative Frobenius error of the 16-bit MFMA path), then one fused
training step (topological loss on) that must give finite losses and a decoder update."""
import pytest
import torch

pytestmark = pytest.mark.gpu

NAME = "facebook/sam-vit-huge"


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def test_vit_huge_parity_and_step(cuda):
    from transformers import SamModel as HFSam
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    from oracle.step_ref import hf_config
    ours = SamModel(NAME)
    ours.init_weights(seed=4)
    assert ours.config.vision.hidden_size // ours.config.vision.num_attention_heads == 80
    hf = HFSam(hf_config(NAME))
    hf.load_state_dict(ours.state_dict())
    ours = ours.to(cuda)
    hf = hf.to(cuda).float().eval()
    g = torch.Generator().manual_seed(1)
    px = torch.randn(2, 3, 1024, 1024, generator=g).to(cuda)
    pts = torch.randint(0, 1024, (2, 3, 1, 2), generator=g).to(cuda).double()
    lo = torch.randint(0, 600, (2, 3, 2), generator=g)
    boxes = torch.cat([lo, lo + torch.randint(50, 400, (2, 3, 2), generator=g)], -1).to(cuda).double()
    with torch.no_grad():
        ref = hf.vision_encoder(px).last_hidden_state
        got = ours.vision_encoder(px)
        enc_err = _rel(got, ref)
        out_ref = hf(image_embeddings=ref, input_points=pts, input_boxes=boxes, multimask_output=False)
        out = ours(image_embeddings=ref, input_points=pts, input_boxes=boxes, multimask_output=False)
    mask_err = _rel(out.pred_masks, out_ref.pred_masks)
    print(f"vit-h encoder rel err {enc_err:.4f}, both-prompt masks rel err {mask_err:.4f}")
    assert enc_err < 3e-2 and mask_err < 3e-2
    del hf
    torch.cuda.empty_cache()
    ds = data.synthetic_oct(seed=5, n=2)
    sd = data.SAMDataset(ds, {"prompt_type": "both"}, epoch_seed=0)
    b = data.to_device_batch(data.process_batch(data.make_processor(),
                                                data.custom_collate([sd[i] for i in range(2)]), "both"), cuda)
    before = ours.mask_decoder.flat.detach().clone()
    step = FusedTrainStep(ours, lr=1e-3, topological=True, graphs=False)
    loss = step.step(b)
    step.flush()
    lh = loss.cpu()
    print("vit-h step loss (dice, ce, topo, total):", lh.tolist())
    assert torch.isfinite(lh).all()
    assert not torch.equal(before, ours.mask_decoder.flat)


def test_vit_huge_fp16_encoder(cuda):
    """BASELINE configs[4] precision: the frozen encoder's GEMMs and attention on fp16 operands (octsam_gemm_f16,
    fp16 attention), fp32 accumulation and residual stream; vs transformers fp32 (fp16's 11-bit significand:
    tighter than the bf16 bound) and one fused training step."""
    from transformers import SamModel as HFSam
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    from oracle.step_ref import hf_config
    ours = SamModel(NAME)
    ours.init_weights(seed=6)
    hf = HFSam(hf_config(NAME))
    hf.load_state_dict(ours.state_dict())
    ours = ours.to(cuda).set_encoder_dtype(torch.float16)
    hf = hf.to(cuda).float().eval()
    px = torch.randn(2, 3, 1024, 1024, generator=torch.Generator().manual_seed(2)).to(cuda)
    with torch.no_grad():
        ref = hf.vision_encoder(px).last_hidden_state
        got = ours.vision_encoder(px)
    err16 = _rel(got, ref)
    ours.set_encoder_dtype(torch.bfloat16)
    with torch.no_grad():
        err_b = _rel(ours.vision_encoder(px), ref)
    ours.set_encoder_dtype(torch.float16)
    print(f"vit-h encoder rel err fp16 {err16:.5f} (bf16 {err_b:.5f})")
    assert err16 < 5e-3 and err16 < err_b
    del hf
    torch.cuda.empty_cache()
    ds = data.synthetic_oct(seed=7, n=2)
    sd = data.SAMDataset(ds, {"prompt_type": "both"}, epoch_seed=0)
    b = data.to_device_batch(data.process_batch(data.make_processor(),
                                                data.custom_collate([sd[i] for i in range(2)]), "both"), cuda)
    step = FusedTrainStep(ours, lr=1e-3, topological=True, graphs=True)
    for _ in range(2):
        loss = step.step(b)
    step.flush()
    assert torch.isfinite(loss.cpu()).all()
