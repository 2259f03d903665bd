"""BASELINE configs[3] model (sam-vit-large: D = 1024, 24 layers, 16 heads, global layers 5/11/17/23) on
the HIP path vs transformers' SamModel in fp32 on the same weights: encoder output and point-prompt
decoder masks (the tolerances of tests/test_gpu_model.py: relative Frobenius error of the bf16 MFMA path),
plus one fused training step (topological loss on, point prompts) that must produce finite losses."""
import pytest
import torch

pytestmark = pytest.mark.gpu

NAME = "facebook/sam-vit-large"


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def test_vit_large_parity_and_step(cuda):
    from transformers import SamModel as HFSam
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    from oracle.step_ref import hf_config
    ours = SamModel(NAME)
    ours.init_weights(seed=2)
    hf = HFSam(hf_config(NAME))
    hf.load_state_dict(ours.state_dict())
    ours = ours.to(cuda)
    hf = hf.to(cuda).float().eval()
    g = torch.Generator().manual_seed(0)
    px = torch.randn(2, 3, 1024, 1024, generator=g).to(cuda)
    pts = torch.randint(0, 1024, (2, 3, 1, 2), generator=g).to(cuda).double()
    with torch.no_grad():
        ref = hf.vision_encoder(px).last_hidden_state
        got = ours.vision_encoder(px)
        assert _rel(got, ref) < 3e-2
        out_ref = hf(image_embeddings=ref, input_points=pts, multimask_output=False)
        out = ours(image_embeddings=ref, input_points=pts, multimask_output=False)
    assert _rel(out.pred_masks, out_ref.pred_masks) < 3e-2
    del hf
    torch.cuda.empty_cache()
    ds = data.synthetic_oct(seed=3, n=2)
    sd = data.SAMDataset(ds, {"prompt_type": "points"}, epoch_seed=0)
    b = data.to_device_batch(data.process_batch(data.make_processor(),
                                                data.custom_collate([sd[i] for i in range(2)]), "points"), cuda)
    step = FusedTrainStep(ours, lr=1e-3, topological=True, graphs=False)
    loss = step.step(b)
    step.flush()
    lh = loss.cpu()
    print("vit-l step loss (dice, ce, topo, total):", lh.tolist())
    assert torch.isfinite(lh).all()
