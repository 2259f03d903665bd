"""One training step of BASELINE configs[0]'s workload and configs[1] - configs[4]'s per-GPU slices on the HIP path against the oracle
(oracle/step_ref.py: transformers SamModel fp32 + restated DiceCE / topo loss, run on the GPU here only for
speed) on the same synthetic weights and batch:

* configs[0]: sam-vit-base, box prompts, --top=False, one image (the reference's CPU plumbing case) through the
  HIP path;
* configs[1]: sam-vit-base, box prompts, --top=False, bf16, 8 images per GPU (the DiceCE-only step,
  ref:octsam/models/training_utils.py:62-68 with topological=False);
* configs[2]: the same with --top=True (the bench's workload);
* configs[3]: sam-vit-large, point prompts, --top=True, bf16, 4 images per GPU (batch 32 over 8 GPUs);
* configs[4]: sam-vit-huge, a box and a point per component, --top=True, 8 images per GPU (batch 64 over 8
  GPUs), with the bf16 encoder and with the fp16 encoder (the configuration's precision).

Checked: the DiceCE (1e-3 relative) and topological (2e-2 relative) loss values and the mask-decoder gradient
(global cosine > 0.99, median per-tensor relative Frobenius error < 0.1 — 0.075 measured for vit-l, the bf16
decoder's own rounding — and every tensor < 0.15). The topo loss of configs[4]'s B > 1 batch covers prompt 0 of each image
(topo_mode "first")."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = {  # name: (model, prompt, images, encoder dtype, topological)
    # configs[0]'s workload (the reference's own CPU-runnable case: vit-b, boxes, --top=False, one image) on the GPU
    "vitb_bboxes_b1_top_off": ("facebook/sam-vit-base", "bboxes", 1, torch.bfloat16, False),
    "vitb_bboxes_b8_top_off": ("facebook/sam-vit-base", "bboxes", 8, torch.bfloat16, False),
    "vitb_bboxes_b8_top_on": ("facebook/sam-vit-base", "bboxes", 8, torch.bfloat16, True),
    "vitl_points_b4_bf16": ("facebook/sam-vit-large", "points", 4, torch.bfloat16, True),
    "vith_both_b8_bf16": ("facebook/sam-vit-huge", "both", 8, torch.bfloat16, True),
    "vith_both_b8_fp16": ("facebook/sam-vit-huge", "both", 8, torch.float16, True),
}


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.mark.parametrize("case", list(CASES))
def test_step_vs_oracle(cuda, case):
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    from oracle.step_ref import CpuReferenceStep, synthetic_state_dict
    name, prompt, B, edt, top = CASES[case]
    state = synthetic_state_dict(name, seed=0)
    sd = data.SAMDataset(data.synthetic_oct(seed=31, n=B), {"prompt_type": prompt}, epoch_seed=0)
    b = data.process_batch(data.make_processor(), data.custom_collate([sd[i] for i in range(B)]), prompt)
    bd = data.to_device_batch(b, cuda)

    ours = SamModel(name)
    ours.load_state_dict(state)
    ours = ours.to(cuda)
    if edt == torch.float16:
        ours.set_encoder_dtype(torch.float16)
    step = FusedTrainStep(ours, topological=top)
    crop = tuple(int(v) for v in b["reshaped_input_sizes"][0])
    orig = tuple(int(v) for v in b["original_sizes"][0])
    loss = step.forward_backward(bd["pixel_values"], bd["gt_u8"], input_boxes=bd.get("input_boxes"),
                                 input_points=bd.get("input_points"), crop=crop, orig=orig).cpu()
    ours.mask_decoder.bind_param_grads()
    got_g = {n: p.grad.detach().double().cpu() for n, p in ours.mask_decoder.named_parameters()
             if p.grad is not None}
    del ours, step
    torch.cuda.empty_cache()

    ref = CpuReferenceStep(name, topological=top, state_dict=state, device=cuda, loss_device=cuda)
    ref.opt.zero_grad()
    rl, rtopo, _ = ref.forward_loss(b)
    rl.backward()
    rl, rtopo = float(rl.detach()), float(torch.as_tensor(rtopo).detach())
    dicece, rdicece = float(loss[3] - loss[2]), rl - rtopo
    print(f"{case}: DiceCE {dicece:.6f} (oracle {rdicece:.6f}), topo {float(loss[2]):.6f} (oracle {rtopo:.6f})")
    assert abs(dicece - rdicece) <= 1e-3 * abs(rdicece), (dicece, rdicece)
    assert abs(float(loss[2]) - rtopo) <= 2e-2 * abs(rtopo) + 1e-6, (float(loss[2]), rtopo)
    if not top:
        assert float(loss[2]) == 0.0 and rtopo == 0.0, (float(loss[2]), rtopo)

    rg = {n: p.grad.double().cpu() for n, p in ref.model.mask_decoder.named_parameters() if p.grad is not None}
    scale = max(g.norm().item() for g in rg.values())
    flat_got, flat_want, bad, errs = [], [], {}, []
    for n, r in rg.items():
        if r.norm().item() < 1e-6 * scale:  # no gradient in the reference (softmax-invariant key biases)
            continue
        g = got_g[n]
        flat_got.append(g.flatten())
        flat_want.append(r.flatten())
        e = _rel(g, r)
        errs.append(e)
        if e > 0.15:  # the ill-conditioned self-attention / token-side query biases reach ~0.1 (tests/test_gpu_model.py)
            bad[n] = e
    got, want = torch.cat(flat_got), torch.cat(flat_want)
    cos = float((got @ want) / (got.norm() * want.norm()))
    print(f"{case}: decoder gradient cosine {cos:.5f}, worst tensors {sorted(bad.items(), key=lambda kv: -kv[1])[:4]}")
    med = sorted(errs)[len(errs) // 2]
    print(f"{case}: median per-tensor relative error {med:.4f}")
    assert cos > 0.99, cos
    assert med < 0.1, med
    assert not bad, bad
