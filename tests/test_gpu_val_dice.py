"""Val-Dice parity (BASELINE.json north_star: "val Dice within ±0.005 of the CPU reference on identical seeds") on
SURVEY.md §8(d)'s protocol: 128 synthetic training scans and 32 held-out ones, B = 8, box prompts, --top=True,
lr 1e-3 (the reference CLI's default), the reference's prompt redraw every epoch (SAMDataset.__getitem__).

Start point. From the random initial weights every run first collapses to all-foreground masks (specificity ~0),
and the step at which it leaves that state is chaotic — the same arithmetic in fp32 leaves it after ~112 steps on
one data seed and not within 384 on another; the HIP path after ~112 / ~128 steps, torch's own bf16 autocast run
after ~176 (profiles/r03/valdice_traj_*.jsonl). A Dice compared during or across that transition measures the
chaos, not the implementation. Both sides therefore start from the decoder the fp32 oracle reached after 256 steps
on another synthetic set (training seed 2000, held-out seed 3000: tests/golden/valdice_start_decoder.safetensors,
made on MI355X by scripts/val_dice_traj.py --seed 0 --no-hip --save-at 256; encoder and prompt encoder: the
synthetic weights, seed 0), which is past the transition.

Then both sides train the same EPOCHS epochs on this test's own 128 scans (seed 2001) and are scored on its 32
held-out scans (seed 3001):
* ours: FusedTrainStep exactly as bench.py runs it (hipGraphs + the encoder lookahead), predict_masks +
  class_confusion (HIP confusion counts);
* oracle: oracle/step_ref.py (transformers SamModel fp32 — on the GPU only to keep the test short; the frozen
  encoder's embeddings computed once per batch — restated DiceCE / topo loss, torch Adam), scored by
  oracle/eval_ref.pooled_confusion_ref (the reference's threshold and break quirk, training_utils.py:126-156).
Asserted: the oracle is in the non-degenerate regime (mean specificity > 0.5 and Dice >= 0.1 above the
random-init weights'), and |Dice_ours - Dice_oracle| <= 0.005 at the final checkpoint (no relaxed bound)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

NAME = "facebook/sam-vit-base"
TOL = 0.005
LR = 1e-3
EPOCHS = 2
BS = 8
START = os.path.join(os.path.dirname(__file__), "golden", "valdice_start_decoder.safetensors")


def _epoch_batches(seed, n, epoch):
    from dilabhelmholtzoct_amd import data
    proc = data.make_processor()
    sd = data.SAMDataset(data.synthetic_oct(seed=seed, n=n), {"prompt_type": "bboxes"}, epoch_seed=seed)
    sd.epoch = epoch
    return [data.process_batch(proc, data.custom_collate([sd[i] for i in range(s, min(n, s + BS))]), "bboxes")
            for s in range(0, n, BS)]


def test_val_dice_parity(cuda):
    from safetensors.torch import load_file
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep, class_confusion, predict_masks
    from oracle.eval_ref import mean_dice_ref, mean_specificity_ref, pooled_confusion_ref
    from oracle.step_ref import CpuReferenceStep, synthetic_state_dict

    state = synthetic_state_dict(NAME, seed=0)
    val_cpu = _epoch_batches(3001, 32, 0)
    val = [data.to_device_batch(v, cuda) for v in val_cpu]
    ref = CpuReferenceStep(NAME, topological=True, lr=LR, state_dict=state, device=cuda, loss_device=cuda)
    val_emb = [ref.embed(v) for v in val_cpu]

    def ref_conf():
        c = torch.zeros(14, 4, dtype=torch.int64)
        with torch.no_grad():
            for v, e in zip(val_cpu, val_emb):
                c += pooled_confusion_ref(ref.predict(v, e), v["gt_u8"], v["mask_values"])
        return c

    dice_init = mean_dice_ref(ref_conf())  # the random-init decoder
    start = {k: v.float() for k, v in load_file(START).items()}
    for k, v in start.items():
        assert k in state and state[k].shape == v.shape, k
        state[k] = v
    ref.model.load_state_dict(state)
    ref.opt = torch.optim.Adam(ref.model.mask_decoder.parameters(), lr=LR)
    ours = SamModel(NAME)
    ours.load_state_dict(state)
    ours = ours.to(cuda)
    step = FusedTrainStep(ours, lr=LR, topological=True, graphs=True, pipeline=True)

    def ours_conf():
        step.flush()
        c = torch.zeros(14, 3, dtype=torch.int64)
        for v in val:
            c += class_confusion(predict_masks(ours, v), v["gt_u8"], v["mask_values"])
        return c

    def dice3(c):  # (tp, fp, fn) -> mean Dice (training_utils.py:156, :246)
        return mean_dice_ref(torch.cat([c, torch.zeros(c.shape[0], 1, dtype=c.dtype)], 1))

    results = [(0, dice3(ours_conf()), mean_dice_ref(ref_conf()))]
    emb_cache = {}
    k = 0
    for ep in range(EPOCHS):
        tr_cpu = _epoch_batches(2001, 128, ep)
        tr = [data.to_device_batch(b, cuda) for b in tr_cpu]
        for i, b in enumerate(tr):
            step.step(b, next_batch=tr[i + 1] if i + 1 < len(tr) else None)
            if i not in emb_cache:
                emb_cache[i] = ref.embed(tr_cpu[i])
            ref.step(tr_cpu[i], emb_cache[i])
            k += 1
        c_ref = ref_conf()
        results.append((k, dice3(ours_conf()), mean_dice_ref(c_ref)))
    spec = mean_specificity_ref(c_ref)
    for kk, got, want in results:
        print(f"after {kk:3d} steps: val Dice HIP {got:.5f}  oracle {want:.5f}  diff {got - want:+.5f}")
    print(f"random-init Dice {dice_init:.5f}; oracle specificity at the end {spec:.4f}")
    kk, got, want = results[-1]
    assert spec > 0.5, f"oracle specificity {spec:.4f}: the degenerate all-foreground regime"
    assert want - dice_init >= 0.1, (want, dice_init)
    assert abs(got - want) <= TOL, (kk, got, want)
