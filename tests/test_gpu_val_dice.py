"""Val-Dice parity (BASELINE.json north_star: "val Dice within ±0.005 of the CPU reference on identical
seeds"). Both sides start from the same synthetic weights, train K steps on the same batch with the
topological loss on (BASELINE configs[2]: boxes, --top=True) and then score the same held-out images with
the reference's per-class pooled Dice (training_utils.py:113-156, with its early `break`):

* ours: HIP path (FusedTrainStep: bf16 MFMA encoder/decoder, fused losses, HIP Adam) + predict_masks;
* oracle: oracle/step_ref.py (transformers SamModel fp32 — run on the GPU here only to keep the test
  short — restated DiceCE / topo loss and torch Adam on the CPU).

Tolerance: |Dice_ours - Dice_ref| <= 0.005 (the north_star bar), after 0 and after K = 3 steps."""
import pytest
import torch

pytestmark = pytest.mark.gpu

NAME = "facebook/sam-vit-base"
TOL = 0.005


def _batches():
    from dilabhelmholtzoct_amd import data
    proc = data.make_processor()

    def mk(seed, n):
        ds = data.synthetic_oct(seed=seed, n=n)
        sd = data.SAMDataset(ds, {"prompt_type": "bboxes"}, epoch_seed=0)
        return data.process_batch(proc, data.custom_collate([sd[i] for i in range(len(sd))]), "bboxes")
    return mk(1000, 2), mk(999, 3)


def _dice(masks, vb):
    from dilabhelmholtzoct_amd.train import class_confusion, mean_dice
    return mean_dice(class_confusion(masks, vb["gt_u8"], vb["mask_values"]))


def test_val_dice_parity(cuda):
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep, predict_masks
    from oracle.step_ref import CpuReferenceStep, synthetic_state_dict

    state = synthetic_state_dict(NAME, seed=0)
    train_cpu, val_cpu = _batches()
    train, val = data.to_device_batch(train_cpu, cuda), data.to_device_batch(val_cpu, cuda)

    ours = SamModel(NAME)
    ours.load_state_dict(state)
    ours = ours.to(cuda)
    step = FusedTrainStep(ours, lr=1e-3, topological=True, graphs=False)
    ref = CpuReferenceStep(NAME, topological=True, lr=1e-3, state_dict=state, device=cuda)

    def both_dice():
        got = _dice(predict_masks(ours, val), val)
        with torch.no_grad():
            rmasks = ref.predict(val_cpu)
        want = _dice(rmasks, val_cpu)
        return got, want

    results = []
    got, want = both_dice()
    results.append((0, got, want))
    for _ in range(3):
        step.step(train)
        ref.step(train_cpu)
    step.flush()
    torch.cuda.synchronize()
    got, want = both_dice()
    results.append((3, got, want))
    for k, got, want in results:
        print(f"after {k} steps: val Dice HIP {got:.5f}  oracle {want:.5f}  diff {got - want:+.5f}")
    for k, got, want in results:
        assert abs(got - want) <= TOL, (k, got, want)
    # the steps must have moved the model (else the second check repeats the first)
    assert results[1][2] != results[0][2]
