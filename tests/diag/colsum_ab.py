"""A/B of the fused bias gradients (column sums inside the k-major weight-gradient GEMM) against the separate
colsum passes they replaced: per-parameter gradient differences after one step, and the val-Dice trajectory
of tests/test_gpu_val_dice.py under both. Diagnostic only."""
import os
import sys

import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
from dilabhelmholtzoct_amd import data, kernels as K  # noqa: E402
from dilabhelmholtzoct_amd.decoder import MaskDecoder  # noqa: E402
from dilabhelmholtzoct_amd.model import SamModel  # noqa: E402
from dilabhelmholtzoct_amd.train import FusedTrainStep, class_confusion, class_dice, mean_dice, predict_masks  # noqa: E402
from oracle.step_ref import synthetic_state_dict  # noqa: E402
from test_gpu_val_dice import _batches  # noqa: E402

_fused = MaskDecoder._dw


def _separate(self, dy, x, M, out, *, db=None, dbx=None, dbx_fold=1, **kw):
    _fused(self, dy, x, M, out, **kw)
    O, I = out.shape
    ldy = kw.get("ldy") or O
    ldx = kw.get("ldx") or I
    if db is not None:
        K.colsum(dy.view(-1, ldy)[:M, :O].contiguous(), M, O, db)
    if dbx is not None:
        K.colsum(x.view(-1, ldx)[:M, :I].contiguous().view(M * dbx_fold, I // dbx_fold), M * dbx_fold,
                 I // dbx_fold, dbx)
    return out


cuda = torch.device("cuda:0")
state = synthetic_state_dict("facebook/sam-vit-base", seed=0)
trains_cpu, val_cpu = _batches()
trains = [data.to_device_batch(t, cuda) for t in trains_cpu]
val = data.to_device_batch(val_cpu, cuda)
grads, dice = {}, {}
for mode in ("fused", "separate"):
    MaskDecoder._dw = _fused if mode == "fused" else _separate
    m = SamModel("facebook/sam-vit-base")
    m.load_state_dict(state)
    m = m.to(cuda)
    step = FusedTrainStep(m, lr=1e-3, topological=True, graphs=False)
    d = []
    for k in range(25):
        if k % 8 == 0:
            step.flush()
            conf = class_confusion(predict_masks(m, val), val["gt_u8"], val["mask_values"])
            d.append(round(mean_dice(conf), 5))
            if k == 16:
                print(mode, "step 16 class Dice", [round(float(x), 4) for x in class_dice(conf)], flush=True)
                print(mode, "step 16 (tp, fp, fn) per class", conf[:, :3].tolist(), flush=True)
        if k == 24:
            break
        step.step(trains[k % 2])
        if k == 0:
            step.flush()
            dec = m.mask_decoder
            grads[mode] = {n: dec.G(n).detach().clone() for n in dec._regions}
    dice[mode] = d
    print(mode, "val Dice", d, flush=True)
worst = []
for n, g in grads["fused"].items():
    r = grads["separate"][n]
    den = r.abs().max().item()
    if den > 0:
        worst.append(((g - r).abs().max().item() / den, n))
worst.sort(reverse=True)
print("largest per-parameter max|diff|/max|g| after step 1:")
for e, n in worst[:8]:
    print(f"  {e:.3e}  {n}")
