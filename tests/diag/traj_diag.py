"""Where does the HIP training trajectory leave the fp32 oracle's? Both train from the val-Dice test's synthetic
weights on its batches (lr 1e-3); at checkpoints: val logit statistics (mean, fraction > 0, mean |diff| vs the
oracle) and the decoder parameters that moved furthest from the oracle's (relative to how far the oracle's
moved from the start). Diagnostic only: python tests/diag/traj_diag.py [steps] (GPU box)."""
import os
import sys

import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
from dilabhelmholtzoct_amd import data  # noqa: E402
from dilabhelmholtzoct_amd.model import SamModel  # noqa: E402
from dilabhelmholtzoct_amd.train import FusedTrainStep, predict_masks  # noqa: E402
from oracle.step_ref import CpuReferenceStep, synthetic_state_dict  # noqa: E402
from test_gpu_val_dice import LR, NAME, _batches  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 16
cuda = torch.device("cuda:0")
state = synthetic_state_dict(NAME, seed=0)
trains_cpu, val_cpu = _batches()
trains = [data.to_device_batch(t, cuda) for t in trains_cpu]
val = data.to_device_batch(val_cpu, cuda)
m = SamModel(NAME)
m.load_state_dict(state)
m = m.to(cuda)
step = FusedTrainStep(m, lr=LR, topological=True, graphs=False)
ref = CpuReferenceStep(NAME, topological=True, lr=LR, state_dict=state, device=cuda, loss_device=cuda)


class AutocastRef(CpuReferenceStep):  # the oracle trained under torch.autocast(bfloat16): a plain bf16 model
    def predict(self, batch):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return super().predict(batch).float()


aref = AutocastRef(NAME, topological=True, lr=LR, state_dict=state, device=cuda, loss_device=cuda)
p0 = {n: p.detach().clone() for n, p in ref.model.mask_decoder.named_parameters()}
for k in range(STEPS + 1):
    if k % 4 == 0:
        step.flush()
        with torch.no_grad():
            a = predict_masks(m, val).float()
            b = ref.predict(val_cpu).float().to(cuda)
            c = aref.predict(val_cpu).float().to(cuda)
        print(f"step {k:2d}: logits ours mean {a.mean():+.4f} >0 {(a > 0).float().mean():.4f} | oracle mean "
              f"{b.mean():+.4f} >0 {(b > 0).float().mean():.4f} | autocast {c.mean():+.4f} | mean|diff| ours "
              f"{(a - b).abs().mean():.4f} autocast {(c - b).abs().mean():.4f}", flush=True)
    if k == STEPS:
        break
    step.step(trains[k % 2])
    ref.step(trains_cpu[k % 2])
    aref.step(trains_cpu[k % 2])
step.flush()
ours = dict(m.mask_decoder.named_parameters())
auto = dict(aref.model.mask_decoder.named_parameters())
rows = []
for n, r in ref.model.mask_decoder.named_parameters():
    moved = (r.detach() - p0[n]).norm().item()
    dev = (ours[n].detach().float() - r.detach()).norm().item()
    adev = (auto[n].detach().float() - r.detach()).norm().item()
    if moved > 0:
        rows.append((dev / moved, adev / moved, moved, n))
rows.sort(reverse=True)
print("decoder parameters, |x - oracle| / |oracle - start| after", STEPS, "steps (x = ours, autocast):")
for q, qa, mv, n in rows[:25]:
    print(f"  ours {q:9.3f}  autocast {qa:9.3f}  moved {mv:.3e}  {n}")
qs = [r[0] for r in rows if "k_proj.bias" not in r[3]]
qa = [r[1] for r in rows if "k_proj.bias" not in r[3]]
print(f"median over parameters (k_proj biases excluded): ours {sorted(qs)[len(qs) // 2]:.3f} autocast "
      f"{sorted(qa)[len(qa) // 2]:.3f}")
