"""How well-conditioned are tests/test_gpu_val_dice.py's checkpoints? The fp32 oracle (oracle/step_ref.py) is
trained from the test's synthetic weights and from copies perturbed at rounding level (every weight times
1 + 2^-E * N(0, 1); E = 22: a few fp32 ulps, E = 9: bf16 rounding), on the test's batches, and scored at the
test's checkpoints.
The spread of those oracle trajectories is the Dice change that rounding alone causes. Diagnostic only:
python tests/diag/dice_sensitivity.py (GPU box)."""
import os
import sys

import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
from oracle.step_ref import CpuReferenceStep, synthetic_state_dict  # noqa: E402
from test_gpu_val_dice import CHECKPOINTS, LR, NAME, _batches, _ref_dice  # noqa: E402

cuda = torch.device("cuda:0")
state = synthetic_state_dict(NAME, seed=0)
trains_cpu, val_cpu = _batches()
for run in range(int(os.environ.get("RUNS", "4"))):
    st = state
    if run:
        g = torch.Generator().manual_seed(run)
        st = {k: (v * (1 + 2.0 ** -float(os.environ.get("E", "22")) * torch.randn(v.shape, generator=g)) if v.is_floating_point() else v)
              for k, v in state.items()}
    ref = CpuReferenceStep(NAME, topological=True, lr=LR, state_dict=st, device=cuda, loss_device=cuda)
    d = []
    for k in range(CHECKPOINTS[-1] + 1):
        if k in CHECKPOINTS:
            with torch.no_grad():
                d.append(round(_ref_dice(ref.predict(val_cpu), val_cpu), 5))
        if k == CHECKPOINTS[-1]:
            break
        ref.step(trains_cpu[k % 2])
    print("perturbed" if run else "exact    ", run, d, flush=True)
