"""Val-Dice trajectories over 24 training steps (configs[2] batches, B = 8): fp32 oracle, the same oracle
under torch.autocast(bfloat16), and the HIP path; measures how far a plain bf16 model drifts from fp32."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from dilabhelmholtzoct_amd import data
from dilabhelmholtzoct_amd.model import SamModel
from dilabhelmholtzoct_amd.train import FusedTrainStep, class_confusion, mean_dice, predict_masks
from oracle.step_ref import CpuReferenceStep, synthetic_state_dict
from oracle.eval_ref import evaluate_metrics_ref

NAME = "facebook/sam-vit-base"
dev = torch.device("cuda", 0)
LR = float(sys.argv[1]) if len(sys.argv) > 1 else 3e-3
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 24
proc = data.make_processor()


def mk(seed, n):
    ds = data.synthetic_oct(seed=seed, n=n)
    sd = data.SAMDataset(ds, {"prompt_type": "bboxes"}, epoch_seed=0)
    return data.process_batch(proc, data.custom_collate([sd[i] for i in range(len(sd))]), "bboxes")


trains_cpu, val_cpu = [mk(1000, 8), mk(1001, 8)], mk(999, 8)
trains = [data.to_device_batch(t, dev) for t in trains_cpu]
val = data.to_device_batch(val_cpu, dev)
state = synthetic_state_dict(NAME, seed=0)


def ref_dice(masks):
    r = evaluate_metrics_ref([masks[b].cpu() for b in range(8)], [val_cpu["gt_u8"][b] for b in range(8)],
                             [val_cpu["mask_values"][b].tolist() for b in range(8)])
    return float(np.mean(r["category"]["dice"]))


class AutocastRef(CpuReferenceStep):
    def predict(self, batch):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return super().predict(batch).float()


runs = {}
for name in ("fp32", "bf16_autocast", "hip"):
    torch.manual_seed(0)
    if name == "hip":
        m = SamModel(NAME)
        m.load_state_dict(state)
        m = m.to(dev)
        st = FusedTrainStep(m, lr=LR, topological=True)
        ev = lambda: mean_dice(class_confusion(predict_masks(m, val), val["gt_u8"], val["mask_values"]))
        stepf = lambda k: st.step(trains[k % 2])
    else:
        cls = CpuReferenceStep if name == "fp32" else AutocastRef
        r = cls(NAME, topological=True, lr=LR, state_dict=state, device=dev, loss_device=dev)
        ev = lambda r=r: ref_dice(r.predict(val_cpu).float())
        stepf = lambda k, r=r: r.step(trains_cpu[k % 2])
    out = []
    for k in range(STEPS + 1):
        if k % 4 == 0:
            if name == "hip":
                st.flush()
            with torch.no_grad():
                out.append(round(ev(), 5))
        if k < STEPS:
            stepf(k)
    runs[name] = out
    print(name, out, flush=True)
for name in ("bf16_autocast", "hip"):
    print(name, "max |diff vs fp32|", max(abs(a - b) for a, b in zip(runs[name], runs["fp32"])))
