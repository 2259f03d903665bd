"""Val-Dice parity (BASELINE.json north_star: "val Dice within ±0.005 of the CPU reference on identical seeds") on
SURVEY.md §8(d)'s protocol: 128 synthetic training scans and 32 held-out ones, B = 8, box prompts, --top=True,
lr 1e-3 (the reference CLI's default), the reference's prompt redraw every epoch (SAMDataset.__getitem__), the
held-out Dice after EVERY epoch asserted, not only the last.

Start point. From the random initial weights every run first collapses to all-foreground masks (specificity ~0),
and the step at which it leaves that state is chaotic (profiles/r03/valdice_traj_*.jsonl). Both sides therefore
start from a decoder past that transition: tests/golden/valdice_start_decoder.safetensors (the fp32 oracle after
256 steps on another synthetic set, training seed 2000 / held-out seed 3000; encoder and prompt encoder: the
synthetic weights, seed 0).

Warm optimizer. Round 3 started both sides with a COLD Adam at that decoder: the first bias-corrected steps are
lr-sized in every coordinate, both sides fall from Dice 0.79 to ~0.45 within 4 steps and climb back, and inside
that dip the oracle's OWN spread under bf16-rounding-sized weight perturbations (1 + 2^-8 u per weight) or
bf16-rounded image embeddings is 0.477-0.507 at step 16 (profiles/r04/valdice_spread.jsonl) -- a HIP-vs-oracle
difference there (round 3: +0.025) measures that chaos, not the implementation. Here the start decoder first takes
WARM steps of the same training on its own set (seed 2000; HIP, the start state only has to be identical on both
sides), and BOTH sides then resume from those weights and that Adam state (FusedTrainStep.optimizer_state ->
torch.optim.Adam state by name), so no cold first step sits inside the compared trajectory.

Then both sides train EPOCHS epochs on this test's own 128 scans (seed 2001) and are scored on its 32 held-out
scans (seed 3001) after every epoch:
* ours: FusedTrainStep exactly as bench.py runs it (hipGraphs + the encoder lookahead), predict_masks +
  class_confusion (HIP confusion counts);
* oracle: oracle/step_ref.py (transformers SamModel fp32 -- on the GPU only to keep the test short; the frozen
  encoder's embeddings computed once per batch -- restated DiceCE / topo loss, torch Adam), scored by
  oracle/eval_ref.pooled_confusion_ref (the reference's threshold and break quirk, training_utils.py:126-156).
Asserted: the oracle is in the non-degenerate regime (mean specificity > 0.5), the compared epochs actually trained
(the oracle's decoder moved by more than 1 % in norm and its Dice changed), and |Dice_ours - Dice_oracle| <= 0.005
at every epoch checkpoint."""
import contextlib
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

NAME = "facebook/sam-vit-base"
TOL = 0.005
LR = 1e-3
WARM = 64
EPOCHS = 4
BS = 8
START = os.path.join(os.path.dirname(__file__), "golden", "valdice_start_decoder.safetensors")


def _epoch_batches(seed, n, epoch):
    from dilabhelmholtzoct_amd import data
    proc = data.make_processor()
    sd = data.SAMDataset(data.synthetic_oct(seed=seed, n=n), {"prompt_type": "bboxes"}, epoch_seed=seed)
    sd.epoch = epoch
    return [data.process_batch(proc, data.custom_collate([sd[i] for i in range(s, min(n, s + BS))]), "bboxes")
            for s in range(0, n, BS)]


def warm_start(cuda, state):
    """The start decoder after WARM steps on its own training set (seed 2000) with the HIP step: decoder weights
    (fp32, HF names) and the Adam state (HF names)."""
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    model = SamModel(NAME)
    model.load_state_dict(state)
    model = model.to(cuda)
    step = FusedTrainStep(model, lr=LR, topological=True, graphs=True, pipeline=True)
    k, ep = 0, 0
    while k < WARM:
        tr = [data.to_device_batch(b, cuda) for b in _epoch_batches(2000, 128, ep)]
        for i, b in enumerate(tr):
            if k >= WARM:
                break
            step.step(b, next_batch=tr[i + 1] if i + 1 < len(tr) and k + 1 < WARM else None)
            k += 1
        ep += 1
    adam = step.optimizer_state()
    weights = {"mask_decoder." + n: t.detach().float().cpu().clone() for n, t in model.mask_decoder.state_dict().items()}
    del step, model
    torch.cuda.empty_cache()
    return weights, adam


@contextlib.contextmanager
def oracle_mode():
    """The oracle's torch ops, run to run reproducible: MIOpen off (its solution choice for the decoder's ConvTranspose2d
    depends on what ran before in the process) and torch's deterministic algorithms (index/scatter backwards without
    atomics). The protocol is chaotic, so an oracle that is not bit-reproducible across processes cannot anchor
    committed values (a whole-suite run once moved the oracle's step-64 Dice by 0.036 against a standalone run)."""
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        with torch.backends.cudnn.flags(enabled=False):
            yield
    finally:
        torch.use_deterministic_algorithms(prev)


def warm_fingerprint(weights):
    """(sum, sum of squares) of the warm decoder's weights in float64: identifies the HIP warm state the committed
    oracle values (tests/golden/valdice_oracle.json) were made from -- bench.py compares it before quoting them."""
    s = sum(float(t.double().sum()) for t in weights.values())
    q = sum(float((t.double() ** 2).sum()) for t in weights.values())
    return [round(s, 6), round(q, 6)]


def load_torch_adam(opt, module, adam):
    """FusedTrainStep.optimizer_state() -> torch.optim.Adam state (parameters that never had a gradient, the IoU
    head, keep no state in torch)."""
    for name, p in module.named_parameters():
        m, v = adam[f"exp_avg.mask_decoder.{name}"], adam[f"exp_avg_sq.mask_decoder.{name}"]
        if not bool(v.any()):
            continue
        opt.state[p] = {"step": torch.tensor(float(adam["step"])), "exp_avg": m.to(p.device).clone(),
                        "exp_avg_sq": v.to(p.device).clone()}


def test_val_dice_parity(cuda):
    from safetensors.torch import load_file
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep, class_confusion, predict_masks
    from oracle.eval_ref import mean_dice_ref, mean_specificity_ref, pooled_confusion_ref
    from oracle.step_ref import CpuReferenceStep, synthetic_state_dict

    state = synthetic_state_dict(NAME, seed=0)
    start = {k: v.float() for k, v in load_file(START).items()}
    for k, v in start.items():
        assert k in state and state[k].shape == v.shape, k
        state[k] = v
    weights, adam = warm_start(cuda, state)
    state.update(weights)

    val_cpu = _epoch_batches(3001, 32, 0)
    val = [data.to_device_batch(v, cuda) for v in val_cpu]
    with oracle_mode():
        ref = CpuReferenceStep(NAME, topological=True, lr=LR, state_dict=state, device=cuda, loss_device=cuda)
    load_torch_adam(ref.opt, ref.model.mask_decoder, adam)
    with oracle_mode():
        val_emb = [ref.embed(v) for v in val_cpu]
    w0 = torch.cat([p.detach().flatten() for p in ref.model.mask_decoder.parameters()]).clone()

    def ref_conf():
        c = torch.zeros(14, 4, dtype=torch.int64)
        with torch.no_grad(), oracle_mode():
            for v, e in zip(val_cpu, val_emb):
                c += pooled_confusion_ref(ref.predict(v, e), v["gt_u8"], v["mask_values"])
        return c

    ours = SamModel(NAME)
    ours.load_state_dict(state)
    ours = ours.to(cuda)
    step = FusedTrainStep(ours, lr=LR, topological=True, graphs=True, pipeline=True)
    step.load_optimizer_state(adam)

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
    c_ref = None
    for ep in range(EPOCHS):
        tr_cpu = _epoch_batches(2001, 128, ep)
        tr = [data.to_device_batch(b, cuda) for b in tr_cpu]
        for i, b in enumerate(tr):
            step.step(b, next_batch=tr[i + 1] if i + 1 < len(tr) else None)
            with oracle_mode():
                if i not in emb_cache:
                    emb_cache[i] = ref.embed(tr_cpu[i])
                ref.step(tr_cpu[i], emb_cache[i])
            k += 1
        c_ref = ref_conf()
        results.append((k, dice3(ours_conf()), mean_dice_ref(c_ref)))
    spec = mean_specificity_ref(c_ref)
    w1 = torch.cat([p.detach().flatten() for p in ref.model.mask_decoder.parameters()])
    moved = float((w1 - w0).norm() / w0.norm())
    for kk, got, want in results:
        print(f"after {kk:3d} steps: val Dice HIP {got:.5f}  oracle {want:.5f}  diff {got - want:+.5f}")
    fp = warm_fingerprint(weights)
    print(f"warm-state fingerprint {fp}")
    if os.environ.get("OCTSAM_VALDICE_OUT"):  # regenerating tests/golden/valdice_oracle.json (scripts/gpu_valdice_golden.sh)
        import json
        with open(os.environ["OCTSAM_VALDICE_OUT"], "w") as f:
            json.dump({"steps": [kk for kk, _, _ in results], "oracle_dice": [round(w, 5) for _, _, w in results],
                       "hip_dice_in_that_run": [round(g, 5) for _, g, _ in results], "warm_fingerprint": fp,
                       "oracle_specificity": round(spec, 4), "oracle_moved": round(moved, 4)}, f, indent=1)
    print(f"oracle specificity at the end {spec:.4f}; oracle decoder moved {moved:.4f} (relative norm)")
    assert spec > 0.5, f"oracle specificity {spec:.4f}: the degenerate all-foreground regime"
    assert moved > 0.01, f"the oracle's decoder barely moved ({moved:.4g}): the compared epochs did not train"
    assert abs(results[-1][2] - results[0][2]) > 1e-4, "the oracle's val Dice never changed"
    bad = [(kk, got, want) for kk, got, want in results if abs(got - want) > TOL]
    assert not bad, f"|Dice_HIP - Dice_oracle| > {TOL} at {bad}"
