"""The training loop mirror (train.training, ref:octsam/models/training_utils.py:27-80) end to end on the GPU:
first-batch skip, train / validation losses, Dice evaluation — with the reference's host data path
(SAMDataset + scipy components + SamProcessor), with the HIP image processor only, and with the full HIP
data path (components / prompts / gt + processor). Every data kernel is bit-identical and every step kernel
deterministic, so all runs must agree exactly; both per-item seeding (data_seed) and the global RNG
stream (no data_seed) are covered."""
import math
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(cuda, gpu_processor, gpu_components, data_seed, prompt="bboxes", **extra):
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.train import training
    np.random.seed(123)
    random.seed(123)
    cfg = {"batch_size": 2, "epochs": 1, "learning_rate": 1e-3, "topological": True, "prompt_type": prompt,
           "evaluate": True, "checkpoint": None, "data_seed": data_seed, "gpu_processor": gpu_processor,
           "gpu_components": gpu_components, **extra}
    return training("facebook/sam-vit-base", cfg, data.synthetic_oct(seed=0, n=6), data.synthetic_oct(seed=1, n=2),
                    device=cuda)


@pytest.mark.parametrize("data_seed,prompt", [(0, "bboxes"), (None, "points"), (0, "both")])
def test_training_loop_host_vs_device_data_path(cuda, data_seed, prompt):
    runs = {"host": _run(cuda, False, False, data_seed, prompt),
            "hip processor": _run(cuda, True, False, data_seed, prompt),
            "hip data path": _run(cuda, True, True, data_seed, prompt)}
    for name, h in runs.items():
        print(f"{name:14s}: train {h['train_loss']} valid {h['valid_loss']} mean dice {h['mean_dice']}")
        assert len(h["train_loss"]) == 1 and len(h["valid_loss"]) == 1
        assert all(math.isfinite(v) for v in h["train_loss"] + h["valid_loss"])
        assert 0.0 <= h["mean_dice"] <= 1.0
    ref = runs["host"]
    for name in ("hip processor", "hip data path"):
        for key in ("train_loss", "valid_loss", "mean_dice", "dice"):
            assert runs[name][key] == ref[key], (name, key)


def test_training_loop_graphs_and_lookahead(cuda):
    """config graphs / pipeline: hipGraph replay and the encoder lookahead (the next batch built one step ahead)
    give the eager loop's numbers exactly (6 scans -> 2 steps per epoch after the skip, 2 epochs)."""
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.train import training
    out = []
    for extra in ({}, {"graphs": True, "pipeline": True}):
        np.random.seed(123)
        random.seed(123)
        cfg = {"batch_size": 2, "epochs": 2, "learning_rate": 1e-3, "topological": True, "prompt_type": "bboxes",
               "evaluate": True, "checkpoint": None, "data_seed": 0, **extra}
        out.append(training("facebook/sam-vit-base", cfg, data.synthetic_oct(seed=0, n=6),
                            data.synthetic_oct(seed=1, n=2), device=cuda))
    for key in ("train_loss", "valid_loss", "mean_dice", "dice"):
        assert out[0][key] == out[1][key], key
