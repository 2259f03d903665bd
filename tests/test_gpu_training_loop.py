"""The training loop mirror (train.training, ref:octsam/models/training_utils.py:27-80) end to end on the GPU:
first-batch skip, train / validation losses, Dice evaluation — once with SamProcessor on the host and once
with the HIP image processor (preprocess.DeviceProcessor). The processor kernel is bit-identical and every
step kernel deterministic, so the two runs must agree exactly."""
import math

import pytest

pytestmark = pytest.mark.gpu


def _run(cuda, gpu_processor):
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.train import training
    cfg = {"batch_size": 2, "epochs": 1, "learning_rate": 1e-3, "topological": True, "prompt_type": "bboxes",
           "evaluate": True, "checkpoint": None, "data_seed": 0, "gpu_processor": gpu_processor}
    return training("facebook/sam-vit-base", cfg, data.synthetic_oct(seed=0, n=6), data.synthetic_oct(seed=1, n=2),
                    device=cuda)


def test_training_loop_host_vs_device_processor(cuda):
    host = _run(cuda, False)
    dev = _run(cuda, True)
    print("host processor:", host)
    print("HIP processor: ", dev)
    for h in (host, dev):
        assert len(h["train_loss"]) == 1 and len(h["valid_loss"]) == 1
        assert all(math.isfinite(v) for v in h["train_loss"] + h["valid_loss"])
        assert 0.0 <= h["mean_dice"] <= 1.0
    assert host["train_loss"] == dev["train_loss"]
    assert host["valid_loss"] == dev["valid_loss"]
    assert host["mean_dice"] == dev["mean_dice"]
