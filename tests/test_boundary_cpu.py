"""Drop-in boundary on CPU (no GPU calls): the CLI mirror's flags (ref:octsam/models/training.py:20-93,
README's --top=True), SamModel.from_pretrained's offline weight lookup (training_utils.py:273-280), and the
on-disk formats of §8(f)4 — a datasets save_to_disk split read by train._load_split
(preprocessing_utils.py:92-98 -> training_utils.py:282-287) and the saved .pt state dict loading into
transformers' SamModel as ref:octsam/inference/app.py:15 does."""
import os
import warnings

import numpy as np
import pytest
import torch


@pytest.mark.parametrize("argv,want", [([], False), (["--top"], True), (["--top=True"], True),
                                        (["--top=False"], False), (["--top", "true"], True)])
def test_cli_top_flag(argv, want):
    from dilabhelmholtzoct_amd.train import build_parser
    assert build_parser().parse_args(argv).top is want


def test_cli_rejects_bad_top():
    from dilabhelmholtzoct_amd.train import build_parser
    with pytest.raises(SystemExit):
        build_parser().parse_args(["--top=maybe"])


def test_cli_defaults_match_reference():
    from dilabhelmholtzoct_amd.train import build_parser
    a = build_parser().parse_args([])
    assert (a.base_model, a.lr, a.weight_decay, a.epochs, a.bs, a.prompt) == (
        "facebook/sam-vit-base", 1e-3, 0, 10, 2, "bboxes")


def test_from_pretrained_reads_local_hf_cache(tmp_path, monkeypatch):
    from safetensors.torch import save_file
    from dilabhelmholtzoct_amd.model import SamModel
    src = SamModel("facebook/sam-vit-base")
    src.init_weights(seed=3)
    snap = tmp_path / "hub" / "models--facebook--sam-vit-base" / "snapshots" / "abc123"
    snap.mkdir(parents=True)
    save_file({k: v.clone().contiguous() for k, v in src.state_dict().items()}, str(snap / "model.safetensors"))
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "hub"))
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # found weights: no warning
        m = SamModel.from_pretrained("facebook/sam-vit-base")
    assert m.weights_path.endswith("model.safetensors")
    for k, v in src.state_dict().items():
        assert torch.equal(m.state_dict()[k], v), k
    # a save_pretrained-style directory
    m2 = SamModel.from_pretrained(str(snap))
    assert m2.weights_path == str(snap / "model.safetensors")


def test_from_pretrained_warns_without_weights(tmp_path, monkeypatch):
    from dilabhelmholtzoct_amd.model import SamModel
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "empty"))
    monkeypatch.setenv("HF_HOME", str(tmp_path / "home"))
    with pytest.warns(UserWarning, match="no local weights"):
        m = SamModel.from_pretrained("facebook/sam-vit-base")
    assert m.weights_path is None
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # explicit opt-in to random weights: silent
        m2 = SamModel.from_pretrained("facebook/sam-vit-base", seed=0)
    for k, v in m.state_dict().items():
        assert torch.equal(m2.state_dict()[k], v)


def test_saved_state_dict_loads_into_transformers_sam(tmp_path):
    """training_utils.py:77 saves model.state_dict(); app.py:15 loads it into transformers' SamModel."""
    from transformers import SamModel as HFSam
    from dilabhelmholtzoct_amd.model import SamModel
    from oracle.step_ref import hf_config
    m = SamModel("facebook/sam-vit-base")
    m.init_weights(seed=1)
    path = tmp_path / "octsam_run.pt"
    torch.save(m.state_dict(), path)
    hf = HFSam(hf_config("facebook/sam-vit-base"))
    sd = torch.load(path, map_location="cpu", weights_only=True)
    res = hf.load_state_dict(sd, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    hsd = hf.state_dict()
    for k, v in sd.items():
        assert torch.equal(hsd[k], v), k
    # and back: an HF state dict loads into the drop-in
    back = SamModel("facebook/sam-vit-base")
    back.load_state_dict(hf.state_dict())
    for k, v in back.state_dict().items():
        assert torch.equal(v, hsd[k]), k


def test_save_to_disk_dataset_roundtrip(tmp_path):
    """preprocessing_utils.py:20-25,92-98 layout: a DatasetDict with train/test splits of {image, label}
    Image columns, save_to_disk; train._load_split reads it the way prepare_data does (:282-287) and
    SAMDataset yields the same prompts as from the in-memory items."""
    import datasets
    from PIL import Image
    from dilabhelmholtzoct_amd import data, train
    items = data.synthetic_oct(seed=4, n=3)
    feats = datasets.Features({"image": datasets.Image(), "label": datasets.Image()})
    d = {"image": [Image.fromarray(it["image"]) for it in items],
         "label": [Image.fromarray(it["label"]) for it in items]}
    ds = datasets.Dataset.from_dict(d, features=feats)
    dd = datasets.DatasetDict({"train": ds.select([0, 1]), "test": ds.select([2])})
    path = str(tmp_path / "processed")
    dd.save_to_disk(path)
    tr = train._load_split({"dataset": path}, "train")
    te = train._load_split({"dataset": path}, "test")
    assert len(tr) == 2 and len(te) == 1
    a = data.SAMDataset(tr, {"prompt_type": "bboxes"}, epoch_seed=0)
    b = data.SAMDataset(items[:2], {"prompt_type": "bboxes"}, epoch_seed=0)
    for i in range(2):
        x, y = a[i], b[i]
        assert np.array_equal(x[0], y[0]) and x[1] == y[1] and x[3] == y[3]
        assert all(np.array_equal(p, q) for p, q in zip(x[2], y[2]))


def test_training_without_gpu_raises_cleanly():
    """train.training() has no CPU fallback (every op of the step is a HIP kernel; the reference's own CPU step is
    oracle/step_ref.py, test infrastructure): on a host without a GPU, or asked for a CPU device, it raises with a
    message instead of failing somewhere inside the data path (ref:octsam/models/training_utils.py:33)."""
    import pytest
    import torch
    from dilabhelmholtzoct_amd.train import training
    cfg = {"batch_size": 1, "epochs": 1, "prompt_type": "bboxes", "evaluate": False, "checkpoint": None}
    with pytest.raises(ValueError, match="GPU device"):
        training("facebook/sam-vit-base", cfg, [], [], device=torch.device("cpu"), log=lambda *a: None)
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="needs an MI355X"):
            training("facebook/sam-vit-base", cfg, [], [], log=lambda *a: None)
