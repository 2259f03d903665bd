"""GPU prompt / gt generation (csrc/components.hip via dilabhelmholtzoct_amd.components) against
(1) the reference's own SAMDataset/custom_collate outputs (tests/golden/data_golden.npz, generated from
ref:octsam/models/training_utils.py:381-458 with per-item seeds) — prompts, gt bits, mask values exact;
(2) the host path (data.SAMDataset + process_batch, scipy.ndimage.label) on synthetic OCT batches;
(3) scipy.ndimage.label directly on adversarial maps (noise with diagonal-only contacts, spirals, one
value, one-pixel lines, unaligned widths)."""
import os
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "data_golden.npz"))


def _hooks(seeds):
    def mk(s):
        def f():
            np.random.seed(int(s))
            random.seed(int(s))
        return f
    return [mk(s) for s in seeds]


@pytest.mark.parametrize("prompt", ["bboxes", "points"])
def test_components_match_reference_golden(cuda, prompt):
    from dilabhelmholtzoct_amd.components import collate_device
    labs = G["labels"]
    imgs = np.stack([np.repeat((lab * 18)[:, :, None], 3, 2).astype(np.uint8) for lab in labs])
    out = collate_device(imgs, labs, prompt, cuda, seed_hooks=_hooks(G["seeds"]))
    assert np.array_equal(out["prompt_raw"].numpy(), G[f"{prompt}_prompt"])
    gt = out["gt_u8"].cpu().numpy()
    assert gt.shape == tuple(G[f"{prompt}_gt_shape"])
    assert np.array_equal(np.packbits(gt, axis=-1), G[f"{prompt}_gt_bits"])
    assert np.array_equal(out["mask_values"].numpy(), G[f"{prompt}_mask_values"])


@pytest.mark.parametrize("prompt", ["bboxes", "points", "both", "boxes"])
def test_components_match_host_path(cuda, prompt):
    """"boxes" (any unrecognised --prompt string) means bboxes, as SAMDataset.__getitem__ decides."""
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.components import collate_device
    ds = data.synthetic_oct(seed=11, n=4)
    sd = data.SAMDataset(ds, {"prompt_type": prompt}, epoch_seed=5)
    sd.epoch = 2
    want = data.process_batch(data.make_processor(), data.custom_collate([sd[i] for i in range(4)]), prompt)
    imgs = np.stack([np.array(ds[i]["image"]) for i in range(4)])
    labs = np.stack([np.array(ds[i]["label"]) for i in range(4)])
    hooks = [lambda i=i: data.seed_sample(2, i, 5) for i in range(4)]
    got = collate_device(imgs, labs, prompt, cuda, seed_hooks=hooks)
    keys = {"points": ["input_points"], "both": ["input_boxes", "input_points"]}.get(prompt, ["input_boxes"])
    for key in keys:
        assert torch.equal(got[key], want[key]), key
    assert torch.equal(got["gt_u8"].cpu(), want["gt_u8"])
    assert torch.equal(got["mask_values"], want["mask_values"])
    assert torch.equal(got["pixel_values"].cpu(), want["pixel_values"])


def _scipy_rank(lab):
    from scipy.ndimage import label
    rank = np.full(lab.shape, -1, dtype=np.int64)
    n0 = 0
    for v in np.unique(lab):
        lb, n = label(lab == v, np.ones((3, 3), dtype=np.int32))
        rank[lb > 0] = lb[lb > 0] - 1 + n0
        n0 += n
    return rank, n0


def _spiral(n):
    a = np.zeros((n, n), dtype=np.uint8)
    y, x, dy, dx = 0, 0, 0, 1
    lo, hi = 0, n - 1
    for _ in range(n * n):
        a[y, x] = 1
        ny, nx = y + dy, x + dx
        if not (0 <= ny < n and 0 <= nx < n) or a[ny, nx] or (
                0 <= ny + dy < n and 0 <= nx + dx < n and a[ny + dy, nx + dx]):
            dy, dx = dx, -dy
            ny, nx = y + dy, x + dx
            if not (0 <= ny < n and 0 <= nx < n) or a[ny, nx]:
                break
        y, x = ny, nx
    return a


def _cases():
    rng = np.random.RandomState(3)
    yield "noise3", rng.randint(0, 3, (64, 80)).astype(np.uint8)
    yield "diag", (np.add.outer(np.arange(48), np.arange(64)) % 2).astype(np.uint8)  # checkerboard: 2 comps
    yield "spiral", _spiral(96)
    yield "const", np.full((33, 47), 7, dtype=np.uint8)
    ln = np.zeros((40, 50), dtype=np.uint8)
    ln[::3] = 1
    yield "lines", ln
    yield "noise2_odd", rng.randint(0, 2, (37, 53)).astype(np.uint8)


@pytest.mark.parametrize("name,lab", list(_cases()), ids=[c[0] for c in _cases()])
def test_components_match_scipy(cuda, name, lab):
    from dilabhelmholtzoct_amd.components import DeviceComponents
    want, n = _scipy_rank(lab)
    labs = torch.from_numpy(np.stack([lab, lab[::-1, ::-1].copy()])).to(cuda)
    out = DeviceComponents(cuda)(labs, want_gt=False)
    comp = out["comp"].cpu().numpy()
    assert out["ncomp"][0] == n
    assert np.array_equal(comp[0], want), name
    w1, n1 = _scipy_rank(lab[::-1, ::-1].copy())
    assert out["ncomp"][1] == n1 and np.array_equal(comp[1], w1)
    for c in range(n):  # statistics vs numpy
        ys, xs = np.nonzero(want == c)
        assert list(out["stats"][0][c]) == [xs.min(), xs.max(), ys.min(), ys.max(), len(xs)]


def test_components_too_many(cuda):
    from dilabhelmholtzoct_amd.components import DeviceComponents
    lab = (np.add.outer(np.arange(64), np.arange(64)) % 2).astype(np.uint8)
    lab[::2, :] = 2 + (np.arange(64) % 2)[None, :]  # stripes of isolated pixels: > 16 components
    from dilabhelmholtzoct_amd.components import ComponentLimitError
    with pytest.raises(ComponentLimitError):
        DeviceComponents(cuda, max_components=16)(torch.from_numpy(lab[None]).to(cuda))


def test_training_falls_back_to_host_path_beyond_limits(cuda, monkeypatch):
    """A label map beyond the device path's component limit is built by the host path (the reference has no
    such limit): train._prep returns the host items instead of raising."""
    from dilabhelmholtzoct_amd import components, data, train
    monkeypatch.setattr(components, "MAX_COMPONENTS", 4)
    orig = components.DeviceComponents.__init__
    monkeypatch.setattr(components.DeviceComponents, "__init__",
                        lambda self, device, max_components=4: orig(self, device, 4))
    ds = data.synthetic_oct(seed=3, n=2)
    sd = data.SAMDataset(ds, {"prompt_type": "bboxes"}, epoch_seed=1)
    kind, state, n = train._prep(sd, [0, 1], "bboxes", cuda, True)
    assert kind == "host" and n == max(len(state[0][3]), len(state[1][3])) > 4
