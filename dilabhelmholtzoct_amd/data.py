"""Host data path of the OCT-SAM step (ref:octsam/models/training_utils.py:282-287, :381-458) and a
synthetic OCT-like dataset standing in for the private 552-image set (ref:README.md:17).

* ``synthetic_oct(seed, n)``   — 496x512 label maps: 12-13 sinusoidal retinal bands of distinct classes
                                 (class 0 = one background component) + 8 intraretinal-fluid disks
                                 (class 3); image = label*18 + U[0,20) replicated to RGB.
* ``SAMDataset`` / ``custom_collate`` — restatement of the reference's per-image prompt + gt generation
  (scipy.ndimage.label 8-connectivity per unique label value, bbox jitter np.random.randint(-10, 10)
  clamped to [0, W] / [0, H], or one random pixel via random.randrange) and its pad_sequence collate.
  ``seed_sample(epoch, idx)`` re-seeds numpy/random per sample so single- and multi-GPU runs see the
  same prompts.
* ``make_processor()`` — transformers' SamProcessor with the PIL image backend (no hub access): the
  same object the reference builds with from_pretrained (resize longest edge 1024, /255, ImageNet
  normalisation, pad to 1024^2; box coordinates scaled to the resized frame).
* ``to_device_batch`` — moves a processed batch to HBM; gt masks travel as uint8 (exactly 0/1), not the
  reference's float64, a lossless 8x reduction of the largest host->device transfer.
"""
from __future__ import annotations

import random

import numpy as np
import torch

H_OCT, W_OCT = 496, 512
MASK_DICT = (
    "background", "epiretinal membrane", "neurosensory retina", "intraretinal fluid", "subretinal fluid",
    "subretinal hyperreflective material", "retinal pigment epithelium", "pigment epithelial detachment",
    "posterior hyaloid membrane", "choroid border", "imaging artifacts", "fibrosis", "vitreous body",
    "image padding",
)  # ref:octsam/models/training.py:146-162


def synthetic_label(rng: np.random.RandomState, H: int = H_OCT, W: int = W_OCT, n_disks: int = 8) -> np.ndarray:
    """Parallel wavy layers (one connected component per class) + fluid disks inside the thickest
    layer, giving N = 20-21 components per image like the survey's maps."""
    nb = int(rng.randint(12, 14))  # number of layers (bands)
    x = np.arange(W, dtype=np.float64)
    spacing = (H - 60) / (nb - 1)
    base = 30 + spacing * np.arange(nb - 1) + rng.uniform(-spacing / 6, spacing / 6, nb - 1)
    common = rng.uniform(3, 8) * np.sin(2 * np.pi * x / rng.uniform(300, 700) + rng.uniform(0, 2 * np.pi))
    bounds = np.stack([base[k] + common + rng.uniform(0.5, 2.5) * np.sin(2 * np.pi * x / rng.uniform(80, 200)
                                                                         + rng.uniform(0, 2 * np.pi))
                       for k in range(nb - 1)], 0)
    yy = np.arange(H, dtype=np.float64)[:, None]
    band = (yy[None] >= bounds[:, None, :]).sum(0)  # [H, W] layer index 0..nb-1
    classes = [0] + [int(c) for c in rng.permutation([1, 2, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13])][: nb - 1]
    label = np.asarray(classes, np.uint8)[band]
    # intraretinal fluid disks (class 3) strictly inside one interior layer
    k = int(rng.randint(2, nb - 2))
    top, bot = bounds[k - 1], bounds[k]
    for _ in range(n_disks):
        cx = rng.uniform(30, W - 30)
        xi = int(cx)
        mid = 0.5 * (top[xi] + bot[xi])
        half = 0.5 * (bot[xi] - top[xi])
        r = max(2.0, min(rng.uniform(4, 10), half - 4))
        m = (yy - mid) ** 2 + (x[None, :] - cx) ** 2 <= r * r
        label[m] = 3
    return label


def synthetic_oct(seed: int = 0, n: int = 8):
    """list of {"image": uint8 [H,W,3], "label": uint8 [H,W]}."""
    rng = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        lab = synthetic_label(rng)
        img = (lab.astype(np.int32) * 18 + rng.randint(0, 20, lab.shape)).clip(0, 255).astype(np.uint8)
        out.append({"image": np.repeat(img[:, :, None], 3, axis=2), "label": lab})
    return out


def seed_sample(epoch: int, idx: int, base: int = 0):
    s = (base * 1000003 + epoch * 7919 + idx) % (2**31 - 1)
    np.random.seed(s)
    random.seed(s)


class SAMDataset(torch.utils.data.Dataset):
    """ref:octsam/models/training_utils.py:381-447 restated."""

    def __init__(self, dataset, config: dict, epoch_seed: int | None = None):
        self.dataset = dataset
        self.config = config
        self.epoch = 0
        self.epoch_seed = epoch_seed

    def __len__(self):
        return len(self.dataset)

    @staticmethod
    def _components(ground_truth_mask):
        from scipy.ndimage import label
        structure = np.ones((3, 3), dtype=np.int32)
        for v in np.unique(ground_truth_mask):
            binary = np.where(ground_truth_mask == v, 1.0, 0.0)
            labeled, n = label(binary, structure)
            for c in range(n):
                yield v, labeled, c

    def get_bboxes_and_gt_masks(self, ground_truth_mask):
        bboxes, gt_masks, values = [], [], []
        H, W = ground_truth_mask.shape
        for v, labeled, c in self._components(ground_truth_mask):
            values.append(v)
            y_idx, x_idx = np.where(labeled == c + 1)
            x_min, x_max = np.min(x_idx), np.max(x_idx)
            y_min, y_max = np.min(y_idx), np.max(y_idx)
            x_min = max(0, x_min + np.random.randint(-10, 10))
            x_max = min(W, x_max + np.random.randint(-10, 10))
            y_min = max(0, y_min + np.random.randint(-10, 10))
            y_max = min(H, y_max + np.random.randint(-10, 10))
            bboxes.append([x_min, y_min, x_max, y_max])
            gt_masks.append(np.where(labeled == c + 1, 1.0, 0.0))
        return bboxes, gt_masks, values

    def get_bboxes_points_and_gt_masks(self, ground_truth_mask):
        """``--prompt=both`` (build extension for BASELINE configs[4]; the reference CLI has bboxes or points):
        per component, the jittered bbox (4 np.random draws) and then one random pixel (random.randrange)."""
        bboxes, points, gt_masks, values = [], [], [], []
        H, W = ground_truth_mask.shape
        for v, labeled, c in self._components(ground_truth_mask):
            values.append(v)
            y_idx, x_idx = np.where(labeled == c + 1)
            x_min, x_max = np.min(x_idx), np.max(x_idx)
            y_min, y_max = np.min(y_idx), np.max(y_idx)
            x_min = max(0, x_min + np.random.randint(-10, 10))
            x_max = min(W, x_max + np.random.randint(-10, 10))
            y_min = max(0, y_min + np.random.randint(-10, 10))
            y_max = min(H, y_max + np.random.randint(-10, 10))
            bboxes.append([x_min, y_min, x_max, y_max])
            k = random.randrange(0, len(x_idx))
            points.append([[x_idx[k], y_idx[k]]])
            gt_masks.append(np.where(labeled == c + 1, 1.0, 0.0))
        return bboxes, points, gt_masks, values

    def get_points_and_gt_masks(self, ground_truth_mask):
        points, gt_masks, values = [], [], []
        for v, labeled, c in self._components(ground_truth_mask):
            values.append(v)
            y_idx, x_idx = np.where(labeled == c + 1)
            k = random.randrange(0, len(x_idx))
            points.append([[x_idx[k], y_idx[k]]])
            gt_masks.append(np.where(labeled == c + 1, 1.0, 0.0))
        return points, gt_masks, values

    def __getitem__(self, idx):
        if self.epoch_seed is not None:
            seed_sample(self.epoch, idx, self.epoch_seed)
        item = self.dataset[idx]
        image = np.array(item["image"])
        if self.config.get("pseudocolor") is not None:  # ref:octsam/models/training_utils.py:439-440
            from .colormaps import apply_colormap, colormap_lut
            image = apply_colormap(image, colormap_lut(self.config["pseudocolor"]))
        gt = np.array(item["label"])
        if self.config.get("prompt_type") == "points":
            return [image, *self.get_points_and_gt_masks(gt)]
        if self.config.get("prompt_type") == "both":
            bboxes, points, gt_masks, values = self.get_bboxes_points_and_gt_masks(gt)
            return [image, bboxes, gt_masks, values, points]
        return [image, *self.get_bboxes_and_gt_masks(gt)]


def custom_collate(data):
    """ref:octsam/models/training_utils.py:449-458 (pad_sequence with zeros)."""
    from torch.nn.utils.rnn import pad_sequence
    images = torch.tensor(np.array([d[0] for d in data]))
    gt_masks = pad_sequence([torch.tensor(np.array(d[2])) for d in data], batch_first=True)
    mask_values = pad_sequence([torch.tensor(d[3]) for d in data], batch_first=True)
    prompt = pad_sequence([torch.tensor(d[1]) for d in data], batch_first=True)
    if len(data[0]) == 5:  # --prompt=both: boxes, then points
        points = pad_sequence([torch.tensor(d[4]) for d in data], batch_first=True)
        return [images, prompt, gt_masks, mask_values, points]
    return [images, prompt, gt_masks, mask_values]


def make_processor():
    from transformers import SamProcessor
    from transformers.models.sam.image_processing_pil_sam import SamImageProcessorPil
    return SamProcessor(image_processor=SamImageProcessorPil())


def process_batch(processor, batch, prompt_type: str = "bboxes"):
    """training_utils.py:46-53 host part: processor call; returns a dict of CPU tensors."""
    image, prompt, gt_masks, mask_values = batch[:4]
    if prompt_type == "points":
        inputs = processor(image, input_points=prompt, return_tensors="pt")
    elif prompt_type == "both":
        inputs = processor(image, input_boxes=prompt, input_points=batch[4], return_tensors="pt")
    else:
        inputs = processor(image, input_boxes=prompt, return_tensors="pt")
    out = dict(inputs)
    out["gt_u8"] = gt_masks.round().clamp(0, 1).to(torch.uint8)
    out["mask_values"] = mask_values
    return out


def process_batch_device(processor, batch, prompt_type: str = "bboxes"):
    """process_batch with the image path on the GPU (preprocess.DeviceProcessor: Pillow-exact resize +
    normalise + pad as one HIP kernel, bit-identical to SamProcessor's pixel_values); prompts, sizes and gt
    stay host tensors like process_batch's, pixel_values is already on the processor's device."""
    image, prompt, gt_masks, mask_values = batch[:4]
    images = image.to(processor.device, non_blocking=True)
    if prompt_type == "points":
        out = processor(images, input_points=prompt)
    elif prompt_type == "both":
        out = processor(images, input_boxes=prompt, input_points=batch[4])
    else:
        out = processor(images, input_boxes=prompt)
    out["gt_u8"] = gt_masks.round().clamp(0, 1).to(torch.uint8)
    out["mask_values"] = mask_values
    return out


def pad_prompts(batch: dict, n_target: int) -> dict:
    """Pad the prompt dimension to n_target with the collate's zero padding (global-N padding across
    data-parallel ranks, so every rank sees the batch the single-process collate would build)."""
    out = dict(batch)
    for key in ("input_boxes", "input_points", "gt_u8", "mask_values"):
        if key not in out:
            continue
        t = out[key]
        n = t.shape[1]
        if n < n_target:
            pad = torch.zeros((t.shape[0], n_target - n) + tuple(t.shape[2:]), dtype=t.dtype)
            out[key] = torch.cat([t, pad], 1)
    return out


def to_device_batch(batch: dict, device) -> dict:
    out = {}
    for k, v in batch.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.to(device, non_blocking=True)
        else:
            out[k] = v
    return out
