"""Prompt and gt generation on the GPU: the label-map half of
``SAMDataset.__getitem__`` + ``custom_collate`` (ref:octsam/models/training_utils.py:381-458).

The reference, per sample: for v in np.unique(label), for each 8-connected component of (label == v) in
scipy.ndimage.label order: the bbox of its pixels jittered by four ``np.random.randint(-10, 10)`` draws
(x_min, x_max, y_min, y_max; clamped to [0, W] / [0, H]) or one ``random.randrange(0, n_pixels)`` pixel in
``np.where`` (raster) order, the float64 component indicator as gt, and v as the mask value; the collate
zero-pads to the batch's max component count.

Here the components, their rank (the reference order = sort by (value, first raster pixel)), per-component
bboxes / pixel counts and the uint8 gt [B, N, H, W] come from csrc/components.hip; only the per-image root
keys (a few dozen ints), the bbox table and the counts cross to the host, where the reference's RNG draws
are replayed in its order (seed hooks per sample as SAMDataset applies them).
"""
from __future__ import annotations

import random

import numpy as np
import torch

from . import _lib

MAX_COMPONENTS = 1024
MAX_PIXELS = 1 << 24  # root keys pack (value << 24 | pixel index)


class ComponentLimitError(ValueError):
    """A batch exceeds the device path's limits (> MAX_COMPONENTS components in a label map, or
    H*W >= MAX_PIXELS); the reference has neither limit, so train.training builds such a batch on the host
    path (SAMDataset + scipy) instead."""


class DeviceComponents:
    """Connected components + component statistics of uint8 label maps on one device."""

    def __init__(self, device, max_components: int = MAX_COMPONENTS):
        self.device = _lib.resolve_device(device)
        self.maxc = int(max_components)
        if not 1 <= self.maxc <= MAX_COMPONENTS:
            raise ValueError(f"max_components must be in [1, {MAX_COMPONENTS}]")

    def __call__(self, labels: torch.Tensor, n_target: int | None = None, want_gt: bool = True):
        """labels uint8 [B, H, W] on the device. Returns dict:
        comp int32 [B, H, W] (component rank per pixel, device), ncomp list[int], values list[np.uint8 [n]],
        stats list[np.int64 [n, 5]] (xmin, xmax, ymin, ymax, pixels), gt uint8 [B, N, H, W] (device,
        N = max(ncomp, n_target), zero-padded components) when want_gt."""
        return self.assign(self.label(labels), n_target, want_gt)

    def label(self, labels: torch.Tensor) -> dict:
        """Phase 1: components and their reference order; ``ncomp`` is known after this (the data-parallel
        loop takes the global max of it before phase 2 sizes the gt)."""
        if labels.dtype != torch.uint8 or labels.dim() != 3:
            raise ValueError(f"labels must be uint8 [B, H, W], got {labels.dtype} {tuple(labels.shape)}")
        if labels.device != self.device:
            raise ValueError(f"labels on {labels.device}, components on {self.device}")
        labels = labels.contiguous()
        B, H, W = labels.shape
        if H * W >= MAX_PIXELS:
            raise ComponentLimitError(f"label maps of {H}x{W} pixels exceed the device path's 2^24 limit")
        dev = self.device
        parent = torch.empty(B * H * W, device=dev, dtype=torch.int32)
        roots = torch.empty(B, self.maxc, device=dev, dtype=torch.int32)
        nroots = torch.empty(B, device=dev, dtype=torch.int32)
        _lib.call("octsam_cc_label", _lib.ptr(labels), B, H, W, _lib.ptr(parent), _lib.ptr(roots), self.maxc,
                  _lib.ptr(nroots))
        counts = nroots.cpu().numpy()
        if int(counts.max()) > self.maxc:
            raise ComponentLimitError(f"a label map has {int(counts.max())} components (> {self.maxc})")
        keys = roots.cpu().numpy()
        sorted_roots = np.zeros((B, self.maxc), dtype=np.int32)
        values = []
        for b in range(B):
            # keys as unsigned 32-bit: (value, first pixel) = the reference's order
            k = np.sort(keys[b, :counts[b]].astype(np.int64) & 0xFFFFFFFF)
            sorted_roots[b, :len(k)] = (k & 0xFFFFFF).astype(np.int32)
            values.append((k >> 24).astype(np.uint8))
        return {"shape": (B, H, W), "parent": parent, "sorted_roots": sorted_roots, "counts": counts,
                "values": values, "ncomp": [int(c) for c in counts]}

    def assign(self, st: dict, n_target: int | None = None, want_gt: bool = True) -> dict:
        """Phase 2: ranks, statistics and (optionally) the gt masks padded to max(ncomp, n_target)."""
        B, H, W = st["shape"]
        dev = self.device
        ncomp = st["ncomp"]
        N = max(max(ncomp), n_target or 0)
        comp = torch.empty(B, H, W, device=dev, dtype=torch.int32)
        stats = torch.empty(B, self.maxc, 5, device=dev, dtype=torch.int32)
        gt = None
        if want_gt:
            if (H * W) % 16:
                raise ValueError("gt output needs H*W % 16 == 0")
            gt = torch.empty(B, max(N, 1), H, W, device=dev, dtype=torch.uint8)
        # (named: a temporary's block would return to the allocator before the launch reads it)
        roots_d = torch.from_numpy(st["sorted_roots"]).to(dev)
        ncomp_d = torch.from_numpy(st["counts"].astype(np.int32)).to(dev)
        _lib.call("octsam_cc_assign", _lib.ptr(st["parent"]), B, H, W, _lib.ptr(roots_d), self.maxc,
                  _lib.ptr(ncomp_d), _lib.ptr(comp), _lib.ptr(stats), _lib.ptr(gt), max(N, 1))
        s = stats.cpu().numpy().astype(np.int64)
        return {"comp": comp, "ncomp": ncomp, "values": st["values"],
                "stats": [s[b, :ncomp[b]] for b in range(B)], "gt": gt[:, :N] if gt is not None else None,
                "N": N}


def bbox_prompts(stats: np.ndarray, H: int, W: int) -> list:
    """get_bboxes_and_gt_masks (training_utils.py:389-415) for one sample, components in order: the
    jittered [x_min, y_min, x_max, y_max] with the reference's draw order and clamps."""
    out = []
    for xmin, xmax, ymin, ymax, _ in stats:
        x_min = max(0, np.int64(xmin) + np.random.randint(-10, 10))
        x_max = min(W, np.int64(xmax) + np.random.randint(-10, 10))
        y_min = max(0, np.int64(ymin) + np.random.randint(-10, 10))
        y_max = min(H, np.int64(ymax) + np.random.randint(-10, 10))
        out.append([x_min, y_min, x_max, y_max])
    return out


def _kth_pixels(cc: dict, ks: list, W: int) -> list:
    """[[x, y]] of the k-th pixel (raster order, the reference's np.where order) of every component: one
    stable device sort of the pixels by (image, component rank), then a gather at the component's offset."""
    comp = cc["comp"]
    B = comp.shape[0]
    hw = comp.shape[1] * comp.shape[2]
    maxc = max(max(cc["ncomp"]), 1)
    key = (comp.view(B, hw).long() + torch.arange(B, device=comp.device).view(B, 1) * maxc).view(-1)
    order = torch.sort(key, stable=True).indices
    starts, flat = [], 0
    for b in range(B):
        cnt = cc["stats"][b][:, 4] if cc["ncomp"][b] else np.zeros(0, np.int64)
        off = flat + np.concatenate([[0], np.cumsum(cnt)[:-1]]) if len(cnt) else np.zeros(0, np.int64)
        starts.append(off + np.asarray(ks[b], dtype=np.int64))
        flat += hw
    pos = torch.from_numpy(np.concatenate(starts).astype(np.int64)).to(comp.device)
    pix = (order[pos] % hw).cpu().numpy() if len(pos) else np.zeros(0, np.int64)
    out, i = [], 0
    for b in range(B):
        n = cc["ncomp"][b]
        out.append([[[np.int64(p % W), np.int64(p // W)]] for p in pix[i:i + n]])
        i += n
    return out


def collate_device_begin(images, labels, prompt_type: str, device, seed_hooks=None) -> dict:
    """Phase 1 of collate_device: upload, components; the state's ``ncomp`` sizes the (global) batch N."""
    dev = _lib.resolve_device(device)
    labels = torch.as_tensor(labels).to(dev)
    dc = DeviceComponents(dev)
    return {"dc": dc, "cc": dc.label(labels), "images": torch.as_tensor(images), "prompt_type": prompt_type,
            "seed_hooks": seed_hooks, "device": dev}


def collate_device_end(state: dict, n_target: int | None = None, processor=None) -> dict:
    """Phase 2: ranks / statistics / gt, the reference's RNG draws per sample, image processing."""
    from .preprocess import DeviceProcessor
    dev, prompt_type, seed_hooks = state["device"], state["prompt_type"], state["seed_hooks"]
    cc = state["dc"].assign(state["cc"], n_target=n_target)
    B, H, W = state["cc"]["shape"]
    # SAMDataset.__getitem__ (training_utils.py:442-447): "points" -> points, anything else -> boxes;
    # "both" (configs[4]) adds a point after each box
    need_pts = prompt_type in ("points", "both")
    need_boxes = prompt_type != "points"
    boxes_l, points_l, ks = [], [], []
    for b in range(B):  # the reference's draws, in its order; pixels are looked up on the device below
        if seed_hooks is not None:
            seed_hooks[b]()
        st_b = cc["stats"][b]
        bx, kk = [], []
        for n in range(cc["ncomp"][b]):
            if need_boxes:
                bx += bbox_prompts(st_b[n:n + 1], H, W)
            if need_pts:
                kk.append(random.randrange(0, int(st_b[n, 4])))
        boxes_l.append(bx)
        ks.append(kk)
    if need_pts:
        points_l = _kth_pixels(cc, ks, W)
    if not need_boxes:
        boxes_l = []
    N = cc["N"]
    mask_values = torch.zeros(B, N, dtype=torch.uint8)
    kw = {}
    for key, lst, tail in (("input_boxes", boxes_l, (4,)), ("input_points", points_l, (1, 2))):
        if not lst:
            continue
        arr = np.zeros((B, N) + tail, dtype=np.int64)
        for b in range(B):
            n = cc["ncomp"][b]
            if n:
                arr[b, :n] = np.asarray(lst[b], dtype=np.int64).reshape((n,) + tail)
        kw[key] = arr
    for b in range(B):
        n = cc["ncomp"][b]
        if n:
            mask_values[b, :n] = torch.from_numpy(cc["values"][b])
    proc = processor if processor is not None else DeviceProcessor(dev)
    out = proc(state["images"].to(dev), **kw)
    prompt = kw["input_boxes"] if "input_boxes" in kw else kw["input_points"]
    out["gt_u8"] = cc["gt"]
    out["mask_values"] = mask_values
    out["prompt_raw"] = torch.from_numpy(prompt)
    return out


def collate_device(images: np.ndarray | torch.Tensor, labels: np.ndarray | torch.Tensor, prompt_type: str,
                   device, seed_hooks=None, n_target: int | None = None, processor=None) -> dict:
    """SAMDataset items + custom_collate + SamProcessor for a batch with the label and image work on the
    device. images uint8 [B, H, W, 3], labels uint8 [B, H, W]; seed_hooks: optional list of B callables
    run before each sample's draws (SAMDataset's per-item seeding). Returns the process_batch dict
    (pixel_values and gt_u8 on the device; prompts float64, mask_values uint8 on the host)."""
    st = collate_device_begin(images, labels, prompt_type, device, seed_hooks)
    return collate_device_end(st, n_target, processor)
