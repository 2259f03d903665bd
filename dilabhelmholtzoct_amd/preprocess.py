"""SamProcessor on the GPU: the image path of ``SamProcessor.__call__``
(hf:processing_sam.py:88-131 -> hf:image_processing_pil_sam.py:227-263) as one HIP kernel, and the prompt
coordinate normalisation (hf:processing_sam.py:215-234) on the host.

The reference resizes with Pillow (``Image.resize(..., BILINEAR)``: 8-bit fixed-point two-pass
ImagingResample), rescales by 1/255 in float64 then casts to float32 (image_transforms.rescale), normalises
``(x - mean) / std`` in float32 (image_transforms.normalize) and zero-pads to 1024². Here:

* ``resample_table`` restates Pillow's ``precompute_coeffs`` + ``normalize_coeffs_8bpc`` in double precision
  on the host (per (source, target) size, cached): per output index the first source index, the tap count
  and int32 weights with 22 fractional bits;
* ``normalize_lut`` evaluates rescale + normalise for the 256 possible byte values of each channel in the
  processor's own float arithmetic (numpy float64 -> float32, float32 subtract/divide);
* ``octsam_sam_preprocess`` (csrc/preprocess.hip) runs both integer passes per output pixel, looks the byte
  up in the table and writes planar fp32 with the padding — the same bytes as the reference path
  (tests/test_preprocess_cpu.py pins the tables against Pillow, tests/test_gpu_preprocess.py the kernel
  against transformers' SamProcessor).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib

PRECISION_BITS = 32 - 8 - 2  # Pillow's 8-bpc fixed point
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
LONGEST_EDGE = 1024
MAX_TAPS = 16


def preprocess_shape(old_h: int, old_w: int, longest_edge: int = LONGEST_EDGE):
    """SamImageProcessor._get_preprocess_shape (hf:image_processing_pil_sam.py:135-144)."""
    scale = longest_edge * 1.0 / max(old_h, old_w)
    return int(old_h * scale + 0.5), int(old_w * scale + 0.5)


def _bilinear(x: float) -> float:
    x = -x if x < 0.0 else x
    return 1.0 - x if x < 1.0 else 0.0


def resample_table(in_size: int, out_size: int):
    """Pillow ImagingResample coefficients for one axis (BILINEAR, support 1, box [0, in_size)):
    int32 [out_size, 2 + k] rows (xmin, count, w_0 .. w_{k-1}) and k."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    k = int(math.ceil(support)) * 2 + 1
    if k > MAX_TAPS:
        raise ValueError(f"resample_table: {in_size} -> {out_size} needs {k} taps (> {MAX_TAPS})")
    tab = np.zeros((out_size, 2 + k), dtype=np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bilinear((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        fixed = [int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
                 for v in w]
        tab[xx, 0], tab[xx, 1] = xmin, xmax
        tab[xx, 2:2 + xmax] = fixed
    return tab.astype(np.int32), k


def normalize_lut(mean=IMAGENET_MEAN, std=IMAGENET_STD, rescale: float = 1 / 255):
    """float32 [3, 256]: byte v of channel c -> ((float32(float64(v) * rescale)) - mean_c) / std_c in float32
    (image_transforms.rescale then normalize)."""
    v = np.arange(256, dtype=np.uint8).astype(np.float64) * rescale
    v = v.astype(np.float32)
    m = np.array(mean, dtype=np.float32)
    s = np.array(std, dtype=np.float32)
    return ((v[None, :] - m[:, None]) / s[:, None]).astype(np.float32)


def normalize_coordinates(coords: np.ndarray, original_size, longest_edge: int = LONGEST_EDGE,
                          is_bounding_box: bool = False) -> np.ndarray:
    """SamProcessor._normalize_coordinates (hf:processing_sam.py:215-234): float64, x by new_w/old_w and y
    by new_h/old_h."""
    old_h, old_w = original_size
    new_h, new_w = preprocess_shape(old_h, old_w, longest_edge)
    c = np.array(coords, dtype=np.float64, copy=True)
    shape = c.shape
    if is_bounding_box:
        c = c.reshape(-1, 2, 2)
    c[..., 0] = c[..., 0] * (new_w / old_w)
    c[..., 1] = c[..., 1] * (new_h / old_h)
    return c.reshape(shape)


class DeviceProcessor:
    """Image side of SamProcessor on one device; tables cached per source size."""

    def __init__(self, device, mean=IMAGENET_MEAN, std=IMAGENET_STD, rescale: float = 1 / 255,
                 longest_edge: int = LONGEST_EDGE):
        self.device = _lib.resolve_device(device)
        self.longest_edge = longest_edge
        self.lut = torch.from_numpy(normalize_lut(mean, std, rescale)).to(self.device)
        self._tables = {}

    def tables(self, H: int, W: int):
        key = (H, W)
        if key not in self._tables:
            rh, rw = preprocess_shape(H, W, self.longest_edge)
            xt, kx = resample_table(W, rw)
            yt, ky = resample_table(H, rh)
            self._tables[key] = (torch.from_numpy(xt).to(self.device), kx, torch.from_numpy(yt).to(self.device),
                                 ky, rh, rw)
        return self._tables[key]

    def images(self, images: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """uint8 [B, H, W, 3] on the device -> pixel_values fp32 [B, 3, L, L] (L = longest_edge)."""
        if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3:
            raise ValueError(f"images must be uint8 [B, H, W, 3], got {images.dtype} {tuple(images.shape)}")
        if images.device != self.device:
            raise ValueError(f"images on {images.device}, processor on {self.device}")
        images = images.contiguous()
        B, H, W, _ = images.shape
        xt, kx, yt, ky, rh, rw = self.tables(H, W)
        L = self.longest_edge
        if out is None:
            out = torch.empty(B, 3, L, L, device=self.device, dtype=torch.float32)
        _lib.call("octsam_sam_preprocess", _lib.ptr(images), B, H, W, H * W * 3, _lib.ptr(xt), kx, _lib.ptr(yt),
                  ky, rh, rw, _lib.ptr(self.lut), _lib.ptr(out), L, L)
        return out

    def __call__(self, images: torch.Tensor, input_boxes=None, input_points=None) -> dict:
        """The SamProcessor(images, input_boxes=... | input_points=..., return_tensors="pt") dict, with
        pixel_values computed on the device (prompts stay host float64 like the processor's)."""
        B, H, W, _ = images.shape
        rh, rw = preprocess_shape(H, W, self.longest_edge)
        out = {"pixel_values": self.images(images),
               "original_sizes": torch.tensor([[H, W]] * B, dtype=torch.int64),
               "reshaped_input_sizes": torch.tensor([[rh, rw]] * B, dtype=torch.int64)}
        if input_boxes is not None:
            b = np.asarray(input_boxes.cpu() if isinstance(input_boxes, torch.Tensor) else input_boxes)
            out["input_boxes"] = torch.from_numpy(normalize_coordinates(b, (H, W), self.longest_edge, True))
        if input_points is not None:
            p = np.asarray(input_points.cpu() if isinstance(input_points, torch.Tensor) else input_points)
            out["input_points"] = torch.from_numpy(normalize_coordinates(p, (H, W), self.longest_edge))
        return out
