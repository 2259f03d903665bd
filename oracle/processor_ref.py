"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

numpy restatement of the SamProcessor image path used to check the HIP kernel
(dilabhelmholtzoct_amd/csrc/preprocess.hip): Pillow's 8-bpc two-pass ImagingResample evaluated from
per-axis coefficient tables (horizontal pass first, uint8 clamp after each pass — Pillow's
ImagingResampleHorizontal_8bpc / ImagingResampleVertical_8bpc), then the per-channel byte lookup
(rescale + normalise) and zero padding (hf:image_processing_pil_sam.py:227-263). Pinned against Pillow
and transformers' SamProcessor themselves in tests/test_preprocess_cpu.py.
"""
from __future__ import annotations

import numpy as np

PB = 22


def _clip8(v: np.ndarray) -> np.ndarray:
    return np.clip(v >> PB, 0, 255)


def _pass(src: np.ndarray, tab: np.ndarray, axis: int) -> np.ndarray:
    """One resample pass along `axis` of an int64 array; tab rows (min, count, weights...)."""
    src = np.moveaxis(src, axis, 0)
    out = np.empty((tab.shape[0],) + src.shape[1:], dtype=np.int64)
    for o, row in enumerate(tab):
        lo, cnt = int(row[0]), int(row[1])
        acc = np.full(src.shape[1:], 1 << (PB - 1), dtype=np.int64)
        for i in range(cnt):
            acc += src[lo + i] * int(row[2 + i])
        out[o] = _clip8(acc)
    return np.moveaxis(out, 0, axis)


def pil_resample_ref(img_hwc: np.ndarray, xtab: np.ndarray, ytab: np.ndarray) -> np.ndarray:
    """uint8 [H, W, C] -> uint8 [len(ytab), len(xtab), C]."""
    t = _pass(img_hwc.astype(np.int64), xtab, 1)
    return _pass(t, ytab, 0).astype(np.uint8)


def sam_preprocess_ref(img_hwc: np.ndarray, xtab, ytab, lut: np.ndarray, out_size: int = 1024) -> np.ndarray:
    """uint8 [H, W, 3] -> fp32 [3, out_size, out_size]."""
    r = pil_resample_ref(img_hwc, xtab, ytab)
    rh, rw = r.shape[:2]
    out = np.zeros((3, out_size, out_size), dtype=np.float32)
    for c in range(3):
        out[c, :rh, :rw] = lut[c][r[..., c]]
    return out
