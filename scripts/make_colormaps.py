#!/usr/bin/env python3
"""Writes dilabhelmholtzoct_amd/colormaps.npz: the 256-entry u8 lookup tables of the --pseudocolor maps this
package can restate without cv2 (the reference's OCV_COLORMAPS, ref:octsam/models/training.py:58-82, applied by
cv2.applyColorMap at ref:octsam/models/training_utils.py:439-440). Tables are [256, 3] in OpenCV's BGR order.

How OpenCV (absent here) builds them (modules/imgproc/src/colormap.cpp, restated): a map holds float r, g, b samples
on linspace(0, 1, n_samples); linear_colormap interpolates them at linspace(0, 1, 256), stacks (b, g, r) and converts
to u8 with scale 255 (round to nearest).
  * Viridis, Magma, Inferno, Plasma, Cividis, Turbo: 256 samples, OpenCV's tables are matplotlib's listed colormap
    data (matplotlib 3.10.8 here, matplotlib._cm_listed) -> u8 = rint(255 * float32(sample)).
  * Autumn (r 1, g t, b 0), Spring (1, t, 1 - t), Cool (t, 1 - t, 1): linear ramps, so interpolation leaves them
    at t = i / 255 and every u8 value is an integer (no rounding tie).
Not restated (they raise): maps whose OpenCV samples are not linear ramps or whose u8 values fall on rounding ties
(Bone, Deepgreen, Hot, HSV, Jet, Ocean, Parula, Pink, Rainbow, Winter, Summer, Twilight, Twilight shifted).
Parity unpinned: cv2 is not in this image and the reference holds no colourised fixture."""
import os

import numpy as np


def tables():
    from matplotlib import _cm_listed as L
    out = {}
    for name, key in (("Viridis", "_viridis_data"), ("Magma", "_magma_data"), ("Inferno", "_inferno_data"),
                      ("Plasma", "_plasma_data"), ("Cividis", "_cividis_data"), ("Turbo", "_turbo_data")):
        rgb = np.asarray(getattr(L, key), dtype=np.float32)
        assert rgb.shape == (256, 3)
        u8 = np.rint(rgb.astype(np.float64) * 255.0).clip(0, 255).astype(np.uint8)
        out[name] = u8[:, ::-1].copy()  # BGR
    i = np.arange(256, dtype=np.int64)
    full, zero = np.full(256, 255), np.zeros(256, dtype=np.int64)
    for name, (r, g, b) in (("Autumn", (full, i, zero)), ("Spring", (full, i, 255 - i)), ("Cool", (i, 255 - i, full))):
        out[name] = np.stack([b, g, r], 1).astype(np.uint8)
    return out


if __name__ == "__main__":
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dilabhelmholtzoct_amd",
                       "colormaps.npz")
    np.savez(dst, **tables())
    print("wrote", dst)
