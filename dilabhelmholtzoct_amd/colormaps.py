"""--pseudocolor: the reference colours channel 0 of every scan through an OpenCV colormap before the processor
(ref:octsam/models/training_utils.py:439-440, `cv2.applyColorMap(image[:, :, 0], OCV_COLORMAPS[name])`, names at
ref:octsam/models/training.py:58-82). cv2 is not in this image: the maps are 256-entry u8 lookup tables in OpenCV's
BGR order (colormaps.npz, written by scripts/make_colormaps.py, which says how each table restates OpenCV's), applied
as one gather per pixel on the host where the reference applies them (the dataset item). A table exported from cv2
elsewhere can be given as a path to a [256, 3] u8 .npy file. Parity unpinned (no cv2, no reference fixture)."""
import os

import numpy as np

# the reference's OCV_COLORMAPS keys (ref:octsam/models/training.py:58-82)
OCV_NAMES = ("Autumn", "Bone", "Cividis", "Cool", "Deepgreen", "Hot", "HSV", "Inferno", "Jet", "Magma", "Ocean",
             "Parula", "Pink", "Plasma", "Rainbow", "Viridis", "Winter", "Spring", "Summer", "Twilight shifted",
             "Twilight", "Turbo", "grayscale")
_TABLES = None


def _tables():
    global _TABLES
    if _TABLES is None:
        with np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "colormaps.npz")) as z:
            _TABLES = {k: z[k] for k in z.files}
    return _TABLES


def available():
    """Names this package restates (the rest of OCV_NAMES raise in colormap_lut)."""
    return tuple(sorted(_tables()))


def colormap_lut(name):
    """name -> [256, 3] u8 BGR table, or None for "grayscale" / None (no colouring, the reference's None entry).
    A KeyError for names outside the reference's set (as OCV_COLORMAPS[name]); NotImplementedError for reference
    names not restated here; a path ending in .npy loads a [256, 3] u8 table."""
    if name is None or name == "grayscale":
        return None
    if isinstance(name, np.ndarray):
        lut = name
    elif str(name).endswith(".npy"):
        lut = np.load(name)  # allow_pickle stays False
    else:
        if name not in OCV_NAMES:
            raise KeyError(name)
        t = _tables()
        if name not in t:
            raise NotImplementedError(f"pseudocolor map {name!r} needs cv2's table (not in this image); restated: "
                                      f"{', '.join(available())}, or pass a [256, 3] u8 .npy table")
        lut = t[name]
    if lut.shape != (256, 3) or lut.dtype != np.uint8:
        raise ValueError(f"a colormap table is [256, 3] uint8, got {lut.shape} {lut.dtype}")
    return lut


def apply_colormap(image, lut):
    """cv2.applyColorMap(image[:, :, 0], map) for a u8 [H, W, C] scan ([H, W] grayscale scans: the scan itself, which
    is channel 0 after the processor's RGB conversion) -> u8 [H, W, 3] (BGR, as OpenCV returns it)."""
    image = np.asarray(image)
    if image.dtype != np.uint8:
        raise TypeError(f"applyColorMap takes u8 scans, got {image.dtype}")
    ch0 = image if image.ndim == 2 else image[:, :, 0]
    return lut[ch0]
