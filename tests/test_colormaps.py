"""--pseudocolor (dilabhelmholtzoct_amd/colormaps.py): the restated OpenCV lookup tables and where they apply
(ref:octsam/models/training_utils.py:439-440). Parity unpinned: cv2 is absent; the anchors below are OpenCV's
documented endpoint colours of its matplotlib-derived maps and the MATLAB ramp definitions."""
import numpy as np
import pytest

from dilabhelmholtzoct_amd import colormaps, data


def test_tables_shape_and_known_endpoints():
    for name in colormaps.available():
        lut = colormaps.colormap_lut(name)
        assert lut.shape == (256, 3) and lut.dtype == np.uint8
    v = colormaps.colormap_lut("Viridis")
    assert tuple(v[0][::-1]) == (68, 1, 84) and tuple(v[255][::-1]) == (253, 231, 37)  # RGB of viridis ends
    a = colormaps.colormap_lut("Autumn")  # BGR: (0, i, 255)
    assert np.array_equal(a[:, 1], np.arange(256)) and (a[:, 0] == 0).all() and (a[:, 2] == 255).all()
    c = colormaps.colormap_lut("Cool")    # BGR: (255, 255 - i, i)
    assert np.array_equal(c[:, 2], np.arange(256)) and np.array_equal(c[:, 1], 255 - np.arange(256))


def test_names_follow_the_reference_table():
    assert colormaps.colormap_lut("grayscale") is None and colormaps.colormap_lut(None) is None
    with pytest.raises(KeyError):
        colormaps.colormap_lut("NotAMap")
    with pytest.raises(NotImplementedError):
        colormaps.colormap_lut("Jet")
    assert set(colormaps.available()) <= set(colormaps.OCV_NAMES)


def test_npy_table(tmp_path):
    lut = np.random.RandomState(0).randint(0, 256, (256, 3)).astype(np.uint8)
    p = tmp_path / "map.npy"
    np.save(p, lut)
    assert np.array_equal(colormaps.colormap_lut(str(p)), lut)
    np.save(p, lut[:, :2].copy())
    with pytest.raises(ValueError):
        colormaps.colormap_lut(str(p))


def test_apply_uses_channel_zero():
    lut = colormaps.colormap_lut("Turbo")
    rng = np.random.RandomState(1)
    img = rng.randint(0, 256, (5, 7, 3)).astype(np.uint8)
    out = colormaps.apply_colormap(img, lut)
    assert out.shape == (5, 7, 3) and out.dtype == np.uint8
    assert np.array_equal(out, lut[img[:, :, 0]])
    assert np.array_equal(colormaps.apply_colormap(img[:, :, 0], lut), out)


def test_dataset_item_is_colourised_prompts_unchanged():
    items = data.synthetic_oct(seed=3, n=2)
    gray = data.SAMDataset(items, {"prompt_type": "bboxes"}, epoch_seed=0)
    col = data.SAMDataset(items, {"prompt_type": "bboxes", "pseudocolor": "Magma"}, epoch_seed=0)
    lut = colormaps.colormap_lut("Magma")
    for i in range(2):
        g, c = gray[i], col[i]
        assert np.array_equal(c[0], lut[items[i]["image"][:, :, 0]])
        assert np.array_equal(np.array(c[1]), np.array(g[1]))
        assert np.array_equal(np.array(c[2]), np.array(g[2]))
