"""CPU pins of the GPU processor's host half (dilabhelmholtzoct_amd/preprocess.py) and of the numpy
restatement the GPU test checks against (oracle/processor_ref.py): resample tables vs Pillow's own
resize (bit-exact bytes, upscale / identity / downscale / odd sizes), the byte lookup vs transformers'
rescale + normalize, the whole image path vs SamProcessor's pixel_values, and prompt coordinates vs the
processor's input_boxes / input_points."""
import numpy as np
import pytest
import torch
from PIL import Image

from dilabhelmholtzoct_amd import preprocess as pp
from oracle.processor_ref import pil_resample_ref, sam_preprocess_ref


def _img(h, w, seed):
    rng = np.random.RandomState(seed)
    a = rng.randint(0, 256, (h, w, 3)).astype(np.uint8)
    a[: h // 3] = (np.arange(w)[None, :, None] * 7 % 256).astype(np.uint8)  # smooth ramps + hard edges
    return a


@pytest.mark.parametrize("hw,out", [((496, 512), (992, 1024)), ((64, 48), (64, 48)), ((37, 53), (101, 97)),
                                    ((300, 700), (439, 1024)), ((180, 260), (61, 83))])
def test_resample_tables_match_pillow(hw, out):
    img = _img(*hw, seed=hw[0])
    xt, kx = pp.resample_table(hw[1], out[1])
    yt, ky = pp.resample_table(hw[0], out[0])
    got = pil_resample_ref(img, xt, yt)
    want = np.asarray(Image.fromarray(img).resize((out[1], out[0]), resample=Image.BILINEAR))
    assert got.shape == want.shape
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    assert kx <= pp.MAX_TAPS and ky <= pp.MAX_TAPS


def test_lut_matches_transformers_rescale_normalize():
    from transformers.image_transforms import normalize, rescale
    from transformers.image_utils import ChannelDimension
    v = np.tile(np.arange(256, dtype=np.uint8)[None, None, :], (3, 1, 1))  # CHW, every byte per channel
    x = rescale(v, 1 / 255, input_data_format=ChannelDimension.FIRST)
    x = normalize(x, pp.IMAGENET_MEAN, pp.IMAGENET_STD, input_data_format=ChannelDimension.FIRST)
    lut = pp.normalize_lut()
    assert x.dtype == np.float32
    assert np.array_equal(lut, x[:, 0, :])


@pytest.mark.parametrize("hw", [(496, 512), (300, 700)])
def test_image_path_matches_sam_processor(hw):
    from dilabhelmholtzoct_amd import data
    proc = data.make_processor()
    img = _img(*hw, seed=7)
    want = proc(torch.from_numpy(img[None]), return_tensors="pt")
    rh, rw = pp.preprocess_shape(*hw)
    xt, _ = pp.resample_table(hw[1], rw)
    yt, _ = pp.resample_table(hw[0], rh)
    got = sam_preprocess_ref(img, xt, yt, pp.normalize_lut())
    assert tuple(want["reshaped_input_sizes"][0].tolist()) == (rh, rw)
    assert np.array_equal(got, want["pixel_values"][0].numpy())


def test_prompt_coordinates_match_sam_processor():
    from dilabhelmholtzoct_amd import data
    proc = data.make_processor()
    img = torch.from_numpy(_img(496, 512, 3)[None].repeat(2, 0))
    rng = np.random.RandomState(0)
    boxes = torch.from_numpy(rng.randint(0, 512, (2, 5, 4)))
    pts = torch.from_numpy(rng.randint(0, 496, (2, 5, 1, 2)))
    want_b = proc(img, input_boxes=boxes, return_tensors="pt")["input_boxes"]
    want_p = proc(img, input_points=pts, return_tensors="pt")["input_points"]
    got_b = pp.normalize_coordinates(boxes.numpy(), (496, 512), is_bounding_box=True)
    got_p = pp.normalize_coordinates(pts.numpy(), (496, 512))
    assert want_b.dtype == torch.float64 and want_p.dtype == torch.float64
    assert np.array_equal(got_b, want_b.numpy())
    assert np.array_equal(got_p, want_p.numpy())
