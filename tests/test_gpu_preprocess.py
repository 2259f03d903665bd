"""GPU processor (csrc/preprocess.hip via dilabhelmholtzoct_amd.preprocess.DeviceProcessor) vs the reference
path, transformers' SamProcessor with the PIL backend (hf:image_processing_pil_sam.py:227-263): pixel_values
must be bit-identical (integer resize + byte lookup), on synthetic OCT scans, random images, odd sizes
(unaligned rows), a downscale and B = 1; plus host-side argument errors and a bandwidth readout."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _random(B, h, w, seed):
    rng = np.random.RandomState(seed)
    return rng.randint(0, 256, (B, h, w, 3)).astype(np.uint8)


def _check(cuda, imgs):
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.preprocess import DeviceProcessor
    want = data.make_processor()(torch.from_numpy(imgs), return_tensors="pt")
    dp = DeviceProcessor(cuda)
    got = dp.images(torch.from_numpy(imgs).to(cuda))
    torch.cuda.synchronize()
    got = got.cpu()
    assert got.shape == want["pixel_values"].shape
    diff = (got != want["pixel_values"]).sum().item()
    assert diff == 0, f"{diff} of {got.numel()} values differ"


def test_preprocess_synthetic_oct(cuda):
    from dilabhelmholtzoct_amd import data
    ds = data.synthetic_oct(seed=5, n=4)
    imgs = np.stack([np.array(ds[i]["image"]) for i in range(4)])
    assert imgs.shape == (4, 496, 512, 3) and imgs.dtype == np.uint8
    _check(cuda, imgs)


@pytest.mark.parametrize("B,h,w", [(2, 496, 512), (1, 37, 53), (2, 300, 701), (1, 1500, 2000), (1, 1024, 1024)])
def test_preprocess_random(cuda, B, h, w):
    _check(cuda, _random(B, h, w, seed=h + w))


def test_preprocess_processor_dict(cuda):
    """DeviceProcessor(images, input_boxes=...) reproduces every SamProcessor output of the training step."""
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.preprocess import DeviceProcessor
    ds = data.synthetic_oct(seed=9, n=2)
    sd = data.SAMDataset(ds, {"prompt_type": "bboxes"}, epoch_seed=0)
    batch = data.custom_collate([sd[i] for i in range(len(sd))])
    want = data.process_batch(data.make_processor(), batch, "bboxes")
    got = DeviceProcessor(cuda)(batch[0].to(cuda), input_boxes=batch[1])
    assert torch.equal(got["pixel_values"].cpu(), want["pixel_values"])
    for k in ("original_sizes", "reshaped_input_sizes", "input_boxes"):
        assert torch.equal(got[k], want[k]), k


def test_preprocess_rejects_bad_inputs(cuda):
    from dilabhelmholtzoct_amd._lib import OctsamError
    from dilabhelmholtzoct_amd.preprocess import DeviceProcessor
    dp = DeviceProcessor(cuda)
    with pytest.raises(ValueError):
        dp.images(torch.zeros(1, 8, 8, 3, device=cuda, dtype=torch.float32))
    with pytest.raises(ValueError):  # 9000 -> 1024 needs 19 taps per output pixel (> 16)
        dp.images(torch.zeros(1, 16, 9000, 3, device=cuda, dtype=torch.uint8))
    from dilabhelmholtzoct_amd import _lib
    img = torch.zeros(1, 16, 16, 3, device=cuda, dtype=torch.uint8)
    tab = torch.zeros(64, 2 + 17, device=cuda, dtype=torch.int32)
    out = torch.empty(1, 3, 64, 64, device=cuda)
    with pytest.raises(OctsamError):  # the C ABI refuses 17 taps before any launch
        _lib.call("octsam_sam_preprocess", _lib.ptr(img), 1, 16, 16, 16 * 16 * 3, _lib.ptr(tab), 17,
                  _lib.ptr(tab), 17, 64, 64, _lib.ptr(dp.lut), _lib.ptr(out), 64, 64)


def test_preprocess_bandwidth(cuda):
    """B = 8 OCT scans (bench batch): fp32 writes + uint8 reads per launch over HIP-event time."""
    from dilabhelmholtzoct_amd.preprocess import DeviceProcessor
    dp = DeviceProcessor(cuda)
    imgs = torch.from_numpy(_random(8, 496, 512, 1)).to(cuda)
    out = torch.empty(8, 3, 1024, 1024, device=cuda)
    for _ in range(3):
        dp.images(imgs, out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        dp.images(imgs, out)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / 20
    byts = out.numel() * 4 + imgs.numel()
    print(f"sam_preprocess B=8 496x512 -> 1024^2: {us:.1f} us/launch, {byts / us / 1e3:.0f} GB/s "
          f"({byts / 1e6:.1f} MB algorithmic)")
    assert us > 0
